// vcfc_decode.hip -- gfx950 kernels for the .vcfc decoder.
//
// Replaces decompress2_data_line (reference src/compress.cpp:741-986) for a
// batch of records resident in HBM.  The reference parses the data section
// byte by byte and never reads a record's LEN header; here the host finds
// record starts by hopping LEN headers, and every record's parse is checked
// to end exactly where the next hop lands.  Where it does not (a record with
// fewer or more samples than the header declares), the rest of the input is
// decoded by k_dec_stream, one lane walking the bytes exactly as the
// reference does.
//
//   k_dec_plan   one wave per record: is the record "simple"?  Then its line
//                is REQ' + 4 * S bytes.  Others are queued for k_dec_seq.
//   k_dec_seq    one lane per queued record: byte-serial parse (size, end,
//                reference error).
//   scan         line offsets (the encoder's exclusive scan).
//   k_dec_write  one wave per record: simple records fill LDS tiles of
//                4-byte token words item by item, then stream each tile out
//                with contiguous 16-byte stores; queued records by the
//                byte-serial writer on lane 0.
//   k_dec_stream one lane: byte-serial decode of a byte range.
//
// A record is simple when: header bits and REQ are sane; REQ holds exactly 9
// TABs; S > 0; the sample section is a sequence of items -- run bytes with a
// non-zero count (0|0: b < 0x80, count b; 0|1 1|0 1|1: 0x80..0xDF, count
// b & 0x1F) and escapes 0xE1 + 3 ASCII bytes (no TAB/LF) + TAB (or the final
// LF) -- whose token counts add up to exactly S; the record's last byte is LF.
// Then every sample token is 3 bytes and the line is REQ' (the C string of
// the REQ bytes: `linebuf.append(buf)` stops at a NUL, compress.cpp:798),
// then S four-byte words "a|b\t" with the last TAB replaced by LF.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

namespace {

constexpr int DEC_WAVES = 4;   // records per 256-thread block
constexpr uint32_t SB = 2048;              // sample bytes staged per piece (k_dec_write)
constexpr uint32_t SBUF = SB + 48;         // + look-ahead, 16-B alignment slack, last block's overhang
constexpr uint32_t TB = 256;   // token words per LDS tile (k_dec_write): 4 per lane (512: +13 %, profiles/r03/ab/ab_dec_tile512.txt)

// per-record status after planning
constexpr uint32_t DS_SIMPLE = 0;   // line = REQ' + 4S bytes, item fill
constexpr uint32_t DS_SEQ = 1;      // byte-serial path, consistent end
constexpr uint32_t DS_INCONS = 2;   // byte-serial parse ends off the LEN hop
constexpr uint32_t DS_ERR = 3;      // the reference throws at this record
constexpr uint32_t DS_SKIP = 5;     // not selected: no line

// result of dec_line_seq
constexpr int DL_OK = 0, DL_END = 1, DL_ERR = 2;

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// bit i set <=> byte i of w is zero (exact)
// (the four flags gathered by one v_dot4_u32_u8, round 5: 6 VALU fewer than
// four shifts, masks and ors)
__device__ __forceinline__ uint32_t zero_bytes4(uint32_t w) {
    const uint32_t t = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
    return vw::dot4u(t >> 7, 0x08040201u, 0u);
}

__device__ __forceinline__ uint32_t be30(const uint8_t *h) {
    return ((uint32_t)(h[0] & 0x3Fu) << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
}

// One data line, byte-serial, exactly as decompress2_data_line
// (compress.cpp:741-986): from the 8 header bytes at in[p] through the
// closing LF.  Writes the line to `out` when non-null.  DL_END: fewer than 8
// bytes left (read_compressed_line_length_headers returns short, :768-774).
__device__ int dec_line_seq(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint8_t *out,
                            uint64_t *size, uint64_t *end) {
    if (n - p < 8) return DL_END;
    const uint8_t *h = in + p;
    if ((h[0] >> 6) != 3u || (h[4] >> 6) != 3u) return DL_ERR;     // utils.hpp:198-206
    const uint32_t req = be30(h + 4);
    uint64_t ip = p + 8, o = 0;
    if (req == 0 || n - ip < req) return DL_ERR;                   // :790-797
    uint64_t tabs = 0;
    bool nul = false;
    for (uint32_t i = 0; i < req; i++) {
        const uint8_t b = in[ip + i];
        tabs += b == '\t';
        nul = nul || b == 0;
        if (!nul) {
            if (out) out[o] = b;
            o++;
        }
    }
    ip += req;
    if (tabs != 9 && !(tabs == 8 && S == 0)) return DL_ERR;        // :818-828
    uint64_t got = 0;
    while (got < S) {                                               // :832-954
        if (ip >= n) return DL_ERR;
        const uint8_t b = in[ip++];
        if ((b & 0x80u) == 0) {
            const uint32_t cnt = b & 0x7Fu;
            for (uint32_t k = 0; k < cnt; k++) {
                if (out) { out[o] = '0'; out[o + 1] = '|'; out[o + 2] = '0'; out[o + 3] = '\t'; }
                o += 4;
            }
            got += cnt;
            if (got >= S && o > 0) o--;                             // pop the last tab
        } else if ((b & 0xE0u) == 0xE0u) {
            const uint32_t uc = b & 0x1Fu;
            uint32_t u = 0;
            while (u < uc) {
                if (ip >= n) return DL_ERR;
                const uint8_t x = in[ip++];
                if (x == '\n') {
                    u++; got++;
                    if (u != uc) return DL_ERR;
                    ip--;                                           // re-read as the line end
                } else if (x == '\t') {
                    u++; got++;
                    if (got < S) { if (out) out[o] = '\t'; o++; }
                } else {
                    if (out) out[o] = x;
                    o++;
                }
            }
        } else {
            const uint32_t m = b & 0xE0u;
            const uint8_t a = m == 0xA0u ? '0' : '1';               // 0|1 -> 0xA0, 1|0 -> 0xC0, 1|1 -> 0x80
            const uint8_t c = m == 0xC0u ? '0' : '1';
            uint32_t cnt = b & 0x1Fu;
            while (cnt--) {
                if (out) { out[o] = a; out[o + 1] = '|'; out[o + 2] = c; }
                o += 3;
                got++;
                if (got < S) { if (out) out[o] = '\t'; o++; }
            }
        }
    }
    if (ip >= n) return DL_ERR;                                     // :958-966
    if (in[ip++] != '\n') return DL_ERR;
    if (out) out[o] = '\n';
    o++;
    *size = o;
    *end = ip;
    return DL_OK;
}

// Record-relative positions below are 32-bit: a record is staged from the
// 16-byte block holding its first byte (rbase), and no record reaches 4 GiB.

// Wave-parallel scan of a record's sample items (see the header comment),
// one window of 256 bytes per call: lane l holds the dword of bytes
// [b0 + 4l, b0 + 4l + 4) (b0 4-aligned); bytes outside [s0, b) are not part
// of the sample section (s0 may lie inside the first dword; byte s1 is the
// record's LF).  Escape flag bytes (0xE1) mark the next 3 bytes as payload
// and the 4th as its terminator; those may spill into the next lane (DPP)
// or the next window (carry).  State carries across windows.
struct ItemState {
    uint32_t got = 0;
    uint32_t ecarry = 0;   // escape flags of the previous window's lane 63
    bool bad = false;
};
struct ItemLane {
    uint32_t start;    // bit j: byte j of the lane's dword starts an item
    uint32_t e1;       // bit j: byte j is an escape flag (0xE1)
    uint32_t gb[4];    // tokens before each byte's item
};

// bit j <- bit 8j + 7 of x (one flag per byte, as 0x80 in that byte)
__device__ __forceinline__ uint32_t msb4(uint32_t x) {
    return vw::dot4u((x >> 7) & 0x01010101u, 0x08040201u, 0u);
}
// bits [lo, hi) of a 4-bit mask (0 <= lo, hi <= 4)
__device__ __forceinline__ uint32_t bits4(uint32_t lo, uint32_t hi) {
    return ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}

// All four bytes of the lane at once (4-bit masks, one bit per byte): which
// bytes are in [s0, b), escape flags (0xE1), payload and terminator bytes,
// item starts and their token counts (a byte < 0x80 counts itself, a byte
// >= 0x80 its low 5 bits: 1 for 0xE1), and the checks of a simple record --
// payload bytes are < 0x80 and neither TAB nor LF, terminators are TAB, a
// start is not an escape code other than 0xE1, an escape's 3 bytes and
// terminator end before s1, and no item counts 0 tokens.
__device__ __forceinline__ ItemLane scan_window(uint32_t v4, uint32_t b0, uint32_t s0, uint32_t b, uint32_t s1,
                                                ItemState &st) {
    const uint32_t l = vw::lane_id();
    const uint32_t k0 = b0 + 4 * l;
    const uint32_t valid = bits4(s0 > k0 ? umin32(s0 - k0, 4u) : 0u, b > k0 ? umin32(b - k0, 4u) : 0u);
    const uint32_t tabM = zero_bytes4(v4 ^ 0x09090909u), lfM = zero_bytes4(v4 ^ 0x0A0A0A0Au);
    const uint32_t e1M = zero_bytes4(v4 ^ 0xE1E1E1E1u), escM = zero_bytes4((v4 & 0xE0E0E0E0u) ^ 0xE0E0E0E0u);
    const uint32_t hb = v4 & 0x80808080u;
    const uint32_t hi8 = (hb << 1) - (hb >> 7);                   // 0xFF in the bytes >= 0x80
    const uint32_t c8 = v4 & (~hi8 | 0x1F1F1F1Fu);                // each byte's token count
    const uint32_t e = valid & e1M;
    const uint32_t ep = vw::shr1(e, st.ecarry);     // escape flags of the previous lane
    st.ecarry = vw::readlane(e, 63);
    const uint32_t c = (e << 4) | ep;               // previous lane's bytes below this lane's
    const uint32_t P = ((c << 1) | (c << 2) | (c << 3)) >> 4 & 0xFu;   // payload bytes
    const uint32_t T = ep;                          // terminator bytes (4 after a flag)
    ItemLane r;
    r.start = valid & ~P & ~T;
    r.e1 = e1M;
    const int32_t lim = (int32_t)(s1 - k0) - 4;     // an escape at byte j needs j <= lim
    const uint32_t overM = lim >= 3 ? 0u : lim < 0 ? 0xFu : (0xFu << (lim + 1)) & 0xFu;
    const uint32_t bad = (P & ~T & (msb4(hb) | tabM | lfM)) | (T & ~tabM) |
                         (r.start & ((escM & ~e1M) | (e1M & overM) | zero_bytes4(c8)));
    st.bad = st.bad || vw::ballot((bad & valid) != 0) != 0;
    // start bits -> 0xFF bytes (bit j -> bit 8j by one 24-bit multiply), the
    // starts' counts, their sum and prefix sums by v_dot4_u32_u8
    const uint32_t s8 = vw::umul24(r.start, 0x00204081u) & 0x01010101u;
    const uint32_t cs = c8 & ((s8 << 8) - s8);      // counts of the starts
    const uint32_t sum = vw::dot4u(cs, 0x01010101u, 0u);
    const uint32_t inc = vw::scan_add(sum);
    const uint32_t base = st.got + (inc - sum);
    r.gb[0] = base;
    r.gb[1] = vw::dot4u(cs, 0x00000001u, base);
    r.gb[2] = vw::dot4u(cs, 0x00000101u, base);
    r.gb[3] = vw::dot4u(cs, 0x00010101u, base);
    st.got += vw::readlane(inc, 63);
    return r;
}

// A record staged through LDS in pieces of up to SB bytes (plus 8 bytes of
// look-ahead), loaded with 16-byte buffer loads: one load latency per piece
// instead of one per 64-byte window, and no global load between the
// writer's stores (vmcnt counts loads and stores together).  One buffer
// resource per record keeps offsets 32-bit for any input size; its range
// is rounded up to whole dwords (a dword only partly in range reads as 0; at
// most 3 bytes past the record are read, inside the input or its slack).
// Positions are relative to rbase = the record start rounded down to 16.
struct Staged {
    uint8_t *lds;
    vw::brsrc rsr;
    uint32_t re, cbase, cend;
    __device__ void init(uint8_t *l, const uint8_t *rec16, uint32_t rend) {
        lds = l;
        re = rend;
        rsr = vw::make_rsrc(rec16, (re + 3u) & ~3u);
        cbase = cend = 0;
    }
    // make [p, min(p + SB, re)) resident (wave-uniform p)
    __device__ void load(uint32_t p) {
        const uint32_t l = vw::lane_id();
        vw::wave_sync();   // everyone is done with the previous piece
        cbase = p & ~15u;
        cend = umin32(p + SB, re);
        const uint32_t lim = umin32(cend + 8, re);
        for (uint32_t o = 16u * l; cbase + o < lim; o += 1024)
            *reinterpret_cast<uint4 *>(lds + o) = vw::bload16(rsr, cbase + o);
        vw::wave_sync();
    }
    // window [k0, k0 + w) (clipped to re) resident
    __device__ __forceinline__ void need(uint32_t k0, uint32_t w = 64) {
        if (k0 < cbase || umin32(k0 + w, re) > cend) load(k0);
    }
    __device__ __forceinline__ uint32_t at(uint32_t k) const { return lds[k - cbase]; }
    // the dword at 4-aligned k (bytes past the staged data read as garbage)
    __device__ __forceinline__ uint32_t at4(uint32_t k) const { return *reinterpret_cast<const uint32_t *>(lds + (k - cbase)); }
};

// REQ bytes [r0, r0 + req): TAB count and the C-string length (first NUL).
__device__ __forceinline__ void scan_req(Staged &sg, uint32_t r0, uint32_t req, uint32_t *tabs, uint32_t *slen) {
    const uint32_t l = vw::lane_id();
    uint32_t t = 0, z = req;
    for (uint32_t b0 = 0; b0 < req; b0 += 64) {
        sg.need(r0 + b0);
        const uint32_t k = b0 + l;
        const uint32_t b = k < req ? sg.at(r0 + k) : 0xFFu;
        t += (uint32_t)vw::popc64(vw::ballot(b == '\t'));
        const uint64_t zm = vw::ballot(b == 0);
        if (zm && z == req) z = b0 + (uint32_t)__builtin_ctzll(zm);
    }
    *tabs = t;
    *slen = z;
}

// FULL = 0 ("light"): the sample section is not scanned; a record whose
// header, REQ and final LF look right is assumed simple, and k_dec_write
// verifies the assumption while it writes (code 4 in err: rerun exactly).
template <bool FULL>
__device__ __forceinline__ void plan_one(const VcfcDecodeArgs &a, uint64_t i, uint8_t *sb) {
    const uint32_t l = vw::lane_id();
    const uint64_t rs_abs = a.rec_start[i], re_abs = a.rec_start[i + 1];
    bool simple = false;
    uint64_t size = 0;
    if (re_abs - rs_abs >= 10 && re_abs - rs_abs < (1ull << 31) && a.S > 0 && a.S < (1ull << 31)) {
        const uint64_t rbase = rs_abs & ~15ull;
        const uint32_t rs = (uint32_t)(rs_abs - rbase), re = (uint32_t)(re_abs - rbase);
        Staged sg;
        sg.init(sb, a.in + rbase, re);
        sg.load(rs);
        const uint32_t h0 = sg.at(rs), h4 = sg.at(rs + 4);
        const uint32_t req = ((h4 & 0x3Fu) << 24) | (sg.at(rs + 5) << 16) | (sg.at(rs + 6) << 8) | sg.at(rs + 7);
        if ((h0 >> 6) == 3u && (h4 >> 6) == 3u && req > 0 && 9 + (uint64_t)req < re - rs) {
            uint32_t tabs, slen;
            scan_req(sg, rs + 8, req, &tabs, &slen);
            sg.need(re - 1);
            if (tabs == 9 && sg.at(re - 1) == '\n') {
                simple = true;
                if (FULL) {
                    ItemState st;
                    const uint32_t s0 = rs + 8 + req, s1 = re - 1;
                    for (uint32_t cur = s0 & ~3u; cur < s1 && !st.bad; cur += 256) {
                        sg.need(cur, 256 + 8);
                        const uint32_t b = umin32(cur + 256, s1);
                        (void)scan_window(sg.at4(cur + 4 * l), cur, s0, b, s1, st);
                    }
                    simple = !st.bad && st.got == a.S;
                }
                size = slen + 4 * a.S;
            }
        }
    }
    if (l == 0) {
        a.st[i] = simple ? DS_SIMPLE : DS_SEQ;
        a.line_size[i] = simple ? (uint32_t)size : 0u;
        if (!simple) {
            const uint32_t q = atomicAdd(a.seq_count, 1u);
            a.seq_list[q] = (uint32_t)i;
        }
    }
}

// Selected decodes (a.select set, the range query): a grid of n / SEL_R
// waves; wave g takes records g, g + G, g + 2G, ... (G = waves in the grid)
// and plans / writes the selected ones, so an unselected record costs a flag
// read instead of a wave launch, and a contiguous selected range (a POS
// window) spreads over all waves.
constexpr uint32_t SEL_R = 8;

template <bool FULL, bool SEL>
__global__ __launch_bounds__(256) void k_dec_plan(VcfcDecodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[DEC_WAVES * SBUF];
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    uint8_t *sb = sbuf + wave * SBUF;
    const uint64_t g = (uint64_t)blockIdx.x * DEC_WAVES + wave;
    if (!SEL) {
        if (g < a.n) plan_one<FULL>(a, g, sb);
        return;
    }
    const uint64_t G = (uint64_t)gridDim.x * DEC_WAVES;
    const uint32_t l = vw::lane_id();
    const uint64_t il = g + (uint64_t)l * G;   // lane l < SEL_R: the wave's l-th record
    const bool mine = l < SEL_R && il < a.n;
    const bool on = mine && a.select[il];
    if (mine && !on) { a.st[il] = DS_SKIP; a.line_size[il] = 0; }
    for (uint64_t m = vw::ballot(on); m; m &= m - 1)
        plan_one<FULL>(a, g + (uint64_t)__builtin_ctzll(m) * G, sb);
}

// Light plan, one lane per record: only the header bits, the REQ length and
// the final LF are read.  A record that passes is assumed simple with
// REQ' = REQ (no NUL inside it) and exactly 9 TABs in it; k_dec_write checks
// both while it copies REQ (and the sample section while it decodes it) and
// reports code 4 where the assumption was wrong, so the batch is planned
// again exactly (plan_one<true>).
template <bool SEL>
__global__ __launch_bounds__(256) void k_dec_plan_light(VcfcDecodeArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    if (SEL && !a.select[i]) {
        a.st[i] = DS_SKIP;
        a.line_size[i] = 0;
        return;
    }
    const uint64_t rs = a.rec_start[i], re = a.rec_start[i + 1];
    bool simple = false;
    uint64_t size = 0;
    if (re - rs >= 10 && re - rs < (1ull << 31) && a.S > 0 && a.S < (1ull << 31)) {
        const uint8_t *h = a.in + rs;
        const uint32_t req = be30(h + 4);
        if ((h[0] >> 6) == 3u && (h[4] >> 6) == 3u && req > 0 && 9 + (uint64_t)req < re - rs && a.in[re - 1] == '\n') {
            simple = true;
            size = req + 4 * a.S;
        }
    }
    a.st[i] = simple ? DS_SIMPLE : DS_SEQ;
    a.line_size[i] = simple && size <= 0xFFFFFFFFull ? (uint32_t)size : 0u;
    if (!simple || size > 0xFFFFFFFFull) {
        if (simple) a.st[i] = DS_SEQ;
        const uint32_t q = atomicAdd(a.seq_count, 1u);
        a.seq_list[q] = (uint32_t)i;
    }
}

// Queued records, one lane each (grid-stride).
__global__ __launch_bounds__(256) void k_dec_seq(VcfcDecodeArgs a) {
    const uint32_t cnt = *a.seq_count;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt; q += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = a.seq_list[q];
        const uint64_t rs = a.rec_start[i], re = a.rec_start[i + 1];
        uint64_t size = 0, end = 0;
        const int r = dec_line_seq(a.in, a.n_bytes, rs, a.S, nullptr, &size, &end);
        uint32_t st;
        if (r != DL_OK || size > 0xFFFFFFFFull) st = DS_ERR;
        else st = end == re ? DS_SEQ : DS_INCONS;
        a.st[i] = st;
        a.line_size[i] = st == DS_ERR ? 0u : (uint32_t)size;
        a.end[i] = end;
        if (st >= DS_INCONS) atomicMin((unsigned long long *)a.err, (unsigned long long)((i << 8) | st));
    }
}

// A record's metadata (record start / end, line start / end, plan status).
struct RecMeta {
    uint64_t rs, re, l0, l1;
    uint32_t st;
};
__device__ __forceinline__ RecMeta rec_meta(const VcfcDecodeArgs &a, uint64_t i) {
    return RecMeta{a.rec_start[i], a.rec_start[i + 1], a.line_off[i], a.line_off[i + 1], a.st[i]};
}

// PRE: the record's metadata comes preloaded in mt (the selected decode),
// else it is loaded here where it is used (the full decode: loading it all
// up front was +1.6 %, profiles/r06/ab/ab_r6selpf_dec.txt)
template <bool PRE>
__device__ __forceinline__ void write_one(const VcfcDecodeArgs &a, uint64_t i, const RecMeta &mt, uint8_t *sb,
                                          uint32_t *W) {
    const uint32_t l = vw::lane_id();
    const uint64_t rs_abs = PRE ? mt.rs : a.rec_start[i];
    const uint64_t L0 = PRE ? mt.l0 : a.line_off[i];
    const uint64_t L1 = PRE ? mt.l1 : a.line_off[i + 1];
    if (L1 > a.out_cap) {
        if (l == 0) atomicMin((unsigned long long *)a.err, (unsigned long long)((i << 8) | 0xFFu));
        return;
    }
    uint8_t *line = a.out + L0;
    const uint32_t rst = PRE ? mt.st : a.st[i];
    if (rst == DS_ERR || rst == DS_SKIP) return;   // no line (size 0)
    if (rst != DS_SIMPLE) {
        if (l == 0) {
            uint64_t size, end;
            (void)dec_line_seq(a.in, a.n_bytes, rs_abs, a.S, line, &size, &end);
        }
        return;
    }
    const uint64_t rbase = rs_abs & ~15ull;
    const uint32_t rs = (uint32_t)(rs_abs - rbase), re = (uint32_t)((PRE ? mt.re : a.rec_start[i + 1]) - rbase);
    const uint32_t S = (uint32_t)a.S;
    Staged sg;
    sg.init(sb, a.in + rbase, re);
    sg.load(rs);
    const uint32_t req = ((sg.at(rs + 4) & 0x3Fu) << 24) | (sg.at(rs + 5) << 16) | (sg.at(rs + 6) << 8) | sg.at(rs + 7);
    const uint32_t slen = (uint32_t)(L1 - L0 - 4ull * S);   // REQ' = line - 4S
    // copy REQ', and check what a light plan assumed: 9 TABs in REQ, REQ'
    // ends at REQ's first NUL (an exact plan made both true)
    // (4 bytes per lane, 256 per step: one step for REQs of the usual size)
    uint32_t tabs = 0, z = req;
    for (uint32_t b0 = 0; b0 < req; b0 += 256) {
        sg.need(rs + 8 + b0, 256);
        const uint32_t k = b0 + 4 * l;
        uint32_t w = 0xFFFFFFFFu, vm = 0;   // vm: bytes of REQ among the four
        if (k < req) {
            __builtin_memcpy(&w, sg.lds + (rs + 8 + k - sg.cbase), 4);   // (unaligned ds_read_b32)
            vm = req - k >= 4 ? 0xFu : (1u << (req - k)) - 1u;
        }
        const uint32_t tm = zero_bytes4(w ^ 0x09090909u) & vm, zmk = zero_bytes4(w) & vm;
        if (k + 4 <= slen) {
            __builtin_memcpy(line + k, &w, 4);
        } else {
            for (uint32_t i = 0; i < 3; i++)
                if (k + i < slen) line[k + i] = (uint8_t)(w >> (8 * i));
        }
        tabs += vw::readlane(vw::scan_add((uint32_t)__builtin_popcount(tm)), 63);
        const uint64_t zl = vw::ballot(zmk != 0);
        if (zl && z == req) {
            const uint32_t f = (uint32_t)__builtin_ctzll(zl);
            z = b0 + 4 * f + (uint32_t)__builtin_ctz(vw::readlane(zmk, f));
        }
    }
    const bool req_bad = tabs != 9 || z != slen;
    uint8_t *tok = line + slen;
    // Token tiles of TB four-byte words "a|b\t".  Each item writes only its
    // word at its first token's slot in the LDS tile (W); a tile then fills
    // every slot from the last item start at or before it ("last non-zero":
    // in-lane, then across lanes by a max-scan of lane indices and one
    // ds_bpermute) and goes out as contiguous 16-byte stores.  Work per tile
    // does not depend on run lengths.
    constexpr uint32_t PL = TB / 64;   // slots per lane
    for (uint32_t q = 0; q < PL; q += 4) *reinterpret_cast<uint4 *>(W + PL * l + q) = make_uint4(0, 0, 0, 0);
    uint32_t j0 = 0, carry = 0;   // tile start; word of the item holding token j0
    // LAST: the line's last tile (n_tok tokens, its LF replacing the last
    // TAB, partial stores); the others are whole tiles of TB tokens
    auto tile_out = [&](auto last_tag, uint32_t n_tok) {
        constexpr bool LAST = decltype(last_tag)::value;
        vw::wave_sync();
        uint32_t w[PL];
#pragma unroll
        for (uint32_t q = 0; q < PL; q += 4) {
            const uint4 v = *reinterpret_cast<const uint4 *>(W + PL * l + q);
            w[q] = v.x; w[q + 1] = v.y; w[q + 2] = v.z; w[q + 3] = v.w;
            *reinterpret_cast<uint4 *>(W + PL * l + q) = make_uint4(0, 0, 0, 0);
        }
        uint32_t lastw = 0;
#pragma unroll
        for (uint32_t q = 0; q < PL; q++) {
            lastw = w[q] ? w[q] : lastw;
            w[q] = lastw;
        }
        // word entering the lane: the last start in an earlier lane (words are
        // never 0: byte 3 is TAB), else carry
        const uint32_t inw = vw::shr1z(vw::scan_last_nz(lastw));
        const uint32_t enter = inw ? inw : carry;
#pragma unroll
        for (uint32_t q = 0; q < PL; q++) w[q] = w[q] ? w[q] : enter;
        const uint32_t t0 = j0 + PL * l;
        if (!LAST) {
#pragma unroll
            for (uint32_t q = 0; q < PL; q += 4)
                // plain stores: 2.645 -> 2.49 ms against non-temporal ones in
                // an A/B (profiles/r03/ab/ab_dec_plain.txt; tools/write_probe.hip:
                // one wave per 10 KB line writes 10.19 GB in 2.07 ms plain,
                // 2.25 ms non-temporal)
                vw::gstore16(tok, 4ull * (t0 + q), make_uint4(w[q], w[q + 1], w[q + 2], w[q + 3]));
        } else {
#pragma unroll
            for (uint32_t q = 0; q < PL; q++)
                if (t0 + q + 1 == S) w[q] = (w[q] & 0x00FFFFFFu) | 0x0A000000u;
            if (t0 + PL <= j0 + n_tok) {
#pragma unroll
                for (uint32_t q = 0; q < PL; q += 4)
                    vw::gstore16(tok, 4ull * (t0 + q), make_uint4(w[q], w[q + 1], w[q + 2], w[q + 3]));
            } else {
                for (uint32_t q = 0; q < PL; q++)
                    if (t0 + q < j0 + n_tok) *reinterpret_cast<uint32_t *>(tok + 4ull * (t0 + q)) = w[q];
            }
        }
        carry = vw::readlane(w[PL - 1], 63);
        vw::wave_sync();
    };
    const uint32_t s0 = rs + 8 + req, s1 = re - 1;
    ItemState st;
#ifdef VCFC_DIAG_DEC_NOSCAN   // (diagnostic, wrong output: the line's tile stores without the item scan)
    for (; j0 + TB < S; j0 += TB) tile_out(std::false_type(), TB);
    st.got = S;
    if (j0 < S) tile_out(std::true_type(), S - j0);
    (void)s0; (void)s1; (void)req_bad;
    return;
#endif
    for (uint32_t cur = s0 & ~3u; cur < s1; cur += 256) {
        sg.need(cur, 256 + 8);
        const uint32_t b = umin32(cur + 256, s1);
        // the lane's dword and the next one (an escape's payload may run into it)
        const uint32_t v4 = sg.at4(cur + 4 * l), v4n = sg.at4(cur + 4 * l + 4);
        const ItemLane it = scan_window(v4, cur, s0, b, s1, st);
        // item words "a|b\t" (little-endian), branch-free: an escape (0xE1)
        // gives its 3 payload bytes, a 0|0 run byte (< 0x80) "0|0", a phased
        // run byte 0x80 / 0xA0 / 0xC0 "1|1" / "0|1" / "1|0"; and the token
        // index of each item start (~0 for bytes that start none: never in a tile)
        // (round 5: the allele bits of all four bytes at once -- a run byte
        // 0x80 / 0xA0 / 0xC0 has a = 1 unless bit 5, b = 1 unless bit 6, a
        // 0|0 run byte (< 0x80) neither -- and each word "a|b\t" by one
        // v_perm of the two bit words: 11 VALU per byte -> 6)
        const uint32_t h7 = (v4 >> 7) & 0x01010101u;
        const uint32_t ab = h7 & ~(v4 >> 5), bb = h7 & ~(v4 >> 6);
        uint32_t w[4], ws[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t pay = (j < 3 ? vw::alignbyte(v4n, v4, j + 1) : v4n) & 0x00FFFFFFu;
            const uint32_t ph = vw::perm(ab, bb, 0x0C000C04u + j * 0x00010001u) | 0x09307C30u;
            w[j] = (it.e1 >> j) & 1u ? (pay | 0x09000000u) : ph;
            ws[j] = (it.start >> j) & 1u ? it.gb[j] : ~0u;
        }
        for (;;) {
            // every item writes: its slot if it starts in this tile, else
            // one dummy word past the tile shared by the wave (no branches;
            // a dummy word per lane collides with other lanes' slot stores
            // on the same banks: -0.9 % in an A/B, ab_dec_shared_dummy.txt)
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t o = ws[j] - j0;
                W[o < TB ? o : TB] = w[j];
            }
            // the tile is not complete yet, or it is the line's last
            if (st.got < j0 + TB || j0 + TB >= S) break;
            tile_out(std::false_type(), TB);
            j0 += TB;
        }
    }
    if (j0 < S) tile_out(std::true_type(), S - j0);
    // a light plan assumed this record simple: check it (tokens past S were
    // never stored; the line's bytes are rewritten by the exact rerun)
    if ((st.bad || st.got != S || req_bad) && l == 0)
        atomicMin((unsigned long long *)a.err, (unsigned long long)((i << 8) | 4u));
}

template <bool SEL>
__global__ __launch_bounds__(256) void k_dec_write(VcfcDecodeArgs a, uint64_t first, uint64_t last) {
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[DEC_WAVES * SBUF];
    __shared__ __attribute__((aligned(16))) uint32_t tbuf[DEC_WAVES * (TB + 4)];   // tile + the shared dummy word (16-B padded)
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    uint8_t *sb = sbuf + wave * SBUF;
    uint32_t *W = tbuf + wave * (TB + 4);
    const uint64_t g = (uint64_t)blockIdx.x * DEC_WAVES + wave;
    if (!SEL) {
        if (first + g < last) write_one<false>(a, first + g, RecMeta{0, 0, 0, 0, 0}, sb, W);
        return;
    }
    const uint64_t G = (uint64_t)gridDim.x * DEC_WAVES;
    const uint32_t l = vw::lane_id();
    const uint64_t il = first + g + (uint64_t)l * G;
    // (round 6: each candidate's metadata loaded with its flag, by its own
    // lane, so the selected record's loads do not wait for the flags)
    const bool cand = l < SEL_R && il < last;
    const RecMeta ml = cand ? rec_meta(a, il) : RecMeta{0, 0, 0, 0, 0};
    for (uint64_t m = vw::ballot(cand && a.select[il]); m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        auto rl64 = [&](uint64_t v) {
            return ((uint64_t)vw::readlane((uint32_t)(v >> 32), j) << 32) | vw::readlane((uint32_t)v, j);
        };
        const RecMeta mj{rl64(ml.rs), rl64(ml.re), rl64(ml.l0), rl64(ml.l1), vw::readlane(ml.st, j)};
        write_one<true>(a, first + g + (uint64_t)j * G, mj, sb, W);
    }
}

// Byte-serial decode of [p, n), at most max_lines lines: out == nullptr
// counts (lines, bytes, end state), else writes.  One lane.  st[0] = DL_OK
// (max_lines reached), DL_END (clean end) or DL_ERR; st[1] = bytes; st[2] =
// lines; st[3] = where the parse stopped.
__global__ void k_dec_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint64_t max_lines, uint8_t *out,
                             uint64_t *st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t o = 0, lines = 0;
    int r = DL_OK;
    while (lines < max_lines) {
        uint64_t size = 0, end = 0;
        r = dec_line_seq(in, n, p, S, out ? out + o : nullptr, &size, &end);
        if (r != DL_OK) break;
        o += size;
        p = end;
        lines++;
    }
    st[0] = (uint64_t)r;
    st[1] = o;
    st[2] = lines;
    st[3] = p;
}


// ---------------------------------------------------------------------------
// Range query: query_compressed_file (reference src/main.cpp:3777-3929).
// Per record the reference reads LEN and REQ (8 bytes), then CHROM and POS
// byte by byte up to a TAB each; POS goes through str_to_uint64
// (src/utils.cpp:152-165: strtoul over the whole field, "" is 0) and throws
// when that fails.  A match (VcfCoordinateQuery::matches, :75-86) decodes the
// line from the record start and goes on where the decode ends; otherwise the
// walk seeks LEN - (bytes read - 4) further, which is the next LEN hop
// whenever CHROM and POS lie inside the record.

// strtoul(s, &end, 10) with end == s + n required; n == 0 parses as 0
__device__ __forceinline__ bool pos_parse(const uint8_t *s, uint64_t n, uint64_t *out) {
    if (n == 0) { *out = 0; return true; }
    uint64_t i = 0;
    while (i < n && (s[i] == ' ' || (s[i] >= '\t' && s[i] <= '\r'))) i++;
    bool neg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    if (i >= n || s[i] < '0' || s[i] > '9') return false;
    uint64_t v = 0;
    bool ovf = false;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        const uint64_t d = (uint64_t)(s[i] - '0');
        ovf = ovf || v > (~0ull - d) / 10;
        v = v * 10 + d;
    }
    if (i != n) return false;
    *out = ovf ? ~0ull : (neg ? 0ull - v : v);
    return true;
}

__device__ __forceinline__ bool query_matches(const VcfcQuery &q, const uint8_t *name, uint64_t name_len, uint64_t pos) {
    if (q.ref_len) {
        if (name_len != q.ref_len) return false;
        for (uint32_t k = 0; k < q.ref_len; k++)
            if (name[k] != q.ref[k]) return false;
    }
    return !q.has_range || (pos >= q.start && pos <= q.end);
}

// CHROM and POS of the record at p (CHROM starts at p + 8): *f1 = POS start,
// *f2 = the TAB after POS (both TABs searched below lim)
__device__ __forceinline__ bool query_fields(const uint8_t *in, uint64_t p, uint64_t lim, uint64_t *f1, uint64_t *f2) {
    uint64_t k = p + 8;
    while (k < lim && in[k] != '\t') k++;
    if (k >= lim) return false;
    *f1 = ++k;
    while (k < lim && in[k] != '\t') k++;
    if (k >= lim) return false;
    *f2 = k;
    return true;
}

// bit j of the result: byte j of x is a TAB (exact per byte)
__device__ __forceinline__ uint32_t tab_bits(uint32_t x) {
    const uint32_t t = x ^ 0x09090909u;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);   // 0x80 in each zero byte
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// One lane per record.  Fast path: the 32 bytes from the 16-byte block
// holding the CHROM start lie inside the record; two 16-byte loads, TABs
// found by SWAR in registers, the fields parsed from an LDS copy.  Otherwise
// (CHROM + POS longer than the window holds) byte by byte.  (32 bytes hold
// "22\t" + a 9-digit POS + TAB from any of the 16 phases; round 6: 48 -> 32,
// one load and ~13 % of the cache lines fewer per record.)
constexpr uint32_t QM_WIN = 32;
__global__ __launch_bounds__(256) void k_query_match(const uint8_t *in, const uint64_t *rec, uint64_t n, VcfcQuery q,
                                                     uint8_t *flag, uint64_t *err) {
    __shared__ __attribute__((aligned(16))) uint8_t win[256 * QM_WIN];
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t rs = rec[i], re = rec[i + 1];
    const uint8_t *p = in + rs + 8;
    const uint8_t *a = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)15);
    uint64_t f1 = 0, f2 = 0, pos = 0;
    uint32_t code = 0;
    bool m = false, done = false;
    if (a + QM_WIN <= in + re) {
        const uint4 *g = reinterpret_cast<const uint4 *>(a);
        const uint4 v0 = g[0], v1 = g[1];
        uint4 *w = reinterpret_cast<uint4 *>(win + threadIdx.x * QM_WIN);
        w[0] = v0; w[1] = v1;
        const uint64_t tabs = (uint64_t)tab_bits(v0.x) | (uint64_t)tab_bits(v0.y) << 4 | (uint64_t)tab_bits(v0.z) << 8 |
                              (uint64_t)tab_bits(v0.w) << 12 | (uint64_t)tab_bits(v1.x) << 16 |
                              (uint64_t)tab_bits(v1.y) << 20 | (uint64_t)tab_bits(v1.z) << 24 |
                              (uint64_t)tab_bits(v1.w) << 28;
        const uint32_t sh = (uint32_t)(p - a);
        const uint64_t t = tabs >> sh;
        const uint64_t t2 = t & (t - 1);
        if (t2) {   // both TABs inside the window
            const uint32_t c = (uint32_t)__builtin_ctzll(t), d = (uint32_t)__builtin_ctzll(t2);
            const uint8_t *f = win + threadIdx.x * QM_WIN + sh;
            if (!pos_parse(f + c + 1, d - c - 1, &pos)) code = 2;
            else m = query_matches(q, f, c, pos);
            done = true;
        }
    }
    if (!done) {
        if (!query_fields(in, rs, re, &f1, &f2)) code = 3;
        else if (!pos_parse(in + f1, f2 - f1, &pos)) code = 2;
        else m = query_matches(q, in + rs + 8, f1 - 1 - (rs + 8), pos);
    }
    flag[i] = m ? 1 : 0;
    if (code) atomicMin((unsigned long long *)err, (unsigned long long)((i << 8) | code));
}

// One lane: the reference's walk over in[p, n); out == nullptr counts.
// st[0] = 0 (clean end) or DL_ERR (the reference throws), st[1] = bytes,
// st[2] = lines.
__global__ void k_query_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, VcfcQuery q, uint8_t *out,
                               uint64_t *st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t o = 0, lines = 0;
    int r = 0;
    while (p < n) {
        if (n - p < 8) { r = DL_ERR; break; }   // "Only read %d bytes, expected 4"
        uint64_t f1, f2, pos = 0;
        if (!query_fields(in, p, n, &f1, &f2)) { r = DL_ERR; break; }   // EOF inside CHROM / POS
        if (!pos_parse(in + f1, f2 - f1, &pos)) { r = DL_ERR; break; }
        if (query_matches(q, in + p + 8, f1 - 1 - (p + 8), pos)) {
            uint64_t size = 0, end = 0;
            if (dec_line_seq(in, n, p, S, out ? out + o : nullptr, &size, &end) != DL_OK) { r = DL_ERR; break; }
            o += size;
            lines++;
            p = end;
        } else {
            if ((in[p] >> 6) != 3u) { r = DL_ERR; break; }   // LEN's extension count
            const uint32_t skip = be30(in + p) - (uint32_t)(f2 + 1 - p - 4);   // uint32, as the reference
            const uint64_t at = f2 + 1;
            if ((uint64_t)skip > n - at) break;          // seek past EOF: the next read returns 0
            p = at + skip;
        }
    }
    st[0] = (uint64_t)r;
    st[1] = o;
    st[2] = lines;
}

}  // namespace

VcfcDecodeLayout vcfc_decode_workspace_layout(uint64_t n) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    VcfcDecodeLayout L;
    uint64_t o = 0;
    L.st = o; o = al(o + 4 * (n + 1));
    L.line_size = o; o = al(o + 4 * (n + 1));
    L.end = o; o = al(o + 8 * (n + 1));
    L.seq_list = o; o = al(o + 4 * (n + 1));
    L.seq_count = o; o = al(o + 8);
    L.err = o; o = al(o + 8);
    L.partials = o; o = al(o + 8 * ((n + 4095) / 4096 + 1));
    L.total = o;
    return L;
}

// the per-call words (error word, queued-record count, and with no records
// line_off[0]) in one launch instead of two or three memset blits (~5 us of
// GPU time each; round 6)
namespace {
__global__ void k_dec_reset(uint64_t *err, uint32_t *seq_count, uint64_t *line_off0) {
    if (threadIdx.x == 0) {
        *err = ~0ull;
        if (seq_count) *seq_count = 0;
        if (line_off0) *line_off0 = 0;
    }
}
}  // namespace

hipError_t vcfc_decode_plan(const VcfcDecodeArgs &a, bool exact, hipStream_t s) {
    hipLaunchKernelGGL(k_dec_reset, dim3(1), dim3(64), 0, s, a.err, a.seq_count, a.n == 0 ? a.line_off : nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || a.n == 0) return e;
    const uint64_t per_wave = a.select ? SEL_R : 1;
    const dim3 grid((unsigned)((a.n + DEC_WAVES * per_wave - 1) / (DEC_WAVES * per_wave))), block(64 * DEC_WAVES);
    const dim3 lgrid((unsigned)((a.n + 255) / 256));
    if (a.select) {
        if (exact) hipLaunchKernelGGL((k_dec_plan<true, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL(k_dec_plan_light<true>, lgrid, dim3(256), 0, s, a);
    } else {
        if (exact) hipLaunchKernelGGL((k_dec_plan<true, false>), grid, block, 0, s, a);
        else hipLaunchKernelGGL(k_dec_plan_light<false>, lgrid, dim3(256), 0, s, a);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t want = (a.n + 255) / 256;
    hipLaunchKernelGGL(k_dec_seq, dim3((unsigned)(want < 1024 ? want : 1024)), dim3(256), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return vcfc_scan_u32(a.line_size, a.n, a.partials, a.line_off, s);
}

hipError_t vcfc_decode_write(const VcfcDecodeArgs &a, uint64_t first, uint64_t last, hipStream_t s) {
    if (last <= first) return hipSuccess;
    const uint64_t per_block = DEC_WAVES * (a.select ? SEL_R : 1);
    const dim3 grid((unsigned)((last - first + per_block - 1) / per_block)), block(64 * DEC_WAVES);
    if (a.select) hipLaunchKernelGGL(k_dec_write<true>, grid, block, 0, s, a, first, last);
    else hipLaunchKernelGGL(k_dec_write<false>, grid, block, 0, s, a, first, last);
    return hipGetLastError();
}

hipError_t vcfc_decode_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint64_t max_lines,
                              uint8_t *out, uint64_t *st, hipStream_t s) {
    hipLaunchKernelGGL(k_dec_stream, dim3(1), dim3(64), 0, s, in, n, p, S, max_lines, out, st);
    return hipGetLastError();
}

hipError_t vcfc_query_match(const uint8_t *in, const uint64_t *rec_start, uint64_t n, const VcfcQuery &q,
                            uint8_t *flag, uint64_t *err, hipStream_t s) {
    hipLaunchKernelGGL(k_dec_reset, dim3(1), dim3(64), 0, s, err, nullptr, nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(k_query_match, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, rec_start, n, q, flag, err);
    return hipGetLastError();
}

hipError_t vcfc_query_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, const VcfcQuery &q, uint8_t *out,
                             uint64_t *st, hipStream_t s) {
    hipLaunchKernelGGL(k_query_stream, dim3(1), dim3(64), 0, s, in, n, p, S, q, out, st);
    return hipGetLastError();
}
