// vcfc_encode.hip -- gfx950 kernels for the `.vcfc` genotype-line encoder.
//
// Replaces compress_data_line (reference src/compress.cpp:5-203) for a batch
// of lines resident in HBM.  Pipeline (all on one stream, no host sync):
//
//   scan<BOUND>  slot_off[i] = sum_{k<i} slot_bytes(len_k)     (tiny)
//   k_encode     one wave64 per row: tokenise, RLE-encode, stage the record
//                in an LDS ring, stream it to the row's slot in 1 KiB bursts
//   scan<IDENT>  rec_off[i] = sum_{k<i} rec_size_k             (tiny)
//   k_compact    16 lanes per row: slot -> final offset, 16-byte stores
//
// Record layout (reference compress.cpp:32-100,188-199):
//   [LEN:4 BE|0xC0][REQ:4 BE|0xC0][cols 0..7 '\t'-joined]['\t'FORMAT]['\t']
//   [genotype bytes]['\n'],  LEN = record bytes - 4.
// Genotype bytes (compress.cpp:124-186, masks utils.hpp:44-56):
//   runs of "0|0" -> count (<=127); runs of "0|1"/"1|0"/"1|1" -> 0xA0/0xC0/0x80
//   | count (<=31), split greedily from the run start; any other token ->
//   0xE1, raw bytes, '\t' unless it is the last token.  Fields are maximal
//   non-TAB runs: empty fields vanish (split_string, utils.cpp:82-112).
//
// Emission rule used by both paths (equivalent to the reference's loop): every
// token start emits, in order, [TAB if the previous token was an escape]
// [pending byte of the previous run if that run ends here and its last chunk
// was partial][0xE1 + raw bytes if escape | full-chunk byte if this token
// completes a chunk of `cap`].  The row end emits the last pending chunk and
// '\n'.  Run starts come from a wave max-scan, byte offsets from an add-scan.
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

namespace {

constexpr int K1_WAVES = 4;            // rows per 256-thread block
constexpr uint32_t RING = 4096;        // per-wave LDS ring (bytes)
constexpr uint32_t RMASK = RING - 1;
constexpr uint32_t BURST = 1024;       // flush granule (64 lanes x 16 B)
constexpr uint32_t CLS_ESC = 4, CLS_NONE = 5;

__device__ __forceinline__ uint32_t cls_cap(uint32_t c) { return c == 0 ? 127u : 31u; }
__device__ __forceinline__ uint32_t cls_mask(uint32_t c) {
    // 0|0 -> 0x00, 0|1 -> 0xA0, 1|0 -> 0xC0, 1|1 -> 0x80 (utils.hpp:45-50)
    return c == 0 ? 0x00u : c == 1 ? 0xA0u : c == 2 ? 0xC0u : 0x80u;
}
// class of a 3-byte token packed little-endian in the low 24 bits
__device__ __forceinline__ uint32_t cls_of(uint32_t k) {
    return k == 0x307C30u ? 0u : k == 0x317C30u ? 1u : k == 0x307C31u ? 2u : k == 0x317C31u ? 3u : CLS_ESC;
}
// bit i set <=> byte i of w is zero (exact, no false positives)
__device__ __forceinline__ uint32_t zero_bytes4(uint32_t w) {
    uint32_t t = ((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu;
    t = ~t;  // 0x80 in every zero byte
    return ((t >> 7) * 0x00204081u >> 21) & 0xFu;
}
__device__ __forceinline__ uint32_t tab_mask16(uint4 v) {
    return zero_bytes4(v.x ^ 0x09090909u) | (zero_bytes4(v.y ^ 0x09090909u) << 4) |
           (zero_bytes4(v.z ^ 0x09090909u) << 8) | (zero_bytes4(v.w ^ 0x09090909u) << 12);
}
__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t i) {
    uint32_t w = i < 4 ? v.x : i < 8 ? v.y : i < 12 ? v.z : v.w;
    return (w >> (8 * (i & 3))) & 0xFFu;
}
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------
// LDS ring: record bytes [fpos, wpos) are pending; slot = global staging.
struct Ring {
    uint8_t *lds;
    uint8_t *slot;
    uint32_t wpos, fpos;
};

__device__ __forceinline__ void ring_put(Ring &r, uint32_t pos, uint32_t b) {
    r.lds[pos & RMASK] = (uint8_t)b;
}

// Stream every complete 1 KiB burst (or, at the end, everything) to the slot.
__device__ void ring_flush(Ring &r, bool final) {
    const uint32_t l = vw::lane_id();
    vw::wave_sync();
    while (r.wpos - r.fpos >= BURST) {
        const uint4 v = *reinterpret_cast<const uint4 *>(r.lds + ((r.fpos + 16u * l) & RMASK));
        *reinterpret_cast<uint4 *>(r.slot + r.fpos + 16u * l) = v;
        r.fpos += BURST;
    }
    if (final && r.wpos > r.fpos) {
        const uint32_t rem = r.wpos - r.fpos;  // < BURST
        if (16u * l < rem) {
            const uint4 v = *reinterpret_cast<const uint4 *>(r.lds + ((r.fpos + 16u * l) & RMASK));
            *reinterpret_cast<uint4 *>(r.slot + r.fpos + 16u * l) = v;
        }
        r.fpos = r.wpos;
    }
    vw::wave_sync();
}

// Finish a record: header words go straight to the slot (lane 0 also wrote
// the slot's first 16 bytes during the flush, so program order keeps them).
__device__ void ring_finish(Ring &r, uint32_t req) {
    ring_flush(r, true);
    if (vw::lane_id() == 0) {
        const uint32_t L = r.wpos - 4;
        const uint32_t h0 = (((L >> 24) & 0xFFu) | 0xC0u) | (((L >> 16) & 0xFFu) << 8) |
                            (((L >> 8) & 0xFFu) << 16) | ((L & 0xFFu) << 24);
        const uint32_t h1 = (((req >> 24) & 0xFFu) | 0xC0u) | (((req >> 16) & 0xFFu) << 8) |
                            (((req >> 8) & 0xFFu) << 16) | ((req & 0xFFu) << 24);
        reinterpret_cast<uint32_t *>(r.slot)[0] = h0;
        reinterpret_cast<uint32_t *>(r.slot)[1] = h1;
    }
}

// ---------------------------------------------------------------------------
// Fast path: clean prefix (no empty fields before the first sample) and a
// genotype region of 3-byte tokens separated by single TABs -- the shape of
// every GT-only VCF.  One wave streams the row in 1 KiB aligned chunks (lane l
// owns bytes [16l, 16l+16) of a chunk), two chunks in flight.  Returns false
// (nothing committed) if the row does not have that shape.
__device__ bool encode_fast(const uint8_t *__restrict__ line, uint32_t len, Ring &r,
                            uint32_t *rec_bytes) {
    const uint32_t l = vw::lane_id();
    const uint4 *A = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(line) & ~uintptr_t(15));
    const uint32_t lead = (uint32_t)(reinterpret_cast<uintptr_t>(line) & 15);
    const uint32_t span = lead + len;
    const uint32_t nch = (span + BURST - 1) / BURST;
    const uint4 zero = make_uint4(0, 0, 0, 0);

    auto load = [&](uint32_t c) -> uint4 {
        const uint32_t bo = c * BURST + 16u * l;
        return bo < span ? A[bo >> 4] : zero;
    };

    uint32_t nf = 0;         // field starts seen so far
    uint32_t carryT = 1;     // byte before this chunk is TAB / outside the line
    int32_t gt0 = -1;        // line offset of the first sample token
    uint32_t T = 0, phi = 0;
    uint32_t pcls = CLS_NONE, prs = 0;  // class / run start(+1) of the previous token
    r.wpos = 8;
    r.fpos = 0;

    uint4 cur = load(0);
    uint4 nxt = nch > 1 ? load(1) : zero;
    for (uint32_t c = 0; c < nch; c++) {
        const uint4 nn = (c + 2 < nch) ? load(c + 2) : zero;
        const uint32_t bo = c * BURST + 16u * l;   // byte offset of this lane from A
        const int32_t x0 = (int32_t)bo - (int32_t)lead;  // line offset of byte 0

        if (gt0 < 0) {
            // ---- prefix: locate the 10th field start, reject empty fields ----
            const int32_t vlo = x0 >= 0 ? 0 : (-x0 >= 16 ? 16 : -x0);
            const int32_t vhi0 = (int32_t)len - x0;
            const int32_t vhi = vhi0 <= 0 ? 0 : (vhi0 >= 16 ? 16 : vhi0);
            const uint32_t vm = vhi > vlo ? (((1u << vhi) - 1u) ^ ((1u << vlo) - 1u)) : 0u;
            const uint32_t m = tab_mask16(cur) & vm;
            const uint32_t Tm = (m | ~vm) & 0xFFFFu;
            const uint32_t pin = vw::shr1((Tm >> 15) & 1u, carryT);
            const uint32_t prevT = ((Tm << 1) | pin) & 0xFFFFu;
            const uint32_t fs = ~Tm & prevT & 0xFFFFu;     // field starts
            const uint32_t et = m & prevT;                 // TAB closing an empty field
            carryT = vw::readlane((Tm >> 15) & 1u, 63);
            const uint32_t cnt = (uint32_t)__builtin_popcount(fs);
            const uint32_t inc = vw::scan_add(cnt);
            const uint32_t exc = inc - cnt;
            const bool has9 = nf + exc <= 9 && 9 < nf + inc;
            uint32_t x9 = 0xFFFFFFFFu;
            if (has9) {
                uint32_t mm = fs;
                for (uint32_t k = nf + exc; k < 9; k++) mm &= mm - 1;
                x9 = (uint32_t)(x0 + __builtin_ctz(mm));
            }
            const uint64_t hb = vw::ballot(has9);
            if (hb) x9 = vw::readlane(x9, (uint32_t)__builtin_ctzll(hb));
            // empty field before the first sample -> general path
            uint32_t below = 0xFFFFu;
            if (hb) {
                const int32_t d = (int32_t)x9 - x0;
                below = d <= 0 ? 0u : d >= 16 ? 0xFFFFu : ((1u << d) - 1u);
            }
            if (vw::ballot((et & below) != 0)) return false;
            // copy prefix bytes [0, min(x9, len)) of this chunk to the record
            const uint32_t lim = hb ? x9 : len;
            for (uint32_t i = 0; i < 16; i++) {
                const int32_t x = x0 + (int32_t)i;
                if (x >= 0 && (uint32_t)x < lim) ring_put(r, 8u + (uint32_t)x, byte_of(cur, i));
            }
            nf += vw::readlane(inc, 63);
            if (!hb) {
                const int32_t upto = (int32_t)((c + 1) * BURST) - (int32_t)lead;
                r.wpos = 8u + umin32(len, upto <= 0 ? 0u : (uint32_t)upto);
                ring_flush(r, false);
                cur = nxt;
                nxt = nn;
                continue;   // (if this was the last chunk: < 10 fields -> general path)
            }
            gt0 = (int32_t)x9;
            r.wpos = 8u + x9;
            const uint32_t glen = len - x9;
            if (((glen + 1) & 3u) != 0) return false;
            T = (glen + 1) >> 2;
            phi = (lead + x9) & 3u;
        }

        // ---- genotype tokens whose first byte lies in this chunk ----
        // slot j of lane l starts at chunk byte 16l + 4j + phi
        const uint32_t nfill = vw::readlane(nxt.x, 0);
        const uint32_t w4 = vw::shl1(cur.x, nfill);
        uint32_t d[4];
        d[0] = vw::alignbyte(cur.y, cur.x, phi);
        d[1] = vw::alignbyte(cur.z, cur.y, phi);
        d[2] = vw::alignbyte(cur.w, cur.z, phi);
        d[3] = vw::alignbyte(w4, cur.w, phi);
        const int32_t xs0 = x0 + (int32_t)phi - gt0;   // offset of slot 0 from gt0 (multiple of 4)
        const int32_t tfirst_i = (int32_t)(c * BURST) + (int32_t)phi - (int32_t)lead - gt0;
        const uint32_t tfirst = tfirst_i <= 0 ? 0u : (uint32_t)tfirst_i >> 2;  // first token of the chunk
        uint32_t cl[4], tt[4];
        bool v[4];
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t xo = xs0 + 4 * j;
            v[j] = xo >= 0 && (uint32_t)(xo >> 2) < T;
            tt[j] = v[j] ? (uint32_t)(xo >> 2) : 0u;
            const uint32_t tok = d[j] & 0xFFFFFFu;
            const bool tab_in_tok = (zero_bytes4((d[j] ^ 0x09090909u) | 0xFF000000u)) != 0;
            const bool sep_ok = (d[j] >> 24) == 9u || tt[j] + 1 == T;
            bad |= v[j] && (tab_in_tok || !sep_ok);
            cl[j] = cls_of(tok);
        }
        if (vw::ballot(bad)) return false;

        // previous-token class and run starts (values stored +1, 0 = none)
        const uint32_t c3prev = vw::shr1(cl[3], CLS_NONE);
        uint32_t p[4], s[4];
        uint32_t lane_rs = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t pj = (tt[j] == tfirst) ? pcls : (j == 0 ? c3prev : cl[j - 1]);
            p[j] = pj;
            s[j] = v[j] && (cl[j] == CLS_ESC || pj == CLS_ESC || cl[j] != pj);
            if (s[j]) lane_rs = tt[j] + 1;
        }
        const uint32_t rs_inc = vw::scan_max(lane_rs);
        const uint32_t rin = vw::umax(vw::shr1(rs_inc, 0u), prs);

        uint32_t nb[4], pend[4], pcnt[4], full[4], rr[4];
        uint32_t lane_sum = 0;
        uint32_t rprev = rin;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t rj = s[j] ? tt[j] + 1 : rprev;
            rr[j] = rj;
            const uint32_t pj = p[j];
            uint32_t pe = 0, pc = 0;
            if (v[j] && s[j] && pj < CLS_ESC) {
                const uint32_t off = (tt[j] - rprev) % cls_cap(pj);   // offset of token t-1 in its run
                pe = off != cls_cap(pj) - 1 ? 1u : 0u;
                pc = off + 1;
            }
            uint32_t fu = 0;
            if (v[j] && cl[j] < CLS_ESC) fu = ((tt[j] + 1 - rj) % cls_cap(cl[j])) == cls_cap(cl[j]) - 1 ? 1u : 0u;
            pend[j] = pe;
            pcnt[j] = pc;
            full[j] = fu;
            const uint32_t n = v[j] ? ((pj == CLS_ESC ? 1u : 0u) + pe + (cl[j] == CLS_ESC ? 4u : fu)) : 0u;
            nb[j] = n;
            lane_sum += n;
            rprev = v[j] ? rj : rprev;
        }
        const uint32_t inc = vw::scan_add(lane_sum);
        uint32_t pos = r.wpos + inc - lane_sum;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!v[j]) continue;
            if (p[j] == CLS_ESC) ring_put(r, pos++, 0x09u);
            if (pend[j]) ring_put(r, pos++, cls_mask(p[j]) | pcnt[j]);
            if (cl[j] == CLS_ESC) {
                ring_put(r, pos, 0xE1u);
                ring_put(r, pos + 1, d[j] & 0xFFu);
                ring_put(r, pos + 2, (d[j] >> 8) & 0xFFu);
                ring_put(r, pos + 3, (d[j] >> 16) & 0xFFu);
                pos += 4;
            } else if (full[j]) {
                ring_put(r, pos++, cls_mask(cl[j]) | cls_cap(cl[j]));
            }
        }
        r.wpos += vw::readlane(inc, 63);
        // carry the last token of the chunk
        uint32_t lcls = CLS_NONE, lrs = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (v[j]) { lcls = cl[j]; lrs = rr[j]; }
        const uint64_t hv = vw::ballot(lcls != CLS_NONE);
        if (hv) {
            const uint32_t src = (uint32_t)vw::hibit64(hv);
            pcls = vw::readlane(lcls, src);
            prs = vw::readlane(lrs, src);
        }
        ring_flush(r, false);
        cur = nxt;
        nxt = nn;
    }
    if (gt0 < 0) return false;   // fewer than 10 fields
    // row end: pending chunk of the last run, then '\n'
    if (l == 0) {
        uint32_t w = r.wpos;
        if (pcls < CLS_ESC) {
            const uint32_t off = (T - prs) % cls_cap(pcls);
            if (off != cls_cap(pcls) - 1) ring_put(r, w++, cls_mask(pcls) | (off + 1));
        }
        ring_put(r, w, 0x0Au);
    }
    if (pcls < CLS_ESC && ((T - prs) % cls_cap(pcls)) != cls_cap(pcls) - 1) r.wpos++;
    r.wpos++;
    ring_finish(r, (uint32_t)gt0);
    *rec_bytes = r.wpos;
    return true;
}

// ---------------------------------------------------------------------------
// General path: any line.  64-byte windows, one byte per lane (plus a 3-byte
// look-ahead for the token-length test), ballot/scan bookkeeping.  Handles
// empty fields anywhere, 9-column rows, tokens of any length, CR, and the
// reference's error cases (< 8 fields: VcfValidationError; 8: abort).
__device__ uint32_t encode_general(const uint8_t *__restrict__ line, uint32_t len, Ring &r,
                                   uint32_t *rec_bytes) {
    const uint32_t l = vw::lane_id();
    const uint64_t lt = vw::lanemask_lt();
    uint32_t nf = 0;          // fields started so far
    uint32_t carry_tab = 1;   // byte before the window is TAB / line start
    uint32_t ccls = CLS_NONE; // class of the last token started (current token)
    uint32_t crs = 0;         // run start (+1) of the last token started
    uint32_t req = 0;
    r.wpos = 8;
    r.fpos = 0;
    const uint32_t nwin = (len + 63) / 64;
    for (uint32_t w = 0; w < nwin; w++) {
        const uint32_t x = w * 64 + l;
        auto at = [&](uint32_t y) -> uint32_t { return y < len ? (uint32_t)line[y] : 0x09u; };
        const uint32_t b0 = at(x), b1 = at(x + 1), b2 = at(x + 2), b3 = at(x + 3);
        const uint32_t tab = b0 == 0x09u ? 1u : 0u;
        const uint32_t ptab = vw::shr1(tab, carry_tab);
        const bool start = !tab && ptab;
        const uint64_t sm = vw::ballot(start);
        // field index of a non-TAB byte = index of the last start at or before it
        const uint32_t kcur = nf + (uint32_t)vw::popc64(sm & (lt | (1ull << l))) - 1u;
        // token class at a start (3-byte test needs 3 bytes of look-ahead)
        const bool len3 = b1 != 0x09u && b2 != 0x09u && b3 == 0x09u;
        const uint32_t mycls = start ? (len3 ? cls_of(b0 | (b1 << 8) | (b2 << 16)) : CLS_ESC) : CLS_NONE;
        const bool tok_start = start && kcur >= 9;
        const uint32_t t = kcur - 9;   // token index (valid when kcur >= 9)
        // previous token class for a start lane / current token class for any byte
        const uint64_t tsm = vw::ballot(tok_start);
        const uint64_t before = tsm & lt;
        const uint32_t cls_from = vw::shfl(mycls, before ? (uint32_t)vw::hibit64(before) : 0u);
        const uint32_t pcls = before ? cls_from : ccls;        // class of the previous token
        const uint64_t upto = tsm & (lt | (1ull << l));
        const uint32_t cls_cur_from = vw::shfl(mycls, upto ? (uint32_t)vw::hibit64(upto) : 0u);
        const uint32_t curcls = upto ? cls_cur_from : ccls;    // class of the token holding this byte
        const bool s = tok_start && (mycls == CLS_ESC || pcls == CLS_ESC || mycls != pcls);
        const uint32_t rs_inc = vw::scan_max(s ? t + 1 : 0u);
        const uint32_t rj = vw::umax(rs_inc, crs);                       // run start (+1) of this token
        const uint32_t rp = vw::umax(vw::shr1(rs_inc, 0u), crs);         // run start (+1) of the previous
        // counts
        uint32_t n = 0;
        const bool pre_byte = !tab && kcur <= 8;
        const bool pre_tab = start && kcur >= 1 && kcur <= 9;
        n += pre_byte ? 1u : 0u;
        n += pre_tab ? 1u : 0u;
        uint32_t pe = 0, pc = 0, fu = 0;
        if (tok_start) {
            if (s && pcls < CLS_ESC) {
                const uint32_t off = (t - rp) % cls_cap(pcls);
                pe = off != cls_cap(pcls) - 1 ? 1u : 0u;
                pc = off + 1;
            }
            if (mycls < CLS_ESC) fu = ((t + 1 - rj) % cls_cap(mycls)) == cls_cap(mycls) - 1 ? 1u : 0u;
            n += (pcls == CLS_ESC ? 1u : 0u) + pe + (mycls == CLS_ESC ? 2u : fu);
        } else if (!tab && kcur >= 9 && curcls == CLS_ESC) {
            n += 1;   // raw byte inside an escaped token
        }
        const uint32_t inc = vw::scan_add(n);
        uint32_t pos = r.wpos + inc - n;
        if (pre_tab) ring_put(r, pos++, 0x09u);
        if (pre_byte) ring_put(r, pos++, b0);
        if (tok_start) {
            if (pcls == CLS_ESC) ring_put(r, pos++, 0x09u);
            if (pe) ring_put(r, pos++, cls_mask(pcls) | pc);
            if (mycls == CLS_ESC) {
                ring_put(r, pos++, 0xE1u);
                ring_put(r, pos++, b0);
            } else if (fu) {
                ring_put(r, pos++, cls_mask(mycls) | cls_cap(mycls));
            }
        } else if (!tab && kcur >= 9 && curcls == CLS_ESC) {
            ring_put(r, pos++, b0);
        }
        // REQ counts the prefix part only
        const uint32_t npre = (pre_byte ? 1u : 0u) + (pre_tab ? 1u : 0u);
        req += vw::readlane(vw::scan_add(npre), 63);
        r.wpos += vw::readlane(inc, 63);
        // carries
        nf += (uint32_t)vw::popc64(sm);
        carry_tab = vw::readlane(tab, 63);
        if (tsm) {
            const uint32_t last = (uint32_t)vw::hibit64(tsm);
            ccls = vw::readlane(mycls, last);
            crs = vw::readlane(rj, last);
        }
        ring_flush(r, false);
    }
    if (nf < 8) return VCFCD_E_LT8COLS;
    if (nf == 8) return VCFCD_E_8COLS;
    const uint32_t T = nf - 9;
    uint32_t extra = 0;
    if (T > 0 && ccls < CLS_ESC && ((T - crs) % cls_cap(ccls)) != cls_cap(ccls) - 1) extra = 1;
    if (l == 0) {
        if (extra) ring_put(r, r.wpos, cls_mask(ccls) | (((T - crs) % cls_cap(ccls)) + 1));
        ring_put(r, r.wpos + extra, 0x0Au);
    }
    r.wpos += extra + 1;
    ring_finish(r, req);
    *rec_bytes = r.wpos;
    return VCFCD_OK;
}

__global__ __launch_bounds__(256) void k_encode(VcfcEncodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[K1_WAVES * RING];
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t row = (uint64_t)blockIdx.x * K1_WAVES + wave;
    if (row >= a.n) return;
    const uint64_t so = a.slot_off[row];
    const uint32_t len = a.line_len[row];
    Ring r;
    r.lds = lds + wave * RING;
    r.slot = a.slots + so;
    r.wpos = 8;
    r.fpos = 0;
    if (a.slot_off[row + 1] > a.slots_cap) {
        if (vw::lane_id() == 0) {
            a.rec_size[row] = 0;
            atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | VCFCD_E_NOSPACE));
        }
        return;
    }
    const uint8_t *line = a.buf + a.line_off[row];
    uint32_t bytes = 0;
    uint32_t st = VCFCD_OK;
    if (!encode_fast(line, len, r, &bytes)) st = encode_general(line, len, r, &bytes);
    if (vw::lane_id() == 0) {
        a.rec_size[row] = st == VCFCD_OK ? bytes : 0u;
        if (st != VCFCD_OK) atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | st));
    }
}

// ---------------------------------------------------------------------------
// Compaction: 16 lanes per row copy slot -> out[rec_off[row]] with aligned
// 16-byte stores (unaligned head/tail bytes stored singly).
__device__ __forceinline__ uint4 realign16(uint4 lo, uint4 hi, uint32_t sh) {
    const uint32_t q = sh >> 2, s = sh & 3u;
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t o[5];
    for (int i = 0; i < 5; i++) {
        const uint32_t a0 = w[i], a1 = w[i + 1 < 8 ? i + 1 : 7], a2 = w[i + 2 < 8 ? i + 2 : 7],
                       a3 = w[i + 3 < 8 ? i + 3 : 7];
        o[i] = q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : a3;
    }
    return make_uint4(vw::alignbyte(o[1], o[0], s), vw::alignbyte(o[2], o[1], s),
                      vw::alignbyte(o[3], o[2], s), vw::alignbyte(o[4], o[3], s));
}

__global__ __launch_bounds__(256) void k_compact(const uint8_t *__restrict__ slots,
                                                 const uint64_t *__restrict__ slot_off,
                                                 const uint64_t *__restrict__ rec_off, uint64_t n,
                                                 uint8_t *__restrict__ out, uint64_t out_cap,
                                                 uint64_t *err) {
    const uint32_t g = threadIdx.x >> 4, gl = threadIdx.x & 15u;
    const uint64_t row = (uint64_t)blockIdx.x * 16 + g;
    if (row >= n) return;
    const uint64_t d0 = rec_off[row], d1 = rec_off[row + 1];
    if (d1 == d0) return;
    if (d1 > out_cap) {
        if (gl == 0) atomicMin((unsigned long long *)err, (unsigned long long)((row << 8) | VCFCD_E_NOSPACE));
        return;
    }
    const uint8_t *src = slots + slot_off[row];
    uint8_t *dst = out + d0;
    const uint64_t sz = d1 - d0;
    uint32_t head = (uint32_t)((16u - (d0 & 15u)) & 15u);
    if (head > sz) head = (uint32_t)sz;
    if (gl < head) dst[gl] = src[gl];
    const uint64_t body = sz - head;
    const uint64_t nblk = body >> 4;
    const uint32_t tail = (uint32_t)(body & 15u);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    for (uint64_t k = gl; k < nblk; k += 16) {
        const uint64_t sb = head + 16 * k;
        const uint4 lo = s4[sb >> 4];
        const uint4 hi = s4[(sb >> 4) + 1];
        *reinterpret_cast<uint4 *>(dst + sb) = realign16(lo, hi, head);
    }
    if (gl < tail) dst[head + 16 * nblk + gl] = src[head + 16 * nblk + gl];
}

// ---------------------------------------------------------------------------
// Exclusive scan u32 -> u64 (n + 1 outputs).  MODE 0: identity, MODE 1:
// vcfc_slot_bytes(len).  4096 items per 256-thread block.
constexpr int SCAN_ITEMS = 16, SCAN_THREADS = 256, SCAN_TILE = SCAN_ITEMS * SCAN_THREADS;

template <int MODE> __device__ __forceinline__ uint64_t scan_xf(uint32_t v) {
    return MODE == 1 ? vcfc_slot_bytes(v) : (uint64_t)v;
}

__device__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t *sh, uint64_t *total) {
    const uint32_t t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < SCAN_THREADS; o <<= 1) {
        const uint64_t a = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    const uint64_t inc = sh[t];
    *total = sh[SCAN_THREADS - 1];
    __syncthreads();
    return inc - v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t *__restrict__ in, uint64_t n,
                                                     uint64_t *__restrict__ partials) {
    __shared__ uint64_t sh[SCAN_THREADS];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
    for (int i = 0; i < SCAN_ITEMS; i++)
        if (base + i < n) s += scan_xf<MODE>(in[base + i]);
    uint64_t tot;
    block_excl_scan_u64(s, sh, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_partials(uint64_t *p, uint64_t np) {
    __shared__ uint64_t sh[SCAN_THREADS];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < np; b += SCAN_THREADS) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < np ? p[i] : 0;
        uint64_t tot;
        const uint64_t e = block_excl_scan_u64(v, sh, &tot);
        if (i < np) p[i] = carry + e;
        carry += tot;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_scan_apply(const uint32_t *__restrict__ in, uint64_t n,
                                                    const uint64_t *__restrict__ partials,
                                                    uint64_t *__restrict__ out) {
    __shared__ uint64_t sh[SCAN_THREADS];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t vals[SCAN_ITEMS];
    uint64_t s = 0;
    for (int i = 0; i < SCAN_ITEMS; i++) {
        vals[i] = base + i < n ? scan_xf<MODE>(in[base + i]) : 0;
        s += vals[i];
    }
    uint64_t tot;
    uint64_t run = partials[blockIdx.x] + block_excl_scan_u64(s, sh, &tot);
    for (int i = 0; i < SCAN_ITEMS; i++) {
        if (base + i < n) out[base + i] = run;
        run += vals[i];
        if (base + i + 1 == n) out[n] = run;
    }
}

template <int MODE>
hipError_t launch_scan(const uint32_t *in, uint64_t n, uint64_t *partials, uint64_t *out,
                       hipStream_t s) {
    const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_reduce<MODE>, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s, in, n, partials);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(SCAN_THREADS), 0, s, partials, nb);
    hipLaunchKernelGGL(k_scan_apply<MODE>, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s, in, n, partials, out);
    return hipGetLastError();
}

}  // namespace

VcfcWorkspaceLayout vcfc_encode_workspace_layout(uint64_t n, uint64_t total_line_bytes) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    VcfcWorkspaceLayout L;
    uint64_t o = 0;
    L.slot_off = o; o = al(o + 8 * (n + 1));
    L.rec_size = o; o = al(o + 4 * (n + 1));
    L.partials = o; o = al(o + 8 * ((n + SCAN_TILE - 1) / SCAN_TILE + 1));
    L.err = o; o = al(o + 8);
    L.slots = o; o = al(o + total_line_bytes + total_line_bytes / 2 + 64 * (n + 1));
    L.total = o;
    return L;
}

hipError_t vcfc_encode_device(const VcfcEncodeArgs &a, hipStream_t s, hipEvent_t *ev) {
    hipError_t e = hipMemsetAsync(a.err, 0xFF, 8, s);
    if (e != hipSuccess) return e;
    if (a.n == 0) return hipMemsetAsync(a.rec_off, 0, 8, s);
    if (ev) (void)hipEventRecord(ev[0], s);
    e = launch_scan<1>(a.line_len, a.n, a.partials, a.slot_off, s);
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[1], s);
    hipLaunchKernelGGL(k_encode, dim3((unsigned)((a.n + K1_WAVES - 1) / K1_WAVES)), dim3(64 * K1_WAVES), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[2], s);
    e = launch_scan<0>(a.rec_size, a.n, a.partials, a.rec_off, s);
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[3], s);
    hipLaunchKernelGGL(k_compact, dim3((unsigned)((a.n + 15) / 16)), dim3(256), 0, s, a.slots, a.slot_off,
                       a.rec_off, a.n, a.out, a.out_cap, a.err);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[4], s);
    return hipSuccess;
}
