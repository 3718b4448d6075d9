// vcfc_encode.hip -- gfx950 kernels for the `.vcfc` genotype-line encoder.
//
// Replaces compress_data_line (reference src/compress.cpp:5-203) for a batch
// of lines resident in HBM.  Pipeline (all on one stream, no host sync):
//
//   k_scan_lb<1>      slot_off[i] = sum_{k<i} slot_bytes(len_k)   (tiny)
//   k_encode_fast     one wave64 per row: tokenise, RLE-encode, stage the
//                     record in an LDS ring, stream it to the row's staging in
//                     1 KiB bursts; rows of another shape are flagged
//   k_encode_var      one wave per 32 rows, encodes the flagged ones: odd-length
//                     tokens on 2-byte half-slots, any other shape by the
//                     general path (encode_general) in the same wave
//   k_scan_lb<0>      rec_off[i] = sum_{k<i} rec_size_k, + each 4 KiB output
//                     tile's first row                           (tiny)
//   k_compact_out     output-ordered: 4 KiB output tiles, 16-byte stores
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

// Diagnostic builds (tools/, tests/simt_emu) pass -DVCFC_DIAG='"hooks.h"' to
// instrument the kernels; the product build defines every hook empty.
#ifdef VCFC_DIAG
#include VCFC_DIAG
#endif
#ifndef VCFC_DIAG_ROW_BEGIN
#define VCFC_DIAG_ROW_BEGIN()            // k_encode_fast: a row starts
#define VCFC_DIAG_ROW_END(a, row)        // k_encode_fast: the row's record is staged
#define VCFC_DIAG_GENERAL_ROW(a)         // a flagged row takes the general path
#define VCFC_DIAG_WS_BYTES(n) 0ull       // extra workspace bytes (at VcfcWorkspaceLayout::dbg)
#endif

namespace {

constexpr int K1_WAVES = 4;            // rows per 256-thread block
constexpr uint32_t RING = 4096;        // per-wave LDS ring (bytes)
constexpr uint32_t RMASK = RING - 1;
// + a 64-byte tail (a lane's bytes written past the ring end, moved to its
// start afterwards; a lane writes at most 48 bytes per step) + one dummy word
// shared by the wave for the stores that emit nothing (branch-free stores,
// see esc8), padded to keep the next wave's ring 16-B aligned
constexpr uint32_t RING_TAIL = 64;
constexpr uint32_t RING_DUMMY = RING + RING_TAIL;
constexpr uint32_t RING_STRIDE = RING_DUMMY + 16;
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
    // gathered by one v_dot4_u32_u8 (a 32-bit multiply here is v_mul_lo_u32,
    // which issues at a quarter of the rate)
    return vw::dot4u(t >> 7, 0x08040201u, 0u);
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
// LDS ring: record bytes [fpos, wpos) are pending.  Global staging: record
// bytes [0, pb) at prim, the rest at slot (see vcfc_device.h; pb is a
// multiple of BURST, so a burst lies wholly in one region).
// mode: RING_STAGE (the staging), RING_SIZE (nothing leaves the ring: the
// row is only sized, k_encode_var's deferred rows), RING_DIRECT (the record
// goes straight to out: prim = its first byte, pb = ~0, and the last partial
// burst stores exactly the record's bytes -- k_encode_defer)
constexpr uint32_t RING_STAGE = 0, RING_SIZE = 1, RING_DIRECT = 2;
struct Ring {
    uint8_t *lds;
    uint8_t *prim;
    uint8_t *slot;
    uint32_t wpos, fpos;
    uint32_t pb;   // prim_bytes
    uint32_t mode;
};

__device__ __forceinline__ void ring_put(Ring &r, uint32_t pos, uint32_t b) {
    r.lds[pos & RMASK] = (uint8_t)b;
}

// Stream complete 1 KiB bursts to the staging.  A 2 KiB chunk adds < 2.5 KiB to
// a ring holding < 1 KiB, so three unrolled bursts suffice (no loop: a store
// loop of unknown trip count makes hipcc's vmcnt tracking give up on the
// prefetch).
// staging address of record byte f (a burst lies wholly in one region)
// (non-temporal: k_compact reads the staging back only after the whole
// batch, so keeping it out of L2's way helps the input stream -- about 1 %,
// profiles/r01/ab/ab_nt_stores.txt)
// (temporal stores, i.e. staging kept in L2 / the 256 MiB Infinity Cache for
// k_compact: k_compact unchanged at 0.283 ms, k_encode +0.4 %; the staging's
// 0.68 GB are written amid the 10 GB input stream, so it does not stay
// resident -- profiles/r03/ab/ab_staging_cache_policy.txt)
// DYN: the ring's mode is read (the variable-token and deferred paths); the
// fast and general paths always stage and compile without the checks
template <bool DYN = false>
__device__ __forceinline__ void ring_stage(Ring &r, uint32_t f, uint4 v) {
#ifdef VCFC_DIAG_NOSTORE   // (diagnostic, wrong output: no staging stores)
    if (f == 0x7FFFFFFFu) vw::gstore16_nt(r.prim, 0, v);
    return;
#endif
    if (DYN && r.mode == RING_SIZE) return;
    if (DYN && r.mode == RING_DIRECT) {
        // a deferred record straight into out, at the record's own (any)
        // alignment: plain stores, so that L2 merges the 16-byte pieces
        // into whole lines (non-temporal output stores were slower in the
        // compaction too, §4)
#ifdef VCFC_DIAG_NODIRECT   // (diagnostic, wrong output: the deferred records' bursts not stored)
        if (f == 0x7FFFFFFFu) vw::gstore16(r.prim, f, v);
        return;
#endif
        vw::gstore16(r.prim, f, v);
        return;
    }
    if (r.fpos < r.pb) vw::gstore16_nt(r.prim, f, v);
    else vw::gstore16_nt(r.slot, f - r.pb, v);
}
template <bool DYN = false>
__device__ __forceinline__ void ring_burst(Ring &r, uint32_t l) {
    const uint4 v = *reinterpret_cast<const uint4 *>(r.lds + ((r.fpos + 16u * l) & RMASK));
    ring_stage<DYN>(r, r.fpos + 16u * l, v);
    r.fpos += BURST;
}
template <bool DYN = false>
__device__ __forceinline__ void ring_flush(Ring &r, bool final) {
    const uint32_t l = vw::lane_id();
    r.wpos = vw::readfirst(r.wpos);
    r.fpos = vw::readfirst(r.fpos);
    vw::wave_sync();
    if (r.wpos - r.fpos >= BURST) {
        ring_burst<DYN>(r, l);
        if (r.wpos - r.fpos >= BURST) {
            ring_burst<DYN>(r, l);
            if (r.wpos - r.fpos >= BURST) ring_burst<DYN>(r, l);
        }
    }
    if (final && r.wpos > r.fpos) {
        const uint32_t rem = r.wpos - r.fpos;  // < BURST
        if (16u * l < rem) {
            const uint4 v = *reinterpret_cast<const uint4 *>(r.lds + ((r.fpos + 16u * l) & RMASK));
            if (!DYN || r.mode != RING_DIRECT || 16u * l + 16u <= rem) {
                ring_stage<DYN>(r, r.fpos + 16u * l, v);
            } else {   // the record's last bytes in out: not one byte past them (the next record's)
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                for (uint32_t i = 0; 16u * l + i < rem; i++)
                    r.prim[r.fpos + 16u * l + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        }
        r.fpos = r.wpos;
    }
    vw::wave_sync();
}

// Bytes a lane wrote past the ring end (into the 64-byte tail) belong at the
// ring start.  At most one lane of a step straddles the end (the lanes after
// it start from a masked position); the wave moves its tail bytes with one
// byte per lane instead of that lane copying them one by one.
__device__ __forceinline__ void ring_unwrap(Ring &r, uint32_t end) {   // end: the lane's unmasked end position
    const uint64_t wb = vw::ballot(end > RING);
    if (wb) {
        const uint32_t n = vw::readlane(end, (uint32_t)__builtin_ctzll(wb)) - RING;   // <= RING_TAIL
        const uint32_t l = vw::lane_id();
        const uint8_t v = r.lds[RING + l];
        if (l < n) r.lds[l] = v;
    }
}

// Finish a record: header words go straight to the staging (lane 0 also
// wrote its first 16 bytes during the flush, so program order keeps them).
template <bool DYN = false>
__device__ void ring_finish(Ring &r, uint32_t req) {
    ring_flush<DYN>(r, true);
    if (vw::lane_id() == 0 && (!DYN || r.mode != RING_SIZE)) {
        const uint32_t L = r.wpos - 4;
        const uint32_t h0 = (((L >> 24) & 0xFFu) | 0xC0u) | (((L >> 16) & 0xFFu) << 8) |
                            (((L >> 8) & 0xFFu) << 16) | ((L & 0xFFu) << 24);
        const uint32_t h1 = (((req >> 24) & 0xFFu) | 0xC0u) | (((req >> 16) & 0xFFu) << 8) |
                            (((req >> 8) & 0xFFu) << 16) | ((req & 0xFFu) << 24);
        reinterpret_cast<uint32_t *>(r.prim)[0] = h0;
        reinterpret_cast<uint32_t *>(r.prim)[1] = h1;
    }
}

// ---------------------------------------------------------------------------
// Fast path: clean prefix (no empty fields before the first sample) and a
// genotype region of 3-byte tokens separated by single TABs -- the shape of
// every GT-only VCF.  One wave streams the row in 2 KiB aligned chunks: lane l
// owns bytes [32l, 32l+32) of a chunk plus the next 4 bytes, so the 8 token
// slots it classifies (slot j starts at 32l + 4j + phi) are complete in its
// own registers.  Loads are unconditional (clamped inside the line) so two
// chunks stay in flight behind counted vmcnt waits.  Returns false (nothing
// committed) if the row does not have this shape.
constexpr uint32_t TPL = 4;                 // token slots per lane
constexpr uint32_t BPL = 4 * TPL;           // bytes per lane per chunk
constexpr uint32_t CHUNK = 64 * BPL;        // bytes per wave iteration (1 KiB)

__device__ __forceinline__ uint32_t cls_mask_f(uint32_t c) { return (0x80C0A000u >> (8 * (c & 3u))) & 0xFFu; }
// exact x mod cap for x < 2^23 (cap 127 for 0|0 runs, 31 otherwise):
// q = floor(x * m / 2^s) with m = ceil(2^s / cap), s = 30 / 28, whose excess
// m*cap - 2^s (123 / 23) stays below 2^(s-23) -- all 24-bit multiplies.
constexpr uint32_t MOD_BIAS = 3937;   // 127 * 31: keeps run offsets non-negative
__device__ __forceinline__ uint32_t mod_cap(uint32_t x, bool is00) {
    x &= 0x7FFFFFu;
    const uint64_t p = (uint64_t)x * (is00 ? 8454661u : 8659209u);
    const uint32_t q = vw::alignbit((uint32_t)(p >> 32), (uint32_t)p, is00 ? 30u : 28u);
    return (uint32_t)vw::mad24((int32_t)q, is00 ? -127 : -31, (int32_t)x);
}
// class of the token packed in the low 24 bits: 0..3 for 0|0 0|1 1|0 1|1, else ESC
__device__ __forceinline__ uint32_t cls_f(uint32_t w) {
    const bool gt = (w & 0xFEFFFEu) == 0x307C30u;
    return gt ? (((w & 1u) << 1) | ((w >> 16) & 1u)) : CLS_ESC;
}
// class of a token dword known to be "a|b\t" with a, b in {0,1}
__device__ __forceinline__ uint32_t cls_classed(uint32_t w) { return ((w & 1u) << 1) | ((w >> 16) & 1u); }

struct Chunk {
    uint4 a;      // BPL = 16 bytes at A + 16*(chunk*64 + lane)
    uint32_t y;   // the 4 bytes after them
    __device__ __forceinline__ uint32_t w(int k) const {
        return k == 0 ? a.x : k == 1 ? a.y : k == 2 ? a.z : k == 3 ? a.w : y;
    }
};

// cache policy of the encoder's line loads: plain (non-temporal loads are
// 30 % slower: the prefix / genotype chunk overlap and the look-ahead rely on
// L2 hits, profiles/r01/ab/ab_nt_loads.txt)
// (genotype stream alone non-temporal: +14 %, ab_staging_cache_policy.txt)
constexpr int PRE_AUX = 0, GT_AUX = 0;

// The look-ahead dword after a lane's bytes is the next lane's first dword:
// only lane 63 loads it (the other lanes' offsets lie past the range, so
// they make no memory request -- a 4-byte load from every lane costs ~8 % of
// the stream, tools/stream_probe.hip), and look_ahead() fills the others by
// DPP once the chunk is consumed.
constexpr uint32_t LA_OFF = 0x80000000u;   // past any row's range (records < 1 GiB)
__device__ __forceinline__ uint32_t la_off(uint32_t lane_bytes, uint32_t last) {
    return lane_bytes == last ? 0u : LA_OFF;
}

__device__ __forceinline__ Chunk load_chunk(vw::brsrc rs, uint32_t c, uint32_t lo16) {
    Chunk k;
    const uint32_t off = c * CHUNK + lo16;   // lo16 = 16 * lane
    k.a = vw::bload16(rs, off, PRE_AUX);
    k.y = vw::bload4(rs, off + 16u + la_off(lo16, 63 * BPL), PRE_AUX);
    return k;
}
__device__ __forceinline__ Chunk look_ahead(Chunk k) {
    k.y = vw::shl1(k.a.x, k.y);
    return k;
}

struct FastState {
    uint32_t nf;        // field starts seen so far (prefix phase)
    uint32_t carryT;    // byte before this chunk is TAB / outside the line
    int32_t gt0;        // line offset of the first sample token (-1: not found yet)
    uint32_t T, phi;    // token count, gt0's byte phase mod 4
    uint32_t pcls, prs; // class / run start(+1) of the previous token
    uint32_t esc;       // lanes of the last genotype chunk holding an escape: test the escape shape first
    uint32_t hand;      // 1: a first genotype chunk of escapes only hands the row on (deferred records,
                        // > 1 chunk, prefix in the line's first KiB); 2: it did
};

// Prefix bytes of 1 KiB chunk c -> ring[8 + x]: realign the lane's bytes to
// ring dwords (ring position of lane byte i is bo + i + 8 - lead); bytes
// outside [0, x9) land below 8 (header, rewritten) or at >= wpos (free,
// overwritten later) -- written before this chunk's tokens.
__device__ __forceinline__ void prefix_to_ring(const Chunk &cur, uint32_t c, uint32_t lead, Ring &r) {
    const uint32_t l = vw::lane_id();
    const uint32_t bo = c * CHUNK + BPL * l;
    const uint32_t e = (8u - lead) & 3u;
    const int32_t dq = (int32_t)(8u - lead) - (int32_t)e;
    const uint32_t pw = vw::shr1(cur.w(TPL - 1), 0u);
    const uint32_t sh = (4u - e) & 3u;
    uint32_t *rd = reinterpret_cast<uint32_t *>(r.lds);
    const uint32_t base = (uint32_t)((int32_t)bo + dq);
    // dword k holds ring bytes [base + 4k, +4) = lane bytes [4k - e, 4k - e + 4)
#pragma unroll
    for (int k = 0; k <= (int)TPL; k++) {
        const uint32_t lo = k == 0 ? pw : cur.w(k - 1);
        const uint32_t hi = cur.w(k);   // w(TPL) = y
        const uint32_t o = e == 0 ? cur.w(k) : vw::alignbyte(hi, lo, sh);
        const bool wr = e == 0 ? (k < (int)TPL) : (k == (int)TPL ? l == 63 : (k != 0 || l != 0));
        if (wr) rd[((base + 4u * k) & RMASK) >> 2] = o;   // lane 0's k=0 dword: written by lane 63 before
    }
}

// Prefix phase for chunk c: 0 = no sample yet, 1 = first sample starts in
// this chunk (its tokens still to do), 2 = not the fast shape, 3 (fast
// kernel) = a clean prefix whose genotype tokens are not all 3 bytes long:
// f.gt0 is the first sample's offset, handed to k_encode_var.  VAR (the
// variable-token kernel): the genotype region need only hold odd-length
// tokens (f.T = its 2-byte half-slots instead of its tokens).
template <bool VAR>
__device__ __forceinline__ int fast_prefix_step(const Chunk &cur, uint32_t c, uint32_t lead, uint32_t len,
                                                FastState &f, Ring &r) {
    const uint32_t l = vw::lane_id();
    const uint32_t bo = c * CHUNK + BPL * l;
    const int32_t x0 = (int32_t)bo - (int32_t)lead;   // line offset of the lane's byte 0
    constexpr uint32_t FULLM = (uint32_t)((1ull << BPL) - 1ull);
    // ---- locate the 10th field start, reject empty fields ----
    const int32_t vlo = x0 >= 0 ? 0 : (-x0 >= (int32_t)BPL ? (int32_t)BPL : -x0);
    const int32_t vhi0 = (int32_t)len - x0;
    const int32_t vhi = vhi0 <= 0 ? 0 : (vhi0 >= (int32_t)BPL ? (int32_t)BPL : vhi0);
    const uint32_t vm = vhi > vlo ? (uint32_t)(((1ull << vhi) - 1ull) ^ ((1ull << vlo) - 1ull)) : 0u;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < (int)TPL; k++) m |= zero_bytes4(cur.w(k) ^ 0x09090909u) << (4 * k);
    m &= vm;
    const uint32_t Tm = (m | ~vm) & FULLM;          // TAB or outside the line
    const uint32_t pin = vw::shr1(Tm >> (BPL - 1), f.carryT);
    const uint32_t prevT = ((Tm << 1) | pin) & FULLM;
    const uint32_t fs = ~Tm & prevT & FULLM;        // field starts
    const uint32_t et = m & prevT;                  // TAB closing an empty field
    f.carryT = vw::readlane(Tm >> (BPL - 1), 63);
    const uint32_t cnt = (uint32_t)__builtin_popcount(fs);
    const uint32_t inc = vw::scan_add(cnt);
    const uint32_t exc = inc - cnt;
    const bool has9 = f.nf + exc <= 9 && 9 < f.nf + inc;
    uint32_t x9l = 0;
    if (has9) {
        uint32_t mm = fs;
        for (uint32_t k = f.nf + exc; k < 9; k++) mm &= mm - 1;
        x9l = (uint32_t)(x0 + __builtin_ctz(mm));
    }
    const uint64_t hb = vw::ballot(has9);
    // (a separate variable: a phi of the per-lane value would make x9 -- and
    // gt0, T, phi, every chunk's tf -- look divergent to the compiler)
    uint32_t x9 = 0;
    if (hb) x9 = vw::readlane(x9l, (uint32_t)__builtin_ctzll(hb));
    uint32_t below = ~0u;
    if (hb) {
        const int32_t d = (int32_t)x9 - x0;
        below = d <= 0 ? 0u : d >= (int32_t)BPL ? ~0u : ((1u << d) - 1u);
    }
    // a '\n' in the row (the hop line index's guess went wrong, see
    // VcfcEncodeArgs::nl_check): not the fast shape
    uint32_t lf = 0;
#pragma unroll
    for (int k = 0; k < (int)TPL; k++) lf |= zero_bytes4(cur.w(k) ^ 0x0A0A0A0Au) << (4 * k);
    // the fast shape: in this chunk's genotype bytes the TABs sit exactly at
    // x9 + 4k + 3 -- rows of other token lengths (haploid "0", GT:DP:GQ, '.')
    // leave here, before the genotype phase puts 6 KiB of loads in flight
    bool odd = false;
    if (!VAR && hb) {
        const int32_t rel = x0 - (int32_t)x9;
        const uint32_t ph = (uint32_t)(3 - rel) & 3u;   // lane bytes i with (rel + i) % 4 == 3
        const uint32_t ge = rel >= 0 ? FULLM : (-rel >= (int32_t)BPL ? 0u : (FULLM & ~((1u << -rel) - 1u)));
        odd = ((m ^ ((0x1111u << ph) & FULLM)) & ge & vm) != 0;
    }
    if (vw::ballot((et & below) != 0 || (lf & vm) != 0)) return 2;
    if (!VAR && vw::ballot(odd)) {   // a clean prefix, tokens of another length: k_encode_var's row, gt0 known
        // the first token 5 bytes or longer (no TAB in line bytes x9 + 1 ..
        // x9 + 4, all inside this chunk and the line): VCFCD_GT0_LONG
        const int32_t w0 = (int32_t)x9 + 1 - x0;   // the window's first byte, lane-relative
        const uint32_t win = w0 >= (int32_t)BPL || w0 + 4 <= 0
                                 ? 0u
                                 : ((w0 < 0 ? 0xFu >> -w0 : 0xFu << w0) & FULLM);
        const bool inside = x9 + 5u <= len && (int32_t)x9 + 5 <= (int32_t)((c + 1) * CHUNK) - (int32_t)lead;
        const bool long1 = inside && vw::ballot((m & win) != 0) == 0;
        f.gt0 = (int32_t)(x9 | (long1 ? VCFCD_GT0_LONG : 0u));
        return 3;
    }
    prefix_to_ring(cur, c, lead, r);
    f.nf += vw::readlane(inc, 63);
    if (!hb) {
        const int32_t upto = (int32_t)((c + 1) * CHUNK) - (int32_t)lead;
        r.wpos = 8u + umin32(len, upto <= 0 ? 0u : (uint32_t)upto);
        ring_flush(r, false);
        return 0;   // (if this was the last chunk: < 10 fields -> general path)
    }
    f.gt0 = (int32_t)x9;
    r.wpos = 8u + x9;
    const uint32_t glen = len - x9;
    f.phi = (lead + x9) & 3u;
    if (VAR) {
        // odd-length tokens and single TABs: glen + 1 is even, and every
        // token starts on an even offset from token 0
        if (((glen + 1) & 1u) != 0) return 2;
        f.T = (glen + 1) >> 1;
    } else {
        if (((glen + 1) & 3u) != 0) return 2;
        f.T = (glen + 1) >> 2;
    }
    if (f.T >= (1u << 23) - 2 * MOD_BIAS) return 2;   // mod_cap is exact below 2^23
    return 1;
}

// General genotype step over one 1 KiB half-chunk (4 slots per lane):
// escapes, the row's last token, anything the clean 2 KiB path rejects.
// tf = token index of the half's first slot.  false = not the fast shape.
__device__ bool gt_general(const Chunk &cur, int32_t tf, FastState &f, Ring &r) {
    const uint32_t l = vw::lane_id();
    const uint32_t T = f.T, phi = f.phi;
    constexpr uint32_t Z = 0x09307C30u;   // "0|0\t"
    if (tf >= (int32_t)T) return true;
    uint32_t d[TPL];
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) d[j] = vw::alignbyte(cur.w(j + 1), cur.w(j), phi);
    const int32_t t0 = tf + (int32_t)(TPL * l);
    const uint32_t u0 = (uint32_t)(t0 + 1);
    const uint32_t dummy = RING_DUMMY;   // shared dummy word (see esc8)
    bool v[TPL];
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) v[j] = (uint32_t)(t0 + j) < T;
    uint32_t cl[TPL];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) {
        const bool isc = (d[j] & 0xFFFEFFFEu) == Z;
        cl[j] = !v[j] ? CLS_NONE : isc ? cls_classed(d[j]) : CLS_ESC;
        if (cl[j] == CLS_ESC) {
            // an escape, or the row's last token (no TAB after it): full check
            // (bytes 0..2 masked to 0xFC: 0x08-0x0B, TAB and '\n' among them, reject)
            const uint32_t x = (d[j] ^ 0x09090909u) & 0xFFFCFCFCu;
            const uint32_t zb = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
            const bool last = (uint32_t)(t0 + j) + 1 == T;
            bad |= (zb & 0x00808080u) != 0 || ((zb >> 31) == 0 && !last);
            cl[j] = cls_f(d[j]);
        }
    }
    if (vw::ballot(bad)) return false;
    const uint32_t p0 = vw::shr1(cl[TPL - 1], f.pcls);
    uint32_t lane_rs = 0;
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) {
        const uint32_t pj = j == 0 ? p0 : cl[j - 1];
        const bool s = cl[j] != CLS_NONE && (cl[j] != pj || cl[j] == CLS_ESC);
        if (s) lane_rs = u0 + j;
    }
    const uint32_t rin = vw::umax(vw::shr1z(vw::scan_max(lane_rs)), f.prs);
    uint32_t mp = mod_cap((uint32_t)(t0 + (int32_t)MOD_BIAS) - rin, p0 == 0);
    uint32_t lane_sum = 0, lrs = rin;
    uint32_t e1_m = 0, full_m = 0, b1s[TPL];
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) {
        const uint32_t pj = j == 0 ? p0 : cl[j - 1], cj = cl[j];
        const bool s = cj != CLS_NONE && (cj != pj || cj == CLS_ESC);
        const uint32_t capm1_p = pj == 0 ? 126u : 30u, capm1_c = cj == 0 ? 126u : 30u;
        const bool tab = cj != CLS_NONE && pj == CLS_ESC;
        const bool pend = s && pj < CLS_ESC && mp != capm1_p;
        b1s[j] = tab ? 0x09u : (cls_mask_f(pj) | (mp + 1));
        const uint32_t m = s ? 0u : (mp == capm1_c ? 0u : mp + 1);
        const bool full = cj < CLS_ESC && m == capm1_c;
        e1_m |= ((tab | pend) ? 1u : 0u) << j;
        full_m |= (full ? 1u : 0u) << j;
        lane_sum += ((tab | pend) ? 1u : 0u) + (cj == CLS_ESC ? 4u : (full ? 1u : 0u));
        mp = m;
        if (s) lrs = u0 + j;
    }
    const uint32_t incl = vw::scan_add(lane_sum);
    const uint32_t pos0 = r.wpos + incl - lane_sum;
    uint32_t pos = pos0;
    bool any_esc = false;
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) {
        const bool e1 = (e1_m >> j) & 1u, full = (full_m >> j) & 1u;
        r.lds[e1 ? (pos & RMASK) : dummy] = (uint8_t)b1s[j];
        pos += e1 ? 1u : 0u;
        r.lds[full ? (pos & RMASK) : dummy] = (uint8_t)(cls_mask_f(cl[j]) | (cl[j] == 0 ? 127u : 31u));
        pos += cl[j] == CLS_ESC ? 4u : (full ? 1u : 0u);
        any_esc |= cl[j] == CLS_ESC;
    }
    if (vw::ballot(any_esc)) {
        // escape payloads: walk the lane's tokens again for their positions
        pos = pos0;
#pragma unroll
        for (int j = 0; j < (int)TPL; j++) {
            pos += ((e1_m >> j) & 1u);
            if (cl[j] == CLS_ESC) {
                ring_put(r, pos, 0xE1u);
                ring_put(r, pos + 1, d[j] & 0xFFu);
                ring_put(r, pos + 2, (d[j] >> 8) & 0xFFu);
                ring_put(r, pos + 3, (d[j] >> 16) & 0xFFu);
            }
            pos += cl[j] == CLS_ESC ? 4u : ((full_m >> j) & 1u);
        }
    }
    r.wpos += vw::readlane(incl, 63);
    // carry the chunk's last token (class, run start)
    bool anyv = false;
    uint32_t lc = CLS_NONE;
#pragma unroll
    for (int j = 0; j < (int)TPL; j++) {
        anyv |= v[j];
        if (v[j]) lc = cl[j];
    }
    const uint64_t hv = vw::ballot(anyv);
    if (hv) {
        const uint32_t src = (uint32_t)vw::hibit64(hv);
        f.pcls = vw::readlane(lc, src);
        f.prs = vw::readlane(lrs, src);
    }
    ring_flush(r, false);
    return true;
}


// ---------------------------------------------------------------------------
// Genotype phase: 2 KiB chunks of the genotype region, based at the 4-byte
// word holding token 0 (phase phi), so slot j of lane l is token
// 512 C + 8 l + j and no slot precedes token 0.  Lane l owns bytes
// [32 l, 32 l + 32) plus a 4-byte look-ahead.
constexpr uint32_t TPL8 = 8;
constexpr uint32_t BPL8 = 4 * TPL8;
constexpr uint32_t CHUNK8 = 64 * BPL8;   // 2 KiB
constexpr uint32_t SLOTS8 = 64 * TPL8;   // 512 tokens per chunk

struct Chunk8 {
    uint4 a, b;
    uint32_t y;
    __device__ __forceinline__ uint32_t w(int k) const {
        return k == 0 ? a.x : k == 1 ? a.y : k == 2 ? a.z : k == 3 ? a.w :
               k == 4 ? b.x : k == 5 ? b.y : k == 6 ? b.z : k == 7 ? b.w : y;
    }
};
__device__ __forceinline__ Chunk8 load_chunk8(vw::brsrc rs, uint32_t C, uint32_t lo32) {
    Chunk8 k;
    const uint32_t off = C * CHUNK8 + lo32;   // lo32 = 32 * lane
    k.a = vw::bload16(rs, off, GT_AUX);
    k.b = vw::bload16(rs, off + 16u, GT_AUX);
    k.y = vw::bload4(rs, off + 32u + la_off(lo32, 63 * BPL8), GT_AUX);   // lane 63 only (see load_chunk)
    return k;
}

// class bytes of four classed tokens: byte j = 0x90 + class ("2a + b", no carries)
__device__ __forceinline__ uint32_t class_bytes(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
    const uint32_t q01 = vw::perm(d1, d0, 0x06040200u), q23 = vw::perm(d3, d2, 0x06040200u);
    return (vw::perm(q23, q01, 0x06040200u) << 1) + vw::perm(q23, q01, 0x07050301u);
}
// bytes 0..3 of lo and hi (one flag or value per slot) -> 4-bit stride: slot j at bit 4j
__device__ __forceinline__ uint32_t stride4(uint32_t lo, uint32_t hi) {
    return vw::perm(hi, lo, 0x06040200u) | (vw::perm(hi, lo, 0x07050301u) << 4);
}

// Clean chunk: every slot in [0, T) is "a|b" with a, b in {0,1}.  The lane's
// output is at most: a full-chunk byte of the run entering the lane (run
// offsets reach cap-1 at most once in 8 slots, and only before the lane's
// first start), the pending byte of that run at the first start, and one
// pending byte per further start (runs that begin and end inside the lane
// are shorter than any cap).  The first chunk treats token 0 as continuing a
// virtual run of its own class begun at token 0 (prs = 1): same output as a
// fresh run.  EDGE (last chunk): slots past T-1 take token T-1's class, so
// they continue its run without starting one; their full bytes are masked.
template <bool EDGE>
__device__ __forceinline__ void clean8(const uint32_t (&d)[TPL8], int32_t t0, int32_t tf, FastState &f, Ring &r) {
    uint32_t cbL = class_bytes(d[0], d[1], d[2], d[3]);
    uint32_t cbH = class_bytes(d[4], d[5], d[6], d[7]);
    if (f.pcls == CLS_NONE) {   // first chunk
        f.pcls = vw::readlane(cbL, 0) & 3u;
        f.prs = 1;
    }
    const uint32_t T = f.T;
    if (EDGE) {
        const uint32_t ol = (uint32_t)((int32_t)T - 1 - tf);   // < SLOTS8 (caller)
        const uint32_t cw = vw::readlane((ol & 4u) ? cbH : cbL, ol >> 3);
        const uint32_t cL = (cw >> (8u * (ol & 3u))) & 3u;
        const int32_t nv = (int32_t)T - t0;                      // valid slots in the lane
        const uint32_t fill = 0x90909090u | (cL * 0x01010101u);
        const uint32_t mL = nv >= 4 ? 0u : (nv <= 0 ? ~0u : (~0u << (8 * nv)));
        const uint32_t mH = nv >= 8 ? 0u : (nv <= 4 ? ~0u : (~0u << (8 * (nv - 4))));
        cbL = (cbL & ~mL) | (fill & mL);
        cbH = (cbH & ~mH) | (fill & mH);
    }
    // predecessor class of each slot; slot 0's comes from the previous lane
    const uint32_t pw = vw::shr1(cbH, (0x90u | f.pcls) << 24);
    const uint32_t cpL = vw::alignbyte(cbL, pw, 3), cpH = vw::alignbyte(cbH, cbL, 3);
    const uint32_t xL = cbL ^ cpL, xH = cbH ^ cpH;
    const uint32_t sb = stride4((xL | (xL >> 1)) & 0x01010101u, (xH | (xH >> 1)) & 0x01010101u);   // bit 4j: slot j starts a run
    const uint32_t cp4 = stride4(cpL & 0x03030303u, cpH & 0x03030303u);   // class of slot j-1 at bits 4j
    // run start (+1) of the lane's last start; wave max-scan -> run entering each lane
    const uint32_t lane_rs = sb ? (uint32_t)(t0 + 8) - ((uint32_t)__builtin_clz(sb) >> 2) : 0u;
    const uint32_t incl = vw::scan_max(lane_rs);
    const uint32_t rin = vw::umax(vw::shr1z(incl), f.prs);
    const uint32_t p0 = cpL & 3u;
    const bool is00 = p0 == 0;
    const uint32_t cap = is00 ? 127u : 31u;
    const uint32_t mp = mod_cap((uint32_t)(t0 + (int32_t)MOD_BIAS) - rin, is00);   // offset of slot -1, mod cap
    const uint32_t fb1 = sb ? (uint32_t)__builtin_ctz(sb) : 32u;
    const uint32_t j1 = fb1 >> 2;                              // first start (8: none)
    const uint32_t m0 = vw::perm(0x80C0A000u, 0x80C0A000u, p0);   // low byte: mask of p0's class
    const uint32_t jf = cap - 2u - mp;                         // slot completing a chunk of cap
    bool full = jf < j1;
    if (EDGE) full = full && (uint32_t)(t0 + (int32_t)jf) < T;
    uint32_t rr = mp + j1;
    rr = umin32(rr, rr - cap);                                 // (mp + j1) mod cap (j1 < cap)
    const bool pend = j1 < TPL8 && rr != cap - 1u;
    uint32_t s2 = sb & (sb - 1u);
    const uint32_t n2 = (uint32_t)__builtin_popcount(s2);
    const uint32_t cnt = (full ? 1u : 0u) + (pend ? 1u : 0u) + n2;
    const uint32_t incl2 = vw::scan_add(cnt);
    uint32_t pos = r.wpos + incl2 - cnt;
    if (full) ring_put(r, pos, m0 | cap);
    pos += full ? 1u : 0u;
    if (pend) ring_put(r, pos, m0 | (rr + 1u));
    pos += pend ? 1u : 0u;
    if (vw::ballot(s2 != 0)) {
        // further starts: each closes a run begun at the previous start.  The
        // group's bytes go to base + k (immediate offsets); a group running
        // past the ring end lands in the 64-byte tail and is moved below.
        const uint32_t base = pos & RMASK;
        uint32_t fp = fb1;
#pragma unroll
        for (int k = 0; k < (int)TPL8 - 1; k++) {
            if (k > 0 && !vw::ballot(s2 != 0)) break;
            if (s2 != 0) {
                const uint32_t fk = vw::ffbl(s2);
                const uint32_t cls = (cp4 >> fk) & 3u;
                r.lds[base + k] = (uint8_t)(vw::perm(0x80C0A000u, 0x80C0A000u, cls) | ((fk - fp) >> 2));
                fp = fk;
            }
            s2 &= s2 - 1u;
        }
        ring_unwrap(r, base + n2);
    }
    r.wpos += vw::readlane(incl2, 63);
    f.pcls = (vw::readlane(cbH, 63) >> 24) & 3u;
    f.prs = vw::umax(vw::readlane(incl, 63), f.prs);
    ring_flush(r, false);
}

// classes of four 3-byte tokens (byte j = 0x90 + 2a + b, or 0x94 for an
// escape) and their escape mask (byte j = 0xFF for an escape)
// CHK: also OR into `bad` a 0x80 for every byte 0-2 of a token that is
// 0x08-0x0B (TAB, '\n': not the 3-byte shape; the other two go the general
// way as in shape3) -- exact "some byte is zero" tests on the gathered bytes
template <bool CHK>
__device__ __forceinline__ void esc_classes(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t &cb,
                                            uint32_t &em, uint32_t &bad) {
    const uint32_t g0 = vw::perm(d1, d0, 0x06040200u), g1 = vw::perm(d3, d2, 0x06040200u);
    const uint32_t A = vw::perm(g1, g0, 0x06040200u), B = vw::perm(g1, g0, 0x07050301u);
    const uint32_t S = vw::perm(vw::perm(d3, d2, 0x05010C0Cu), vw::perm(d1, d0, 0x0C0C0501u), 0x07060100u);
    // bytes: nonzero iff the token is not plain
    const uint32_t y = (((A ^ 0x30303030u) | (B ^ 0x30303030u)) & 0xFEFEFEFEu) | (S ^ 0x7C7C7C7Cu);
    const uint32_t n = (((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;   // 0x80 per nonzero byte
    em = (n << 1) - (n >> 7);
    const uint32_t c = (((A & 0x01010101u) << 1) + (B & 0x01010101u)) | 0x90909090u;
    cb = (c & ~em) | (0x94949494u & em);
    if (CHK) {
        auto tabish = [](uint32_t x) {   // 0x80 in some byte iff one is 0x08-0x0B
            const uint32_t t = (x & 0xFCFCFCFCu) ^ 0x08080808u;
            return (t - 0x01010101u) & ~t & 0x80808080u;
        };
        bad |= tabish(A) | tabish(B) | tabish(S);
    }
}

// Escape chunk: every slot in [0, T) is a 3-byte token followed by one TAB
// (the last token by the line end) -- the shape of multi-allelic ("0|2"),
// missing ("./.") and unphased ("0/1") genotypes.  Escapes get class 4 (class
// byte 0x94) and always start a run.  Per lane, in token order: the full-chunk
// byte of the entering run (as clean8), then per start its lead byte -- TAB
// after an escape, else the pending byte of the run it closes (for the first
// start only if that run's last chunk is partial; runs closed by a further
// start are shorter than any cap) -- and, for an escape, 0xE1 + its 3 bytes.
// The incoming class may be an escape (p0 == 4 makes slot 0 a start whose
// lead byte is TAB).  EDGE: slots past T-1 take token T-1's class and are
// masked out of the starts and escapes.
// false (nothing written, no state changed): the chunk is not the escape
// shape (interior chunks: byte 3 of some slot is not TAB, or a token byte is
// 0x08-0x0B -- the caller's general step takes it), or it is chunk 0 of a
// row that f.hand allows to hand on and holds escapes only (f.hand = 2).
// (Round 5: the interior shape test folded into the classification's
// gathered bytes instead of shape3's pass over the slots.)
template <bool EDGE>
__device__ __forceinline__ bool esc8(const uint32_t (&d)[TPL8], int32_t t0, int32_t tf, FastState &f, Ring &r) {
    // per 4 slots: gather bytes 0 (allele a), 2 (allele b) and 1 (separator)
    // of the tokens into one word each; a token is plain ("a|b", a, b in
    // {0,1}) iff a and b are '0'/'1' and the separator is '|'.  Class byte =
    // 0x90 + 2a + b, escapes 0x94; an escape's bytes never reach a neighbour.
    uint32_t cbL, cbH, eL, eH;   // eL/eH: 0xFF in the byte of each escape slot
    uint32_t badL = 0, badH = 0;
    esc_classes<true>(d[0], d[1], d[2], d[3], cbL, eL, badL);
    esc_classes<true>(d[4], d[5], d[6], d[7], cbH, eH, badH);
    if (!EDGE) {
        uint32_t at = 0;   // byte 3 of every slot a TAB
#pragma unroll
        for (int j = 0; j < (int)TPL8; j++) at |= d[j] ^ 0x09090909u;
        if (vw::ballot((badL | badH | (at & 0xFF000000u)) != 0)) return false;
    } else {
        // the row's last chunk: only slots t0 + j < T count (the bytes of the
        // others lie above theirs in each word, so a borrow of theirs cannot
        // reach a valid byte), and the last token has no TAB after it
        const int32_t nv = (int32_t)f.T - t0;   // valid slots in the lane
        const uint32_t vL = nv >= 4 ? 0x80808080u : (nv <= 0 ? 0u : (0x80808080u & ((1u << (8 * nv)) - 1u)));
        const uint32_t vH = nv >= 8 ? 0x80808080u : (nv <= 4 ? 0u : (0x80808080u & ((1u << (8 * (nv - 4))) - 1u)));
        uint32_t at = 0;   // byte 3 of every slot but the last valid one a TAB
#pragma unroll
        for (int j = 0; j < (int)TPL8; j++) at |= (d[j] ^ 0x09090909u) & (j < nv - 1 ? 0xFF000000u : 0u);
        if (vw::ballot(((badL & vL) | (badH & vH) | at) != 0)) return false;
    }
    // Round 5: every token of chunk 0 an escape (unphased "0/1", "./."):
    // records ~1.25x the line, so the row goes to k_encode_var, which sizes
    // it without reading it (VCFCD_GT0_LONG) and has it written straight to
    // out (deferred records) instead of staged and copied
    if (!EDGE && f.hand == 1u && tf == 0 && vw::ballot((eL & eH) != ~0u) == 0) {
        f.hand = 2u;
        return false;
    }
    f.esc = (uint32_t)__builtin_popcountll(vw::ballot((eL | eH) != 0));
    if (f.pcls == CLS_NONE) {   // first chunk: see clean8 (an escape token 0 -> class 0: no lead byte)
        f.pcls = vw::readlane(cbL, 0) & 3u;
        f.prs = 1;
    }
    const uint32_t T = f.T;
    uint32_t vbits = 0x11111111u;   // bit 4j: slot j holds a token
    if (EDGE) {
        const uint32_t ol = (uint32_t)((int32_t)T - 1 - tf);
        const uint32_t cw = vw::readlane((ol & 4u) ? cbH : cbL, ol >> 3);
        const uint32_t cL = (cw >> (8u * (ol & 3u))) & 7u;
        const int32_t nv = (int32_t)T - t0;
        const uint32_t fill = 0x90909090u | (cL * 0x01010101u);
        const uint32_t mL = nv >= 4 ? 0u : (nv <= 0 ? ~0u : (~0u << (8 * nv)));
        const uint32_t mH = nv >= 8 ? 0u : (nv <= 4 ? ~0u : (~0u << (8 * (nv - 4))));
        cbL = (cbL & ~mL) | (fill & mL);
        cbH = (cbH & ~mH) | (fill & mH);
        vbits = nv >= 8 ? 0x11111111u : (nv <= 0 ? 0u : (0x11111111u & ((1u << (4 * nv)) - 1u)));
    }
    const uint32_t pw = vw::shr1(cbH, (0x90u | f.pcls) << 24);
    const uint32_t cpL = vw::alignbyte(cbL, pw, 3), cpH = vw::alignbyte(cbH, cbL, 3);
    const uint32_t xL = cbL ^ cpL, xH = cbH ^ cpH;
    // a start: class differs from the predecessor's (bits 0-2), or an escape (bit 2 of the class byte)
    const uint32_t sL = (xL | (xL >> 1) | (xL >> 2) | (cbL >> 2)) & 0x01010101u;
    const uint32_t sH = (xH | (xH >> 1) | (xH >> 2) | (cbH >> 2)) & 0x01010101u;
    const uint32_t sb = stride4(sL, sH) & vbits;
    const uint32_t eb = stride4((cbL >> 2) & 0x01010101u, (cbH >> 2) & 0x01010101u) & vbits;   // escape slots
    const uint32_t lane_rs = sb ? (uint32_t)(t0 + 8) - ((uint32_t)__builtin_clz(sb) >> 2) : 0u;
    const uint32_t incl = vw::scan_max(lane_rs);
    const uint32_t rin = vw::umax(vw::shr1z(incl), f.prs);
    const uint32_t p0 = cpL & 7u;
    const bool is00 = p0 == 0;
    const uint32_t cap = is00 ? 127u : 31u;
    const uint32_t mp = mod_cap((uint32_t)(t0 + (int32_t)MOD_BIAS) - rin, is00);
    const uint32_t fb1 = sb ? (uint32_t)__builtin_ctz(sb) : 32u;
    const uint32_t j1 = fb1 >> 2;
    const uint32_t m0 = vw::perm(0x80C0A000u, 0x80C0A000u, p0 & 3u);
    const uint32_t jf = cap - 2u - mp;
    bool full = p0 < CLS_ESC && jf < j1;
    if (EDGE) full = full && (uint32_t)(t0 + (int32_t)jf) < T;
    uint32_t rr = mp + j1;
    rr = umin32(rr, rr - cap);
    const bool pesc = p0 == CLS_ESC;
    const bool lead1 = j1 < TPL8 && (pesc || rr != cap - 1u);
    const uint32_t b1 = pesc ? 0x09u : (m0 | (rr + 1u));
    const uint32_t n2 = (uint32_t)__builtin_popcount(sb & (sb - 1u));
    const uint32_t cnt = (full ? 1u : 0u) + (lead1 ? 1u : 0u) + n2 + 4u * (uint32_t)__builtin_popcount(eb);
    const uint32_t incl2 = vw::scan_add(cnt);
    // The lane's bytes go to base + [0, cnt) (cnt <= 41 < RING_TAIL: no
    // masking per byte; bytes past the ring end are moved below).  Stores are
    // unconditional: a byte or escape word the lane does not emit goes to its
    // dummy word, so the slots need no branches; an escape's four bytes
    // (0xE1 and its token) leave as one unaligned ds_write_b32.
    const uint32_t base = (r.wpos + incl2 - cnt) & RMASK;
    uint8_t *const lb = r.lds + base;
    // Stores that emit nothing go to one dummy word shared by the wave:
    // same-address stores add no bank conflict, where a dummy word per lane
    // collides with the real stores of other lanes on the same banks (law 0:
    // 3.09 -> 2.64 ms k_encode in an A/B, profiles/r02/ab/ab_dummy_law0.txt).
    uint8_t *const dm = r.lds + RING_DUMMY;
    *(full ? lb : dm) = (uint8_t)(m0 | cap);
    uint32_t o = full ? 1u : 0u;
    // The first start's lead byte follows the full byte (nothing else comes
    // before the first start: escapes are starts).  Later starts close the
    // run begun at the previous start: lead = mask(class) + length, where the
    // class table gives 0x08 for an escape predecessor, whose run has length
    // 1 (0x09 = TAB).  Per slot: the byte's address is dm + s * (lb + o - dm)
    // (s, e in {0, 1}; one 24-bit multiply-add instead of a compare and a
    // select), and the offsets advance by s and 4 e.
    *(lead1 ? lb + o : dm) = (uint8_t)b1;
    o += lead1 ? 1u : 0u;
    const uint32_t sbr = sb & (sb - 1u);   // starts after the first
    const uint32_t dmi = RING_DUMMY;
    const int32_t ldm = (int32_t)base - (int32_t)dmi;
    const uint32_t mL = vw::perm(0x08u, 0x80C0A000u, cpL & 0x07070707u) + 0x03020100u;   // mask + slot index
    const uint32_t mH = vw::perm(0x08u, 0x80C0A000u, cpH & 0x07070707u) + 0x07060504u;
    int32_t njp = -(int32_t)j1;   // minus the previous start
    // (round 5: the addresses as hand-written v_mad_i32_i24, vw::lds_sel --
    // the compiler had made most of them 64-bit v_mad_u64_u32)
    int32_t ro = ldm + (int32_t)o;
#ifndef VCFC_DIAG_NOESCEMIT   // (diagnostic, wrong output: esc8 without its per-slot stores)
#pragma unroll
    for (int j = 0; j < (int)TPL8; j++) {
        const int32_t s = (int32_t)((sbr >> (4 * j)) & 1u);
        const int32_t e = (int32_t)((eb >> (4 * j)) & 1u);
        const uint32_t b = ((((j < 4) ? mL : mH) >> (8 * (j & 3))) & 0xFFu) + (uint32_t)njp;
        vw::lds_st8<0, false>(vw::lds_sel(r.lds, s, ro, (int32_t)dmi), b);
        ro += s;
        // (round 6: as four byte stores instead, law 0 +3.5 %, missing-./.
        // rows +2.2 %: profiles/r06/ab/ab_r6eb_*.txt)
        const uint32_t pay = (d[j] << 8) | 0xE1u;   // 0xE1, then the token's three bytes
        vw::lds_st32(vw::lds_sel(r.lds, e, ro, (int32_t)dmi), pay);
        ro += 4 * e;
        njp = s ? -j : njp;
    }
#else
    (void)ro; (void)njp; (void)mL; (void)mH; (void)sbr;
#endif
    ring_unwrap(r, base + cnt);
    r.wpos += vw::readlane(incl2, 63);
    f.pcls = (vw::readlane(cbH, 63) >> 24) & 7u;
    f.prs = vw::umax(vw::readlane(incl, 63), f.prs);
    ring_flush(r, false);
    return true;
}

// Genotype chunk C (2 KiB) on the skip / clean / escape paths.  false = not
// handled (nothing written): the chunk needs the general step.
__device__ __forceinline__ bool gt_step8(const Chunk8 &cur, uint32_t C, FastState &f, Ring &r) {
    const uint32_t l = vw::lane_id();
    const uint32_t T = f.T, phi = f.phi;
    constexpr uint32_t Z = 0x09307C30u;   // "0|0\t"
    const int32_t tf = (int32_t)(C * SLOTS8);
    if (tf >= (int32_t)T) return true;
    uint32_t d[TPL8];
    const uint32_t ya = vw::shl1(cur.a.x, cur.y);   // look-ahead dword (see load_chunk)
#pragma unroll
    for (int j = 0; j < (int)TPL8; j++) d[j] = vw::alignbyte(j + 1 == (int)TPL8 ? ya : cur.w(j + 1), cur.w(j), phi);
    const int32_t t0 = tf + (int32_t)(TPL8 * l);
    const bool pclean = f.pcls < CLS_ESC || f.pcls == CLS_NONE;
#ifdef VCFC_DIAG_NOSTEP   // (diagnostic, wrong output: the genotype stream without its step)
    {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < (int)TPL8; j++) x ^= d[j];
        if (x == 0x12345678u) r.lds[RING_DUMMY] = (uint8_t)t0;
        return true;
    }
#endif
    if (tf + (int32_t)SLOTS8 < (int32_t)T) {
        // interior chunk: every slot a token, none of them the last.  After
        // a chunk with escapes the next one most likely has some too (the
        // random_vcf law: ~20 per chunk): test the escape shape alone.
        if (f.esc) {
            return esc8<false>(d, t0, tf, f, r);   // (its own shape test)
        }
        const uint32_t o = ((d[0] ^ Z) | (d[1] ^ Z)) | ((d[2] ^ Z) | (d[3] ^ Z)) |
                           ((d[4] ^ Z) | (d[5] ^ Z)) | ((d[6] ^ Z) | (d[7] ^ Z));
        if (f.pcls == 0 && vw::ballot(o != 0) == 0) {
            // one 0|0 run through the whole chunk: only full 127-chunks
            // complete.  Token t has run offset t + 1 - prs; count the
            // multiples of 127 in [a0 + 1, a0 + 512].
            const uint32_t a0 = (uint32_t)tf + 1 - f.prs;
            const uint32_t kfull = (a0 + SLOTS8) / 127 - a0 / 127;
            if (l < kfull) ring_put(r, r.wpos + l, 0x7Fu);
            r.wpos += kfull;
            ring_flush(r, false);
            return true;
        }
        if (pclean && vw::ballot((o & 0xFFFEFFFEu) != 0) == 0) {
#ifdef VCFC_DIAG_CLEAN_SKIP   // (diagnostic, wrong output: the clean step costs nothing)
            return true;
#endif
            clean8<false>(d, t0, tf, f, r);
            return true;
        }
        return esc8<false>(d, t0, tf, f, r);   // (its own shape test; false: the general step)
    } else {
        // last chunk: slots past T-1 are ignored; token T-1 has no TAB after it
        // (after a chunk with escapes in 4+ lanes the escape shape alone, as in
        // interior chunks: round 5, law 0 pays no clean test on its rows' last
        // chunk; a row with a few escapes most likely ends clean)
        if (f.esc < 4u) {
            bool bad = false;
#pragma unroll
            for (int j = 0; j < (int)TPL8; j++) {
                const int32_t t = t0 + j;
                const uint32_t m = (uint32_t)t < T ? ((uint32_t)t + 1u == T ? 0x00FEFFFEu : 0xFFFEFFFEu) : 0u;
                bad |= ((d[j] ^ Z) & m) != 0;
            }
            if (pclean && vw::ballot(bad) == 0) {
                clean8<true>(d, t0, tf, f, r);
                return true;
            }
        }
        return esc8<true>(d, t0, tf, f, r);   // (its own shape test; false: the general step)
    }
    return false;   // tokens of another length or empty fields: the caller runs gt_general on this chunk
}

// false: not the fast shape; *gt0_hint = the first sample's offset when the
// prefix (in the first 1 KiB) was clean and only the tokens were of another
// shape (k_encode_var then skips the prefix parse), else ~0
__device__ bool encode_fast(const uint8_t *__restrict__ line, uint32_t len, Ring &r, uint32_t *rec_bytes,
                            uint32_t *gt0_hint, bool defer) {
    const uint32_t l = vw::lane_id();
    const uint32_t lead = (uint32_t)(reinterpret_cast<uintptr_t>(line) & 15);
    const uint8_t *A = line - lead;
    const uint32_t span = lead + len;
    *gt0_hint = ~0u;
    if (len == 0) return false;
    const uint32_t nch = (span + CHUNK - 1) / CHUNK;
    const uint32_t lo16 = BPL * l;
    FastState f;
    f.nf = 0; f.carryT = 1; f.gt0 = -1; f.T = 0; f.phi = 0; f.pcls = CLS_NONE; f.prs = 0; f.esc = 0;
    f.hand = 0;
    r.wpos = 8;
    r.fpos = 0;

    // prefix phase: 1 KiB chunks of the line until the first sample starts
    // (loads past the row read 0: no clamping)
    const vw::brsrc rsA = vw::make_rsrc(A, (span + 3u) & ~3u);
    uint32_t c = 0;
    Chunk b = load_chunk(rsA, 0, lo16);
    int st;
    for (;;) {
        st = (int)vw::readfirst((uint32_t)fast_prefix_step<false>(look_ahead(b), c, lead, len, f, r));
        if (st != 0) break;
        c = vw::readfirst(c + 1);
        if (c >= nch) return false;   // < 10 fields
        b = load_chunk(rsA, c, lo16);
    }
    if (st == 3 && c == 0) *gt0_hint = (uint32_t)f.gt0;
    if (st >= 2) return false;

    // genotype phase: runs of clean chunks, three chunks in flight, broken
    // by the (rare) chunks that need the general step.  The inner loop has a
    // single exit (early exits merge into the latch and make hipcc's vmcnt
    // tracking fall back to vmcnt(0)); the general step sits outside it so
    // its registers do not add to the prefetch buffers'.
    const uint32_t phi = f.phi, T = f.T;
    vw::brsrc rsG = vw::make_rsrc(line + f.gt0 - phi, (phi + len - (uint32_t)f.gt0 + 3u) & ~3u);
    const vw::brsrc rsZ = vw::make_rsrc(line, 0u);   // an empty range: loads read 0 and touch no memory
    const uint32_t ncG = (T + SLOTS8 - 1) / SLOTS8;
    const uint32_t lo32 = BPL8 * l;
    f.hand = defer && c == 0 && ncG > 1 ? 1u : 0u;   // (esc8: an all-escape chunk 0 hands the row on)
    uint32_t C0 = 0;
    // three chunks in flight per wave (two: 8 waves/SIMD but +3 % on the
    // headline law, ab_depth_occupancy.txt; four: 5 waves/SIMD, slower,
    // ab_depth4*.txt)
    for (;;) {
        Chunk8 b0 = load_chunk8(rsG, C0, lo32);
        Chunk8 b1 = load_chunk8(rsG, C0 + 1, lo32);
        Chunk8 b2 = load_chunk8(rsG, C0 + 2, lo32);
        vw::pin_loads();
        uint32_t C = C0, gen = C0;
        bool ok = true;
        for (;;) {
            if (ok) { ok = vw::readfirst(gt_step8(b0, C, f, r)); gen = C; }
            // a row handed on at chunk 0 (esc8, f.hand = 2) loads nothing
            // more: the loop's remaining loads go to an empty range (the same
            // instructions, so the counted vmcnt waits stay as they are;
            // unphased rows 7.06 -> 6.63 ms, profiles/r06/ab/ab_r6hn_*.txt)
            rsG = f.hand == 2u ? rsZ : rsG;
            b0 = load_chunk8(rsG, C + 3, lo32);
            vw::pin_loads();
            if (ok && C + 1 < ncG) { ok = vw::readfirst(gt_step8(b1, C + 1, f, r)); gen = C + 1; }
            b1 = load_chunk8(rsG, C + 4, lo32);
            vw::pin_loads();
            if (ok && C + 2 < ncG) { ok = vw::readfirst(gt_step8(b2, C + 2, f, r)); gen = C + 2; }
            b2 = load_chunk8(rsG, C + 5, lo32);
            vw::pin_loads();
            C = vw::readfirst(C + 3);
            if (!ok || C >= ncG) break;
        }
        if (ok) break;
        if (f.hand == 2u) {   // chunk 0 all escapes: k_encode_var's row, to be deferred (esc8)
            *gt0_hint = (uint32_t)f.gt0 | VCFCD_GT0_LONG;
            return false;
        }
        // chunk `gen`: the general step over its two 1 KiB halves
        for (uint32_t h = 0; h < 2; h++) {
            const Chunk hc = look_ahead(load_chunk(rsG, 2 * gen + h, lo16));
            if (!vw::readfirst(gt_general(hc, (int32_t)(gen * SLOTS8 + h * 64 * TPL), f, r))) return false;
        }
        C0 = vw::readfirst(gen + 1);
        if (C0 >= ncG) break;
    }
    const uint32_t pcls = f.pcls, prs = f.prs;
    const int32_t gt0 = f.gt0;
    // row end: pending chunk of the last run, then '\n'
    uint32_t extra = 0, pb = 0;
    if (pcls < CLS_ESC) {
        const uint32_t off = mod_cap(T - prs, pcls == 0);
        if (off != (pcls == 0 ? 126u : 30u)) { extra = 1; pb = cls_mask_f(pcls) | (off + 1); }
    }
    if (l == 0) {
        if (extra) ring_put(r, r.wpos, pb);
        ring_put(r, r.wpos + extra, 0x0Au);
    }
    r.wpos += extra + 1;
    ring_finish(r, (uint32_t)gt0);
    *rec_bytes = r.wpos;
    return true;
}


// ---------------------------------------------------------------------------
// Variable-token path (k_encode_var): rows the fast kernel hands back whose
// genotype tokens all have odd length and are separated by single TABs --
// haploid "0" beside diploid "0|1", "." for missing samples, "0|1:35:99"
// (GT:DP:GQ).  Then every token starts an even number of bytes after token 0,
// so the genotype region is a sequence of 2-byte half-slots: a token is a
// start half and continuation halves up to the half whose second byte is its
// TAB.  One wave streams 2 KiB chunks (lane l: half-slots [16 l, 16 l + 16)),
// three in flight, with fixed-trip per-half work:
//   - TAB masks give the token starts; a start whose 4 bytes read "a|b\t"
//     (a, b in {0,1}) is a plain token of class 2a + b, any other an escape;
//   - classes fill forward to the continuation halves (segmented doubling),
//     so a half's predecessor class is the class of the half before it;
//   - run starts, the entering run (wave max-scan) and its offset mod cap
//     follow esc8's rules over token indices (a wave add-scan of starts);
//   - emission (round 5): the run entering a lane is closed by the lead byte
//     of the lane's first run start; every run that starts and ends inside
//     the lane emits its pending byte at its last half (END).  Per half:
//     [pending byte at an END half | 0xE1 at an escape start][both bytes of
//     an escape half].  An escape's last half carries its trailing TAB, so a
//     start after an escape needs no lead byte (the reference's '\t' after
//     an escape, compress.cpp:181-184, is that TAB); the row's last half
//     drops its second byte (the line end).  The pending byte's value runs
//     along the halves in one register (class mask at the run start, + 1/2
//     per half), and every byte is one ds_write_b8 at dummy + f * offset.
// Rows of other shapes stay flagged for the general path.
constexpr uint32_t HPC = 1024;   // half-slots per 2 KiB chunk

struct VarState : FastState {
    uint32_t ntok;   // tokens started so far
    uint32_t nlc;    // refuse a row holding a '\n' (VcfcEncodeArgs::nl_check: the hop line index guessed its end)
    uint32_t nlhit;  // ... and this one does
    uint32_t defer;  // the row may be deferred (k_encode_var, genotype region over one chunk) ...
    uint32_t sizeonly;   // ... and is: its chunk 0 was an escape chunk, the ring keeps its bytes (RING_SIZE)
};

struct Chunk8v {
    uint4 a, b;
    uint32_t y, y2;   // lane 63: the 8 bytes after the chunk (others: from the next lane by DPP)
};
__device__ __forceinline__ Chunk8v load_chunk8v(vw::brsrc rs, uint32_t C, uint32_t lo32) {
    Chunk8v k;
    const uint32_t off = C * CHUNK8 + lo32;
    const uint32_t la = la_off(lo32, 63 * BPL8);
    k.a = vw::bload16(rs, off, GT_AUX);
    k.b = vw::bload16(rs, off + 16u, GT_AUX);
    k.y = vw::bload4(rs, off + 32u + la, GT_AUX);
    k.y2 = vw::bload4(rs, off + 36u + la, GT_AUX);
    return k;
}

// 4-bit zero-byte mask -> its even bytes (0, 2) / odd bytes (1, 3) as 2 bits
__device__ __forceinline__ uint32_t even2(uint32_t z) { return (z & 1u) | ((z >> 1) & 2u); }
__device__ __forceinline__ uint32_t odd2(uint32_t z) { return ((z >> 1) & 1u) | ((z >> 2) & 2u); }

// Flush in 512-byte granules: a half burst (lanes 0..31) to reach a 1 KiB
// boundary, full bursts, then a half burst, so < 512 bytes stay pending and
// the next chunk (<= 49 bytes per lane, < 3.2 KiB) fits the 4 KiB ring.  No
// burst straddles the staging regions (fpos stays a multiple of 512 and a
// full burst starts on a 1 KiB boundary).
template <bool DYN>
__device__ __forceinline__ void ring_half_burst(Ring &r, uint32_t l) {
    if (l < 32) {
        const uint4 v = *reinterpret_cast<const uint4 *>(r.lds + ((r.fpos + 16u * l) & RMASK));
        ring_stage<DYN>(r, r.fpos + 16u * l, v);
    }
    r.fpos += BURST / 2;
}
template <bool DYN>
__device__ __forceinline__ void ring_flush_var(Ring &r) {
    const uint32_t l = vw::lane_id();
    r.wpos = vw::readfirst(r.wpos);
    r.fpos = vw::readfirst(r.fpos);
    vw::wave_sync();
    if ((r.fpos & (BURST / 2)) && r.wpos - r.fpos >= BURST / 2) ring_half_burst<DYN>(r, l);
    if (r.wpos - r.fpos >= BURST) {
        ring_burst<DYN>(r, l);
        if (r.wpos - r.fpos >= BURST) {
            ring_burst<DYN>(r, l);
            if (r.wpos - r.fpos >= BURST) ring_burst<DYN>(r, l);
        }
    }
    if (r.wpos - r.fpos >= BURST / 2) ring_half_burst<DYN>(r, l);
    vw::wave_sync();
}

// Variable-token path modes: VAR_PLAIN (the default encode: every record
// staged), VAR_DEFER (k_encode_var with deferred records enabled: a row may
// switch its ring to RING_SIZE), VAR_DIRECT (k_encode_defer: the ring writes
// the record into out).  Plain builds none of the mode checks.
constexpr int VAR_PLAIN = 0, VAR_DEFER = 1, VAR_DIRECT = 2;

// One 2 KiB chunk C of a variable-token row.  false: not this shape (the
// row takes the general path; nothing of it is kept).
template <int VM>
__device__ __forceinline__ bool gt_var8(const Chunk8v &cur, uint32_t C, VarState &f, Ring &r) {
    const uint32_t l = vw::lane_id();
    const uint32_t NH = f.T, phi = f.phi;
    // dwords realigned to token 0: d[j] = token-relative bytes [2048 C + 32 l + 4 j, +4); d[8] the next lane's first
    const uint32_t ya = vw::shl1(cur.a.x, cur.y), yb = vw::shl1(cur.a.y, cur.y2);
    const uint32_t w[10] = {cur.a.x, cur.a.y, cur.a.z, cur.a.w, cur.b.x, cur.b.y, cur.b.z, cur.b.w, ya, yb};
    uint32_t d[9];
#pragma unroll
    for (int j = 0; j < 9; j++) d[j] = vw::alignbyte(w[j + 1], w[j], phi);
    const int32_t lastrel = (int32_t)NH - 1 - (int32_t)(C * HPC + 16u * l);   // the row's last half, lane-relative
    const uint32_t vm = lastrel >= 15 ? 0xFFFFu : lastrel < 0 ? 0u : (2u << lastrel) - 1u;   // valid halves
    if (f.nlc) {
        // a '\n' among the row's genotype bytes (token-relative offsets below
        // 2 NH - 1; past them lie the line's own '\n' and the next line): the
        // hop line index merged two lines.  haszero per dword is exact here:
        // a borrow only runs upwards, from a '\n' inside the row.
        const int32_t rel0 = (int32_t)(2u * NH - 1u) - (int32_t)(C * CHUNK8 + 32u * l);
        uint32_t z = 0;
        if ((C + 1u) * CHUNK8 <= 2u * NH - 1u) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t x = d[j] ^ 0x0A0A0A0Au;
                z |= (x - 0x01010101u) & ~x;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t x = d[j] ^ 0x0A0A0A0Au;
                const int32_t k = rel0 - 4 * j;
                const uint32_t vb = k >= 4 ? 0x80808080u : k <= 0 ? 0u : (0x80808080u & ((1u << (8 * k)) - 1u));
                z |= (x - 0x01010101u) & ~x & vb;
            }
        }
        if (vw::ballot((z & 0x80808080u) != 0)) {
            f.nlhit = 1;
            return false;
        }
    }
    // TAB masks over halves 0..17: tb0 = first byte TAB (never valid), tb1 = second byte TAB (a token's end);
    // plain 3-byte candidates: bytes "a|b" from the half, a, b in {0,1}; a, b bits
    // (SWAR over the halves' first bytes A and second bytes P, four halves a
    // word: half 4k + i is byte i of A[k] / P[k])
    // (round 5: 0x80 in each TAB byte of a dword, then the flags of its
    // first bytes (0, 2: halves 2j, 2j + 1) and of its second bytes (1, 3)
    // weighted into the masks by v_dot4_u32_u8 -- byte weights up to 128, so
    // two accumulators of eight halves each)
    auto tabz = [](uint32_t x) {
        const uint32_t w = x ^ 0x09090909u;
        return ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
    };
    uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t z = tabz(d[j]);
        const uint32_t wf = (1u << (2 * (j & 3))) | (2u << (2 * (j & 3) + 16));   // bytes 0, 2
        const uint32_t ws = wf << 8;                                              // bytes 1, 3
        if (j < 4) {
            a0 = vw::dot4u(z, wf, a0);
            a1 = vw::dot4u(z, ws, a1);
        } else {
            b0 = vw::dot4u(z, wf, b0);
            b1 = vw::dot4u(z, ws, b1);
        }
    }
    const uint32_t z8 = tabz(d[8]);   // halves 16, 17
    uint32_t tb0 = (a0 >> 7) | ((b0 >> 7) << 8) | ((vw::dot4u(z8, 0x00020001u, 0u) >> 7) << 16);
    uint32_t tb1 = (a1 >> 7) | ((b1 >> 7) << 8) | ((vw::dot4u(z8, 0x02000100u, 0u) >> 7) << 16);
    if (lastrel >= 0 && lastrel <= 17) tb1 |= 1u << lastrel;   // the row's last half ends its token (line end)
    if (vw::ballot((tb0 & vm) != 0)) return false;           // an empty field, or a token of even length
    // token starts: after a half whose second byte is a TAB (lane 0: the chunk carry)
    const uint32_t pin = vw::shr1((tb1 >> 15) & 1u, f.carryT);
    const uint32_t S = ((tb1 << 1) | pin) & vm;
    const uint32_t L3 = S & ~tb1 & (tb1 >> 1);                 // 3-byte tokens (plain or not)
    const uint32_t nt = (uint32_t)__builtin_popcount(S);
    const uint32_t tinc = vw::scan_add(nt);
    // Escape chunk: the token entering the chunk is an escape (or this is
    // token 0: no lead byte) and every token of the chunk is an escape -- no
    // 3-byte token starts here (1-byte tokens, 5 and more: GT:DP:GQ), or,
    // found after the classification below, none of its 3-byte tokens is
    // plain (unphased "0/1", "./." beside haploid or GT:DP:GQ tokens).  Every half then belongs to an escape: each emits
    // its bytes, a start 0xE1 first -- the input with 0xE1 before every token.
    const bool pesc = f.pcls == CLS_ESC || f.pcls == CLS_NONE;
    auto esc_chunk = [&]() {
        const bool lastin = lastrel >= 0 && lastrel < 16;
        const uint32_t cnt = nt + 2u * (uint32_t)__builtin_popcount(vm) - (lastin ? 1u : 0u);
        const uint32_t incl2 = vw::scan_add(cnt);
        const uint32_t base = (r.wpos + incl2 - cnt) & RMASK;
        // byte stores (unaligned dword stores from every lane wait ~100x
        // longer to issue: SQ_WAIT_INST_LDS, profiles/r03/pmc/pmc_var_kind1*;
        // packed aligned dwords cost more VALU than they save, ab_var_packer.txt),
        // addressed as in the mixed step below
        const int32_t dmi = (int32_t)RING_DUMMY;
        int32_t ro = (int32_t)base - dmi;
        // A row whose first chunk is all escapes (GT:DP:GQ, records about
        // 1.1x the input) is deferred: sized here, its record written
        // straight to out by k_encode_defer once the size scan has placed it,
        // instead of staged and copied (deferred records).
        if (VM == VAR_DEFER && f.defer && C == 0) {
            f.sizeonly = 1;
            r.mode = RING_SIZE;
        }
#ifndef VCFC_VAR_SIZE_ONLY   // (diagnostic: the cost of a size-only pass, wrong output)
        if (VM == VAR_DEFER && f.sizeonly) {
        } else if (vw::ballot(vm != 0xFFFFu) == 0) {
            // Interior chunk (every half valid; the row's last half can only be
            // lane 63's half 15, when the region is a whole number of chunks:
            // its second byte, the line end, is then stored at a + 31, the
            // row end's own slot, which cnt leaves out and lane 0's row-end
            // ring_put rewrites -- test_escape_rows_ending_on_a_chunk_end): half h's
            // two bytes sit at lane offset 2h + c_h, c_h = starts in halves
            // 0..h, and its 0xE1 (a start) just before them.  Half h's 0xE1
            // store is issued before half h-1's second byte: when h starts
            // nothing that is exactly where it lands, so the byte store after
            // it rewrites it (same lane, later instruction) -- no per-store
            // dummy select; half 0's goes to the dummy word unless it is a
            // start (its slot would be the previous lane's last byte).  The
            // bytes come straight from the dwords (ds_write_b8 / _d16_hi):
            // ~3 VALU per half instead of ~10.
            uint32_t a = base;   // base + c_{h-1}
            r.lds[(S & 1u) ? base : RING_DUMMY] = (uint8_t)0xE1u;
            a += S & 1u;
            r.lds[a] = (uint8_t)d[0];
            uint32_t hi8 = d[0] >> 8;
#pragma unroll
            for (int h = 1; h < 16; h++) {
                const uint32_t an = a + ((S >> h) & 1u);
                r.lds[an + 2u * h - 1u] = (uint8_t)0xE1u;
                r.lds[a + 2u * h - 1u] = (uint8_t)((h & 1) ? hi8 : (hi8 >> 16));   // half h-1's second byte
                r.lds[an + 2u * h] = (uint8_t)((h & 1) ? (d[h >> 1] >> 16) : d[h >> 1]);
                if (!(h & 1)) hi8 = d[h >> 1] >> 8;
                a = an;
            }
            r.lds[a + 31u] = (uint8_t)(hi8 >> 16);   // half 15's second byte
        } else {
        // (the row's last half: its second byte, the line end, goes to the
        // row end's own slot, which lane 0 rewrites; see the mixed step)
#pragma unroll
        for (int h = 0; h < 16; h++) {
            const int32_t es = (int32_t)((S >> h) & 1u);
            const int32_t e1 = (int32_t)((vm >> h) & 1u);
            const uint32_t w = d[h >> 1], wh = w >> 8;
            vw::lds_st8<0, false>(vw::lds_sel(r.lds, es, ro, dmi), 0xE1u);
            ro += es;
            const vw::ldsp pa = vw::lds_sel(r.lds, e1, ro, dmi);
            if (h & 1) {
                vw::lds_st8<0, true>(pa, w);
                vw::lds_st8<1, true>(pa, wh);
            } else {
                vw::lds_st8<0, false>(pa, w);
                vw::lds_st8<1, false>(pa, wh);
            }
            ro += 2 * e1;
        }
        }
#endif
        ring_unwrap(r, base + cnt);
        r.wpos += vw::readlane(incl2, 63);
        const uint32_t tot = vw::readlane(tinc, 63);
        f.ntok += tot;
        if (tot) f.prs = f.ntok;   // every escape starts a run: the last token's
        f.pcls = CLS_ESC;
        f.carryT = vw::readlane((tb1 >> 15) & 1u, 63);
        ring_flush_var<VM != VAR_PLAIN>(r);
    };
    if (pesc && vw::ballot(L3 != 0) == 0) {
        esc_chunk();
        return true;
    }
    // plain 3-byte candidates: bytes "a|b" from the half, a, b in {0,1}; a, b bits
    // (SWAR, four halves a word: A = first bytes, P = second bytes, B = the
    // byte after each half, i.e. the next half's first; bit 0 of the bytes
    // of A / B gathered by one multiply)
    uint32_t p3 = 0, am = 0, bm = 0;
    // bit 0 of each byte gathered by one v_dot4_u32_u8 (not a v_mul_lo_u32)
    auto bits0 = [](uint32_t x) { return vw::dot4u(x & 0x01010101u, 0x08040201u, 0u); };
    uint32_t Y[4];   // per half of word k (byte i: half 4k + i): 2a + b, the class index of a plain start
    uint32_t An = vw::perm(d[1], d[0], 0x06040200u);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t A = An;
        An = k < 3 ? vw::perm(d[2 * k + 3], d[2 * k + 2], 0x06040200u) : d[8];   // (byte 0 of d[8]: half 16's first)
        const uint32_t P = vw::perm(d[2 * k + 1], d[2 * k], 0x07050301u);
        const uint32_t B = vw::alignbyte(An, A, 1);
        const uint32_t y = (((A ^ 0x30303030u) | (B ^ 0x30303030u)) & 0xFEFEFEFEu) | (P ^ 0x7C7C7C7Cu);
        p3 |= zero_bytes4(y) << (4 * k);
        am |= bits0(A) << (4 * k);
        bm |= bits0(B) << (4 * k);
        Y[k] = ((A & 0x01010101u) << 1) | (B & 0x01010101u);
    }
    const uint32_t PL = S & p3 & ~tb1 & (tb1 >> 1);           // plain: exactly 3 bytes "a|b"
    if (pesc && vw::ballot(PL != 0) == 0) {   // no plain token: the escape chunk (above)
        esc_chunk();
        return true;
    }
    // tokens longer than 3 bytes beside 3-byte ones (or after a plain token)
    // are left to the general path
    if (vw::ballot((S & ~tb1 & ~(tb1 >> 1)) != 0)) return false;
    const uint32_t X0 = PL & bm, X1 = PL & am, XE = S & ~PL;  // class bits at the starts (bit 2: escape)
    if (f.pcls == CLS_NONE) {
        // first chunk: token 0 continues a virtual run of its own class begun at token 0 (see clean8)
        f.pcls = vw::readlane(((X1 & 1u) << 1) | (X0 & 1u), 0);
        f.prs = 1;
    }
    // class entering the lane: that of the last start in an earlier lane, else the chunk carry
    const uint32_t hs = S ? 31u - (uint32_t)__builtin_clz(S) : 0u;
    const uint32_t lastc = (((XE >> hs) & 1u) << 2) | (((X1 >> hs) & 1u) << 1) | ((X0 >> hs) & 1u);
    const uint32_t pek = vw::shr1z(vw::scan_max(S ? ((l + 1u) << 3) | lastc : 0u));
    const uint32_t cin = pek ? (pek & 7u) : f.pcls;
    // fill each start's class forward over its continuation halves: adding
    // M << 1 to the non-start mask T carries through each run of T after a
    // start in M and stops at the next start, so T & ((T + (M << 1)) ^ T)
    // is those runs (starts of other masks split the carries)
    const uint32_t T = ~S & 0xFFFFu;
    auto fill = [T](uint32_t m) { return (m | (T & ((T + (m << 1)) ^ T))) & 0xFFFFu; };
    uint32_t c0 = fill(X0), c1 = fill(X1), ce = fill(XE);
    const uint32_t pre = S ? (S & (0u - S)) - 1u : 0xFFFFu;   // halves before the lane's first start: the entering token's
    c0 = (c0 | ((cin & 1u) ? pre : 0u)) & 0xFFFFu;
    c1 = (c1 | ((cin & 2u) ? pre : 0u)) & 0xFFFFu;
    ce = (ce | ((cin & 4u) ? pre : 0u)) & 0xFFFFu;
    // predecessor class of each half (half 0: the entering class)
    const uint32_t q0 = (c0 << 1) | (cin & 1u), q1 = (c1 << 1) | ((cin >> 1) & 1u), qe = (ce << 1) | ((cin >> 2) & 1u);
    const uint32_t RS = S & ((c0 ^ q0) | (c1 ^ q1) | (ce ^ qe) | ce);   // run starts (escapes always)
    const uint32_t EH = ce & vm;                                         // halves of escape tokens
    // token indices, the run entering the lane and its offset mod cap
    const uint32_t t0 = f.ntok + tinc - nt;
    const uint32_t hr = RS ? 31u - (uint32_t)__builtin_clz(RS) : 0u;
    const uint32_t lane_rs = RS ? t0 + (uint32_t)__builtin_popcount(S & ((1u << hr) - 1u)) + 1u : 0u;
    const uint32_t incl = vw::scan_max(lane_rs);
    const uint32_t rin = vw::umax(vw::shr1z(incl), f.prs);
    const bool is00 = cin == 0;
    const uint32_t cap = is00 ? 127u : 31u;
    const uint32_t mp = mod_cap((t0 + MOD_BIAS) - rin, is00);   // offset of token t0 - 1 in its run, mod cap
    const uint32_t lr = RS ? (uint32_t)__builtin_ctz(RS) : 16u;  // the first run start
    const uint32_t j1 = RS ? (uint32_t)__builtin_popcount(S & ((1u << lr) - 1u)) : nt;
    const uint32_t jf = cap - 2u - mp;                           // token completing a chunk of cap
    const bool full = cin < CLS_ESC && jf < j1;
    uint32_t rr = mp + j1;
    rr = umin32(rr, rr - cap);
    const bool lead1 = j1 < nt && cin < CLS_ESC && rr != cap - 1u;
    const uint32_t b1v = cls_mask_f(cin) | (rr + 1u);
    // Emission.  The run entering the lane is closed by b1v, the lead byte
    // of the lane's first run start (lr), as before.  Every run that starts
    // in the lane at or after lr and ends in it -- its next token, a run
    // start, lies at most at half 15 -- emits its pending byte at its last
    // half (END: the second half of its last token; runs inside a lane are
    // shorter than any cap, so the byte always exists).  The output is then
    // per half [lead][p0 p1]: lead = the pending byte at an END half or 0xE1
    // at an escape start (LX), p0 p1 the two bytes of an escape half (EH; the
    // row's last half has only p0, its p1 lands on the row end's slot, which
    // lane 0 rewrites).  Output order is the reference's: a pending byte, a
    // TAB after an escape (its half's p1), 0xE1 and raw bytes.
    const uint32_t lrbit = RS & (0u - RS);
    const uint32_t END = (RS >> 1) & ~S & ~ce & vm & (0u - (lrbit << 1));   // (lrbit 0: none)
    const uint32_t LX = END | XE;
    const bool lastin = lastrel >= 0 && lastrel < 16 && ((EH >> lastrel) & 1u);
    const uint32_t cnt = (full ? 1u : 0u) + (lead1 ? 1u : 0u) + (uint32_t)__builtin_popcount(LX) +
                         2u * (uint32_t)__builtin_popcount(EH) - (lastin ? 1u : 0u);
    const uint32_t incl2 = vw::scan_add(cnt);
    const uint32_t base = (r.wpos + incl2 - cnt) & RMASK;
    // A byte goes to dummy + f * (base + o - dummy) (f in {0, 1}: one
    // v_mad_i32_i24); the stores that emit nothing land on the shared dummy
    // word.  The lead value runs along the halves in byte 2 of lv:
    // lv = (mask << 16) + 0x8000 at a run start (mask = the run's class mask,
    // 0xE1 for an escape) and + 0x8000 per half after it, so at a run's last
    // half byte 2 holds mask | its length in tokens (two halves a token).
    const int32_t dmi = (int32_t)RING_DUMMY;
    int32_t ro = (int32_t)base - dmi;           // base + o - dummy
#ifndef VCFC_VAR_SIZE_ONLY
    if (full) r.lds[base] = (uint8_t)(cls_mask_f(cin) | cap);
    r.lds[(uint32_t)vw::mad24(lead1 ? 1 : 0, ro + (full ? 1 : 0), dmi)] = (uint8_t)b1v;
    ro += (full ? 1 : 0) + (lead1 ? 1 : 0);
    // class masks of the run starts, byte i of MW[k] for half 4k + i: plain
    // 2a + b -> 0x00 0xA0 0xC0 0x80, escape (index 4..7) -> 0xE1
    uint32_t MW[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t xs = vw::umul24((XE >> (4 * k)) & 0xFu, 0x00204081u) & 0x01010101u;   // XE bits -> bytes
        MW[k] = vw::perm(0xE1E1E1E1u, 0x80C0A000u, Y[k] | (xs << 2));
    }
    uint32_t lv = 0;
#pragma unroll
    for (int h = 0; h < 16; h++) {
        // (mask << 16) | 0x8000: byte h & 3 of MW to byte 2, 0x80 to byte 1
        const uint32_t m3 = vw::perm(MW[h >> 2], 0x00008000u, 0x0C04010Cu + ((uint32_t)(h & 3) << 16));
        lv = vw::bfi((uint32_t)vw::sbit(RS, h), m3, lv + 0x8000u);
        const int32_t fl = (int32_t)((LX >> h) & 1u), fe = (int32_t)((EH >> h) & 1u);
        const uint32_t w = d[h >> 1], wh = w >> 8;
        vw::lds_st8<0, true>(vw::lds_sel(r.lds, fl, ro, dmi), lv);   // byte 2
        ro += fl;
        const vw::ldsp pa = vw::lds_sel(r.lds, fe, ro, dmi);
        if (h & 1) {
            vw::lds_st8<0, true>(pa, w);
            vw::lds_st8<1, true>(pa, wh);
        } else {
            vw::lds_st8<0, false>(pa, w);
            vw::lds_st8<1, false>(pa, wh);
        }
        ro += 2 * fe;
    }
#endif
    ring_unwrap(r, base + cnt);
    r.wpos += vw::readlane(incl2, 63);
    f.ntok += vw::readlane(tinc, 63);
    // carries: the class of the chunk's last valid half, whether it ended a token, the last run start
    const uint32_t hl = lastrel >= 15 ? 15u : lastrel < 0 ? 0u : (uint32_t)lastrel;
    const uint32_t lcls = (((ce >> hl) & 1u) << 2) | (((c1 >> hl) & 1u) << 1) | ((c0 >> hl) & 1u);
    const uint64_t endl = vw::ballot(lastrel >= 0 && lastrel < 16);
    const uint32_t src = endl ? (uint32_t)__builtin_ctzll(endl) : 63u;
    f.pcls = vw::readlane(lcls, src);
    f.carryT = vw::readlane((tb1 >> 15) & 1u, 63);
    f.prs = vw::umax(vw::readlane(incl, 63), f.prs);
    ring_flush_var<VM != VAR_PLAIN>(r);
    return true;
}

// The chunk loop of a variable-token row from chunk C on: x, y, z hold
// chunks C, C + 1, C + 2 (three in flight, a single loop exit, see
// encode_fast).  false: not this shape.
template <int VM>
__device__ __forceinline__ bool var_chunks(Chunk8v &x, Chunk8v &y, Chunk8v &z, uint32_t C, uint32_t ncG,
                                           vw::brsrc rsG, uint32_t lo32, VarState &f, Ring &r, bool may_predict) {
    bool ok = true;
    for (;;) {
        ok = vw::readfirst(gt_var8<VM>(x, C, f, r));
        // a deferred row sized by prediction (VAR_DEFER): nothing after chunk 0
        if (VM == VAR_DEFER && may_predict && f.sizeonly) break;
        x = load_chunk8v(rsG, C + 3, lo32);
        vw::pin_loads();
        if (ok && C + 1 < ncG) ok = vw::readfirst(gt_var8<VM>(y, C + 1, f, r));
        y = load_chunk8v(rsG, C + 4, lo32);
        vw::pin_loads();
        if (ok && C + 2 < ncG) ok = vw::readfirst(gt_var8<VM>(z, C + 2, f, r));
        z = load_chunk8v(rsG, C + 5, lo32);
        vw::pin_loads();
        C = vw::readfirst(C + 3);
        if (!ok || C >= ncG) break;
    }
    return ok;
}

// k_encode_var with deferred records (VAR_DEFER) decides a row's fate on its
// first genotype chunk (deferred when it is an escape chunk and more chunks
// follow).  (A copy of the chunk loop per fate, so that staged rows would
// run the default kernel's code, spilled 156 bytes per lane.)  *deferred:
// the row was only sized (RING_SIZE), the ring's bytes never left it.
// gt0_hint (< VCFCD_GT0_NONE): the first sample's offset, found by
// k_encode_fast in a clean prefix inside the line's first 1 KiB -- the
// prefix is then copied without its parse, and the genotype chunks load
// beside it instead of after it (one memory latency fewer per row).
// ntok_ref (VAR_DEFER; 0: none): the token count of the wave's earlier rows.
// A row deferred on its first chunk is then not read further: its record is
// predicted as all escapes -- 8 + len + 1 + ntok_ref bytes (each token gains
// 0xE1, the line its '\n') -- and k_encode_defer's first pass, which encodes
// it in full, checks the prediction (*predicted).  *ntok: the row's token
// count (rows encoded in full).
template <int VM>
__device__ __forceinline__ bool encode_var(const uint8_t *__restrict__ line, uint32_t len, Ring &r, uint32_t *rec_bytes, bool nlc,
                           bool *nlhit, bool *deferred, uint32_t gt0_hint, uint32_t ntok_ref = 0,
                           bool *predicted = nullptr, uint32_t *ntok = nullptr) {
    const uint32_t l = vw::lane_id();
    const uint32_t lead = (uint32_t)(reinterpret_cast<uintptr_t>(line) & 15);
    const uint8_t *A = line - lead;
    const uint32_t span = lead + len;
    if (len == 0) return false;
    const uint32_t nch = (span + CHUNK - 1) / CHUNK;
    const uint32_t lo16 = BPL * l;
    VarState f;
    f.nf = 0; f.carryT = 1; f.gt0 = -1; f.T = 0; f.phi = 0; f.pcls = CLS_NONE; f.prs = 0; f.esc = 0; f.hand = 0; f.ntok = 0;
    f.nlc = nlc ? 1u : 0u; f.nlhit = 0; f.defer = 0; f.sizeonly = 0;
    *nlhit = false;
    *deferred = false;
    if (predicted) *predicted = false;
    r.wpos = 8;
    r.fpos = 0;
    const vw::brsrc rsA = vw::make_rsrc(A, (span + 3u) & ~3u);
    uint32_t c = 0;
    const bool long1 = gt0_hint < VCFCD_GT0_NONE && (gt0_hint & VCFCD_GT0_LONG) != 0;
    if (gt0_hint < VCFCD_GT0_NONE) gt0_hint &= ~VCFCD_GT0_LONG;
    const bool known = gt0_hint < VCFCD_GT0_NONE && gt0_hint < len;
    // A deferred row's size predicted before any load: it starts with
    // escapes (k_encode_fast's VCFCD_GT0_LONG: a first token of 5+ bytes, or
    // a first 2 KiB chunk of 3-byte escapes only), the genotype region spans
    // more than one chunk and has odd-length tokens' parity.
    // (k_encode_defer<1> checks it as it writes the record.)
    if (VM == VAR_DEFER && known && long1 && ntok_ref != 0 && ntok_ref <= (len + 1) / 2) {
        const uint32_t glen = len - gt0_hint;
        const uint32_t nh = (glen + 1) >> 1;
        if (((glen + 1) & 1u) == 0 && nh < (1u << 23) - 2 * MOD_BIAS && (nh + HPC - 1) / HPC > 1) {
            *rec_bytes = len + 9u + ntok_ref;
            *deferred = true;
            *predicted = true;
            return true;
        }
    }
    Chunk b = load_chunk(rsA, 0, lo16);
    if (!known) {
        // prefix phase: as encode_fast
        int st;
        for (;;) {
            st = (int)vw::readfirst((uint32_t)fast_prefix_step<true>(look_ahead(b), c, lead, len, f, r));
            if (st != 0) break;
            c = vw::readfirst(c + 1);
            if (c >= nch) return false;
            b = load_chunk(rsA, c, lo16);
        }
        if (st == 2) return false;
    } else {
        // (fast_prefix_step<true>'s genotype-region checks on the known gt0)
        f.gt0 = (int32_t)gt0_hint;
        f.phi = (lead + gt0_hint) & 3u;
        const uint32_t glen = len - gt0_hint;
        if (((glen + 1) & 1u) != 0) return false;
        f.T = (glen + 1) >> 1;
        if (f.T >= (1u << 23) - 2 * MOD_BIAS) return false;
    }
    f.carryT = 1;   // token 0 starts the genotype region
    const uint32_t phi = f.phi, NH = f.T;
    const vw::brsrc rsG = vw::make_rsrc(line + f.gt0 - phi, (phi + len - (uint32_t)f.gt0 + 3u) & ~3u);
    const uint32_t ncG = (NH + HPC - 1) / HPC;
    f.defer = VM == VAR_DEFER && ncG > 1 ? 1u : 0u;
    const uint32_t lo32 = BPL8 * l;
    Chunk8v b0 = load_chunk8v(rsG, 0, lo32);
    Chunk8v b1 = load_chunk8v(rsG, 1, lo32);
    Chunk8v b2 = load_chunk8v(rsG, 2, lo32);
    vw::pin_loads();
    // The prefix bytes while the genotype chunks are in flight: with gt0
    // known, chunk 0 (loaded first) is copied here; without, the prefix
    // step wrote them and this rewrites chunk c's the same (unconditional,
    // so the loop is entered from one path: a branch here made hipcc's
    // counted vmcnt waits in the chunk loop fall back to vmcnt(0) and the
    // variable-token rows 9-12 % slower)
    prefix_to_ring(look_ahead(b), c, lead, r);
    r.wpos = 8u + (uint32_t)f.gt0;
    ring_flush_var<VM != VAR_PLAIN>(r);   // < 512 bytes pending before the first chunk
    // (an all-escape row of ntok tokens has len >= 2 ntok - 1: a larger
    // count cannot be its own, and the predicted record stays within the
    // per-row bound len + len / 2 + 16 that out_cap is sized by)
    const bool may_predict = VM == VAR_DEFER && ntok_ref != 0 && ntok_ref <= (len + 1) / 2;
    const bool ok = var_chunks<VM>(b0, b1, b2, 0, ncG, rsG, lo32, f, r, may_predict);
    if (!ok) {
        *nlhit = f.nlhit != 0;
        return false;
    }
    if (VM == VAR_DEFER && may_predict && f.sizeonly) {
        *rec_bytes = len + 9u + ntok_ref;
        *deferred = true;
        *predicted = true;
        return true;
    }
    // row end: pending chunk of the last run, then '\n'
    const uint32_t T = f.ntok, pcls = f.pcls, prs = f.prs;
    uint32_t extra = 0, pb = 0;
    if (pcls < CLS_ESC) {
        const uint32_t off = mod_cap(T - prs, pcls == 0);
        if (off != (pcls == 0 ? 126u : 30u)) { extra = 1; pb = cls_mask_f(pcls) | (off + 1); }
    }
    if (l == 0) {
        if (extra) ring_put(r, r.wpos, pb);
        ring_put(r, r.wpos + extra, 0x0Au);
    }
    r.wpos += extra + 1;
    ring_flush_var<VM != VAR_PLAIN>(r);   // (< 512 pending: the final partial burst stays inside one staging region)
    ring_finish<VM != VAR_PLAIN>(r, (uint32_t)f.gt0);
    *rec_bytes = r.wpos;
    *deferred = VM == VAR_DEFER && f.sizeonly != 0;
    if (ntok) *ntok = f.ntok;
    return true;
}


// General path: any line (empty fields anywhere, 9-column rows, tokens of any
// length, CR, the reference's error cases: < 8 fields VcfValidationError, 8
// fields abort).  1 KiB chunks, 16 bytes per lane (+ a 4-byte look-ahead),
// SWAR masks per lane:
//   T   TAB or outside the line;  fs = field starts (non-T after T);
//   the wave add-scan of |fs| numbers the fields; fields 0..8 are the prefix
//   (copied, one TAB before each of fields 1..9), fields >= 9 are tokens.
// Tokens are classed one per loop step (<= 8 per lane: each needs a T before
// it) into a 4-bit-stride class word, then run starts, the entering run
// (max-scan) and its offset mod cap follow esc8's rules.  Every input byte
// emits [lead][mid][raw]: lead = TAB before fields 1..9 or a token's run-end
// byte / TAB after an escape; mid = 0xE1 (escape) or a full-run byte; raw =
// a prefix byte or any byte of an escape token.  The raw bytes go to the
// ring in one pass over the lane's 16 bytes (one ds_write_b8 each, a dummy
// byte when there is none), the lead / mid bytes in a second pass over the
// insertion points only (<= 8 per lane; the pass ends with the lane that
// has the most).
__device__ __forceinline__ uint32_t mask_range16(int32_t lo, int32_t hi) {   // bits [lo, hi) of 0..19
    lo = lo < 0 ? 0 : lo > 20 ? 20 : lo;
    hi = hi < 0 ? 0 : hi > 20 ? 20 : hi;
    return hi > lo ? ((1u << hi) - 1u) ^ ((1u << lo) - 1u) : 0u;
}

__device__ __forceinline__ uint32_t encode_general(const uint8_t *__restrict__ line, uint32_t len, Ring &r,
                                   uint32_t *rec_bytes) {
    const uint32_t l = vw::lane_id();
    const uint32_t lead = (uint32_t)(reinterpret_cast<uintptr_t>(line) & 15);
    const uint8_t *A = line - lead;
    const uint32_t span = lead + len;
    const uint32_t nch = (span + CHUNK - 1) / CHUNK;
    const vw::brsrc rs = vw::make_rsrc(A, (span + 3u) & ~3u);
    const uint32_t lo16 = BPL * l;
    uint32_t nf = 0;             // fields started so far
    uint32_t ntok = 0;           // tokens started so far
    uint32_t carryT = 1;         // byte before the chunk is T
    uint32_t pcls = CLS_NONE;    // class of the last token so far
    uint32_t prs = 1;            // run start (+1) of the last token (token 0: a virtual run begun at it, see esc8)
    uint32_t req = 0;
    r.wpos = 8;
    r.fpos = 0;
    Chunk nxt = load_chunk(rs, 0, lo16);
    for (uint32_t c = 0; c < nch; c = vw::readfirst(c + 1)) {
        const Chunk cur = look_ahead(nxt);
        if (c + 1 < nch) nxt = load_chunk(rs, c + 1, lo16);
        const int32_t x0 = (int32_t)(c * CHUNK + lo16) - (int32_t)lead;   // line offset of lane byte 0
        // ---- T mask over the lane's 16 bytes + 4 look-ahead bytes ----
        uint32_t tab = 0;
#pragma unroll
        for (int k = 0; k <= (int)TPL; k++) tab |= zero_bytes4(cur.w(k) ^ 0x09090909u) << (4 * k);
        const uint32_t inl = mask_range16(-x0, (int32_t)len - x0);
        const uint32_t T20 = (tab & inl) | (~inl & 0xFFFFFu);
        const uint32_t Tm = T20 & 0xFFFFu;
        const uint32_t pin = vw::shr1(Tm >> 15, carryT);
        const uint32_t fs = ~Tm & ((Tm << 1) | pin) & 0xFFFFu;
        const uint32_t nfs = (uint32_t)__builtin_popcount(fs);
        const uint32_t finc = vw::scan_add(nfs);
        const uint32_t fb = nf + finc - nfs;   // field index of the lane's first start
        // ---- escape-copy chunk: every token an escape of another length than
        // 3 (e.g. "a|b:DP:GQ", haploid "0"), single TABs, entered inside an
        // escape token: every token start emits TAB (its predecessor is an
        // escape) and 0xE1, every other non-TAB byte itself.
        if (nf >= 10 && pcls == CLS_ESC) {
            const uint32_t tabs = tab & inl & 0xFFFFu;
            const bool odd = (tabs & ((T20 >> 1) | (Tm << 1) | pin)) != 0 ||          // empty field / trailing TAB
                             (fs & ~(T20 >> 1) & ~(T20 >> 2) & (T20 >> 3) & 0xFFFFu) != 0;   // a 3-byte token
            if (!vw::ballot(odd)) {
                const uint32_t in16 = ~Tm & 0xFFFFu;   // in-line non-TAB bytes
                const uint32_t cnt = (uint32_t)__builtin_popcount(in16) + 2u * nfs;
                const uint32_t inc2 = vw::scan_add(cnt);
                const uint32_t base = (r.wpos + inc2 - cnt) & RMASK;
                uint8_t *const lb = r.lds + base;
                uint8_t *const dm = r.lds + RING_DUMMY;   // shared dummy word (see esc8)
                uint32_t o = 0;
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const bool st = (fs >> i) & 1u;
                    const uint16_t te = 0xE109u;   // TAB, 0xE1
                    __builtin_memcpy(st ? lb + o : dm, &te, 2);
                    o += st ? 2u : 0u;
                    const bool in = (in16 >> i) & 1u;
                    *(in ? lb + o : dm) = (uint8_t)byte_of(cur.a, (uint32_t)i);
                    o += in ? 1u : 0u;
                }
                ring_unwrap(r, base + o);
                r.wpos += vw::readlane(inc2, 63);
                const uint32_t nst = vw::readlane(finc, 63);
                nf += nst;
                ntok += nst;
                if (nst) prs = ntok;   // every escape starts a run
                carryT = vw::readlane(Tm >> 15, 63);
                ring_flush(r, false);
                continue;
            }
        }
        // ---- prefix / token split ----
        uint32_t ts = fs, pmask = 0, leadp = 0;
        if (nf < 10) {   // (wave-uniform) the prefix may end in this chunk
            for (uint32_t k = fb; k < 9 && ts; k++) ts &= ts - 1u;
            const uint32_t tok0 = fb <= 9 ? (ts & (0u - ts)) : 0u;   // start of field 9 (token 0)
            pmask = tok0 ? tok0 - 1u : (fb <= 9 ? 0xFFFFu : 0u);
            const uint32_t f0 = fb == 0 ? (fs & (0u - fs)) : 0u;     // field 0: no TAB before it
            leadp = (fs & pmask & ~f0) | tok0;
            const uint32_t nreq = (uint32_t)__builtin_popcount(pmask & ~Tm) + (uint32_t)__builtin_popcount(leadp);
            req += vw::readlane(vw::scan_add(nreq), 63);
        }
        // ---- classify the lane's tokens (in order) ----
        const uint32_t nt = (uint32_t)__builtin_popcount(ts);
        const uint32_t tinc = vw::scan_add(nt);
        const uint32_t t0 = ntok + tinc - nt;   // token index of the lane's first token
        uint32_t cl4 = 0, rem = ts;
        for (uint32_t k = 0; vw::ballot(rem != 0); k++) {
            if (rem) {
                const uint32_t i = vw::ffbl(rem);
                const uint32_t q = i >> 2;
                const uint32_t lo = q == 0 ? cur.a.x : q == 1 ? cur.a.y : q == 2 ? cur.a.z : cur.a.w;
                const uint32_t hi = q == 0 ? cur.a.y : q == 1 ? cur.a.z : q == 2 ? cur.a.w : cur.y;
                const uint32_t d = vw::alignbyte(hi, lo, i & 3u);
                const bool len3 = ((T20 >> (i + 1)) & 7u) == 4u;   // bytes i+1, i+2 not T; i+3 T
                const uint32_t cls = len3 ? cls_f(d) : CLS_ESC;
                cl4 |= cls << (4 * k);
                rem &= rem - 1u;
            }
        }
        const uint32_t vbits = nt >= 8 ? 0x11111111u : (0x11111111u & ((1u << (4 * nt)) - 1u));
        // the token before the lane: previous lanes' last token, else the chunk carry
        const uint32_t lastc = nt ? (cl4 >> (4 * (nt - 1))) & 7u : 0u;
        const uint32_t pk = nt ? ((t0 + nt) << 3) | lastc : 0u;
        const uint32_t skc = vw::scan_max(pk);
        const uint32_t pe = vw::shr1z(skc);
        const uint32_t cin = pe ? (pe & 7u) : pcls;                  // class of the token before the lane
        const uint32_t p0 = cin == CLS_NONE ? (cl4 & 3u) : cin;      // token 0: virtual run of its own class
        const uint32_t cp4 = (cl4 << 4) | p0;                         // class of token k-1 at bits 4k
        const uint32_t xc = cl4 ^ cp4;
        const uint32_t sb = (xc | (xc >> 1) | (xc >> 2) | (cl4 >> 2)) & vbits;   // run starts (escapes always)
        const uint32_t eb = (cl4 >> 2) & vbits;                                  // escapes
        const uint32_t lane_rs = sb ? (t0 + 8u) - ((uint32_t)__builtin_clz(sb) >> 2) : 0u;
        const uint32_t incl = vw::scan_max(lane_rs);
        const uint32_t rin = vw::umax(vw::shr1z(incl), prs);
        const bool is00 = p0 == 0;
        const uint32_t cap = is00 ? 127u : 31u;
        const uint32_t mp = mod_cap(t0 + MOD_BIAS - rin, is00);   // run offset of token t0 - 1, mod cap
        const uint32_t fb1 = sb ? (uint32_t)__builtin_ctz(sb) : 32u;
        const uint32_t j1 = fb1 >> 2;                                // first start (8: none)
        const uint32_t m0 = vw::perm(0x80C0A000u, 0x80C0A000u, p0 & 3u);
        const uint32_t jf = cap - 2u - mp;                           // token completing a chunk of cap
        const bool full = p0 < CLS_ESC && jf < j1 && jf < nt;
        uint32_t rr = mp + j1;
        rr = umin32(rr, rr - cap);
        const bool pesc = p0 == CLS_ESC;
        const bool lead1 = j1 < nt && (pesc || rr != cap - 1u);
        const uint32_t b1 = pesc ? 0x09u : (m0 | (rr + 1u));
        // per-byte masks: LEAD (a byte before the input byte: TAB before
        // fields 1..9, a token's run-end byte or TAB after an escape), MID
        // (0xE1 of an escape, a full-run byte), RAW (the input byte itself:
        // prefix bytes, bytes of escape tokens)
        uint32_t leadt = 0, midt = 0, escm = 0;
        for (uint32_t k = 0, rm = ts; vw::ballot(rm != 0); k++) {
            if (rm) {
                const uint32_t bit = rm & (0u - rm);
                const bool s = (sb >> (4 * k)) & 1u, e = (eb >> (4 * k)) & 1u;
                leadt |= (s && (k != j1 || lead1)) ? bit : 0u;
                midt |= (e || (full && k == jf)) ? bit : 0u;
                escm |= e ? bit : 0u;
                rm &= rm - 1u;
            }
        }
        // bytes of escape tokens: fill each token start's escape flag up to the next start
        uint32_t ev = escm, em = ts;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            ev |= (ev << d) & ~em;
            em |= em << d;
        }
        ev = (ev | (cin == CLS_ESC ? ~em : 0u)) & 0xFFFFu;
        const uint32_t RAW = (pmask | ev) & ~Tm & 0xFFFFu;
        const uint32_t LEAD = leadp | leadt, MID = midt;
        const uint32_t cnt = (uint32_t)__builtin_popcount(RAW) + (uint32_t)__builtin_popcount(LEAD) +
                             (uint32_t)__builtin_popcount(MID);
        const uint32_t inc2 = vw::scan_add(cnt);
        const uint32_t base = (r.wpos + inc2 - cnt) & RMASK;
        uint8_t *const lb = r.lds + base;
        uint8_t *const dm = r.lds + RING_DUMMY;   // shared dummy word (see esc8)
        // pass 1: the raw bytes, each at its place after the bytes inserted before it
        uint32_t o = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            o += ((LEAD >> i) & 1u) + ((MID >> i) & 1u);
            const bool ri = (RAW >> i) & 1u;
            *(ri ? lb + o : dm) = (uint8_t)byte_of(cur.a, (uint32_t)i);
            o += ri ? 1u : 0u;
        }
        // pass 2: the inserted bytes, one insertion point (a field or token
        // start) per step
        for (uint32_t rm = LEAD | MID; vw::ballot(rm != 0);) {
            if (rm) {
                const uint32_t i = vw::ffbl(rm);
                const uint32_t below = (1u << i) - 1u;
                const uint32_t oi = (uint32_t)__builtin_popcount(RAW & below) + (uint32_t)__builtin_popcount(LEAD & below) +
                                    (uint32_t)__builtin_popcount(MID & below);
                const bool li = (LEAD >> i) & 1u, mi = (MID >> i) & 1u;
                uint32_t lv = 0x09u, mv = 0xE1u;
                if ((ts >> i) & 1u) {   // a token start: its run-end byte (not token 0's TAB), its escape / full byte
                    const uint32_t k = (uint32_t)__builtin_popcount(ts & below);
                    const uint32_t pc = (cp4 >> (4 * k)) & 7u;
                    const uint32_t sbk = sb & ((1u << (4 * k)) - 1u);   // starts before token k
                    const uint32_t kp = sbk ? (31u - (uint32_t)__builtin_clz(sbk)) >> 2 : 0u;
                    if ((leadt >> i) & 1u)
                        lv = k == j1 ? b1 : (pc == CLS_ESC ? 0x09u : (vw::perm(0x80C0A000u, 0x80C0A000u, pc & 3u) | (k - kp)));
                    mv = (eb >> (4 * k)) & 1u ? 0xE1u : (m0 | cap);
                }
                *(li ? lb + oi : dm) = (uint8_t)lv;
                *(mi ? lb + oi + (li ? 1u : 0u) : dm) = (uint8_t)mv;
                rm &= rm - 1u;
            }
        }
        ring_unwrap(r, base + o);
        r.wpos += vw::readlane(inc2, 63);
        // carries
        nf += vw::readlane(finc, 63);
        ntok += vw::readlane(tinc, 63);
        carryT = vw::readlane(Tm >> 15, 63);
        const uint32_t last = vw::readlane(skc, 63);
        if (last) pcls = last & 7u;
        prs = vw::umax(vw::readlane(incl, 63), prs);
        ring_flush(r, false);
    }
    if (nf < 8) return VCFCD_E_LT8COLS;
    if (nf == 8) return VCFCD_E_8COLS;
    // row end: pending chunk of the last run, then '\n'
    const uint32_t T = ntok;
    uint32_t extra = 0, pb = 0;
    if (T > 0 && pcls < CLS_ESC) {
        const uint32_t off = mod_cap(T - prs, pcls == 0);
        if (off != (pcls == 0 ? 126u : 30u)) { extra = 1; pb = cls_mask_f(pcls) | (off + 1); }
    }
    if (l == 0) {
        if (extra) ring_put(r, r.wpos, pb);
        ring_put(r, r.wpos + extra, 0x0Au);
    }
    r.wpos += extra + 1;
    ring_finish(r, req);
    *rec_bytes = r.wpos;
    return VCFCD_OK;
}

// Row prologue shared by both encode kernels: slot bounds check + ring setup.
__device__ __forceinline__ bool row_setup(const VcfcEncodeArgs &a, uint64_t row, uint8_t *lds, Ring &r) {
    r.lds = lds;
    r.pb = a.prim_bytes;
    r.prim = a.prim + (uint64_t)a.prim_bytes * row;
    r.slot = a.slots + a.slot_off[row];
    r.wpos = 8;
    r.fpos = 0;
    r.mode = RING_STAGE;
    const uint32_t st = a.line_len[row] > VCFCD_MAX_LINE ? VCFCD_E_TOOLONG
                        : a.slot_off[row + 1] > a.slots_cap ? VCFCD_E_NOSPACE : VCFCD_OK;
    if (st != VCFCD_OK) {
        if (vw::lane_id() == 0) {
            a.rec_size[row] = 0;
            atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | st));
        }
        return false;
    }
    return true;
}

// Fast kernel: one wave per row; rows without the GT-only shape are queued
// for the general path.
// Pinned to 6 waves/SIMD (the SGPR count allows no more): without the pin the
// branch-free escape emission takes 84 VGPRs and 5 waves, +5 % on the
// headline rows (profiles/r02/ab/ab_esc8_emit.txt).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 6))) void k_encode_fast(VcfcEncodeArgs a, uint64_t row_lo, uint64_t row_hi) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[K1_WAVES * RING_STRIDE];
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);   // wave-uniform: scalar row/len/loop control
    const uint64_t row = row_lo + (uint64_t)blockIdx.x * K1_WAVES + wave;   // rows [row_lo, row_hi): one piece
    if (row >= row_hi) return;
    VCFC_DIAG_ROW_BEGIN();
    Ring r;
    if (!row_setup(a, row, lds + wave * RING_STRIDE, r)) return;
    uint32_t bytes = 0, gt0 = ~0u;
    const bool ok = encode_fast(a.buf + a.line_off[row], a.line_len[row], r, &bytes, &gt0, a.defer_records != 0);
    VCFC_DIAG_ROW_END(a, row);
    if (vw::lane_id() == 0) {
        // not the fast shape: k_encode_var's wave for this row takes it
        // (a flag per row, no shared queue: 750k rows appending to one
        // counter serialise at the memory side, ~8 ms on the law-2 rows),
        // with the first sample's offset when the prefix was parsed clean
        a.rec_size[row] = ok ? bytes : (gt0 < VCFCD_GT0_NONE ? (VCFCD_RETRY_GT | gt0) : VCFCD_RETRY);
    }
}

// a '\n' among the row's bytes (VcfcEncodeArgs::nl_check): 4 KiB per round
__device__ bool row_has_nl(const uint8_t *__restrict__ line, uint32_t len) {
    const uint32_t l = vw::lane_id();
    const uint32_t lead = (uint32_t)(reinterpret_cast<uintptr_t>(line) & 15);
    const uint32_t span = lead + len;
    const vw::brsrc rs = vw::make_rsrc(line - lead, (span + 3u) & ~3u);
    for (uint32_t c = 0; c < span; c = vw::readfirst(c + 4096u)) {
        uint4 v[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) v[k] = vw::bload16(rs, c + 1024u * k + 16u * l, 0);
        bool hit = false;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const int32_t o = (int32_t)(c + 1024u * k + 16u * l);
            const uint32_t m = zero_bytes4(v[k].x ^ 0x0A0A0A0Au) | (zero_bytes4(v[k].y ^ 0x0A0A0A0Au) << 4) |
                               (zero_bytes4(v[k].z ^ 0x0A0A0A0Au) << 8) | (zero_bytes4(v[k].w ^ 0x0A0A0A0Au) << 12);
            hit |= (m & mask_range16((int32_t)lead - o, (int32_t)span - o)) != 0;
        }
        if (vw::ballot(hit)) return true;
    }
    return false;
}

// rows per wave of the variable-token kernel (16: law 2 -1.8 %, headline
// step +0.2 % in empty waves; 8: -1.7 % / +0.5 %; profiles/r03/ab/ab_var_rows.txt)
// (round 6, profiles/r06/ab/ab_r6vr_*.txt: 16 / 8 rows take the grid's
// last-round tail off the haploid-mix rows, kind 0 -1.4 / -2.8 %, but the
// prediction learns its token count per wave: GT:DP:GQ rows +3 / +10 %, law
// 2 +1.3 / +3.6 %)
constexpr uint32_t VAR_ROWS = 32;
// Variable-token kernel: the rows the fast kernel flagged, VAR_ROWS per wave
// (a flag load per 32 rows, so a batch without such rows costs next to
// nothing); a row of another shape takes the general path in the same wave
// (round 2 ran it as a kernel of its own, k_encode_general: one more launch,
// ~4.5 us on the headline rows, which flag none).  A resident grid striding
// over rows was 13.6 % slower on law 2 (profiles/r02/ab/ab_gen_persist.txt).
template <int VM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5))) void k_encode_var(VcfcEncodeArgs a, uint64_t row_lo, uint64_t row_hi) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[K1_WAVES * RING_STRIDE];
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    const uint32_t l = vw::lane_id();
    const uint64_t row0 = row_lo + ((uint64_t)blockIdx.x * K1_WAVES + wave) * VAR_ROWS;
    // a flagged row: VCFCD_RETRY, or VCFCD_RETRY_GT | the first sample's offset
    const uint32_t rs = l < VAR_ROWS && row0 + l < row_hi ? a.rec_size[row0 + l] : 0u;
    const bool flagged = (rs & VCFCD_RETRY_GT) == VCFCD_RETRY_GT;
    uint64_t todo = vw::ballot(flagged);
    uint32_t dmask = 0;   // rows deferred (bit: row - row0)
    // (VAR_DEFER) token counts of the wave's rows encoded in full: once two
    // in a row agree, later deferred rows are predicted from it (a VCF's
    // rows all hold one token per sample; a wrong guess costs the batch a
    // second size scan, compaction and deferred pass, never wrong output)
    uint32_t ntok_ref = 0, ntok_last = ~0u;
    while (todo) {
        const uint64_t row = row0 + (uint64_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        Ring r;
        if (!row_setup(a, row, lds + wave * RING_STRIDE, r)) continue;
        // a.nl_check (the hop line index guessed line ends): a row holding a
        // '\n' is not encoded and the caller indexes the lines again.  The
        // variable-token path checks its genotype chunks as it reads them
        // (round 4; a separate scan of every flagged row cost law 2 ~1 ms on
        // the device file), the general path scans the row first.
        uint32_t bytes = 0, ntok = 0;
        bool nlhit = false, deferred = false, predicted = false;
        const uint32_t gt0 = vw::readlane(rs, (uint32_t)(row - row0)) & VCFCD_GT0_NONE;
        const bool var_ok = encode_var<VM>(a.buf + a.line_off[row], a.line_len[row], r, &bytes, a.nl_check, &nlhit,
                                           &deferred, gt0, ntok_ref, &predicted, &ntok);
        if (VM == VAR_DEFER && var_ok && !predicted) {
            ntok_ref = ntok == ntok_last ? ntok : 0u;
            ntok_last = ntok;
        }
        if (!var_ok && !nlhit && a.nl_check) nlhit = row_has_nl(a.buf + a.line_off[row], a.line_len[row]);
        if (nlhit) {
            if (l == 0) {
                a.rec_size[row] = 0;
                atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | VCFCD_E_NEWLINE));
            }
            continue;
        }
        if (var_ok) {
            if (l == 0) a.rec_size[row] = deferred ? (bytes | VCFCD_DEFER) : bytes;
            if (VM == VAR_DEFER && deferred) dmask |= 1u << (uint32_t)(row - row0);
            continue;
        }
        // not the variable-token shape: the general path, in this wave
        VCFC_DIAG_GENERAL_ROW(a);
        row_setup(a, row, lds + wave * RING_STRIDE, r);   // (the ring again; the slot fits, checked above)
        const uint32_t st = encode_general(a.buf + a.line_off[row], a.line_len[row], r, &bytes);
        if (l == 0) {
            a.rec_size[row] = st == VCFCD_OK ? bytes : 0u;
            if (st != VCFCD_OK) atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | st));
        }
    }
    if (VM == VAR_DEFER && dmask) {   // one append per wave
        uint32_t q0 = 0;
        if (l == 0) q0 = atomicAdd(a.defer_count, (uint32_t)__builtin_popcount(dmask));
        q0 = vw::readfirst(q0);
        if (l < VAR_ROWS && ((dmask >> l) & 1u))
            a.defer_list[q0 + (uint32_t)__builtin_popcount(dmask & ((1u << l) - 1u))] = (uint32_t)(row0 + l);
    }
}

// scan shape (k_scan_lb / launch_scan below): items per thread, threads and items per block
constexpr int SCAN_ITEMS = 16, SCAN_THREADS = 256, SCAN_TILE = SCAN_ITEMS * SCAN_THREADS;

// Deferred rows (VCFCD_DEFER): after the size scan and the compaction, each
// record is encoded again from its line straight into out at rec_off[row]
// (RING_DIRECT; whole 16-byte blocks, the last few bytes one by one, so a
// neighbour's bytes -- the compaction's -- are never touched).  A resident
// grid strides over the deferred-row list; an empty list costs the launch.
// PASS 1 also checks the sizes k_encode_var predicted (it reads each line in
// full anyway): a record of another size, a line of another shape (then
// encoded by the general path into its staging, no longer deferred), a line
// holding '\n' (a.nl_check) or a record not certainly inside out_cap (its
// offset may rest on predictions) sets a.mispredict.  The first wave to set
// it rearms the size scan's look-back state, and the gated size scan,
// compaction and PASS 2 then redo the layout on exact sizes; without a
// misprediction they return at once (the scan merging the first scan's
// out_cap report into err).
template <int PASS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5))) void k_encode_defer(VcfcEncodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[K1_WAVES * RING_STRIDE];
    if (PASS == 2 && *a.mispredict == 0) return;
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    const uint32_t l = vw::lane_id();
    const uint32_t cnt = vw::readfirst(*a.defer_count);
    const uint32_t G = gridDim.x * K1_WAVES;
    auto miss = [&]() {
        uint32_t first = 0;
        if (l == 0) first = atomicExch(a.mispredict, 1u) == 0u ? 1u : 0u;
        if (vw::readfirst(first)) {
            // the first wave to miss rearms the size scan's ticket and tile
            // flags for its second launch (the whole wave: nt + 1 words)
            const uint64_t nt = (a.n + SCAN_TILE - 1) / SCAN_TILE;
            uint32_t *tickets = reinterpret_cast<uint32_t *>(a.lb);
            uint64_t *flags_b = reinterpret_cast<uint64_t *>(a.lb + 16) + nt + 1;
            if (l == 0) tickets[1] = 0;
            for (uint64_t i = l; i <= nt; i += 64) flags_b[i] = 0;
        }
    };
    for (uint32_t q = blockIdx.x * K1_WAVES + wave; q < cnt; q += G) {
        const uint64_t row = vw::readfirst(a.defer_list[q]);
        const uint32_t rsz = a.rec_size[row];
        if (PASS == 2 && !(rsz & VCFCD_DEFER)) continue;   // (taken by the general path in pass 1)
        const uint32_t size = rsz & ~VCFCD_DEFER;
        const uint32_t len = a.line_len[row];
        const uint64_t o = a.rec_off[row];
        // pass 1, a record not certainly inside out_cap (its offset may rest
        // on predictions): sized only, never written, so that the exact
        // layout (pass 2) rests on its true size or its true fate (general
        // path, '\n') -- a prediction kept here could be short of the record
        // pass 2 then writes (a write past out_cap)
        const bool capx = PASS == 1 && o + (uint64_t)len + (len >> 1) + 16u > a.out_cap;
        if (PASS == 2 && o + size > a.out_cap) {   // (the size scan reported it)
            if (l == 0) atomicAdd(a.defer_fallback, 1u);   // (not written: not counted as deferred)
            continue;
        }
        Ring r;
        r.lds = lds + wave * RING_STRIDE;
        r.prim = a.out + o;
        r.slot = nullptr;
        r.pb = 0xFFFFFFFFu;
        r.wpos = 8;
        r.fpos = 0;
        r.mode = capx ? RING_SIZE : RING_DIRECT;
        uint32_t bytes = 0;
        bool nlhit = false, deferred = false;
        const bool ok = encode_var<VAR_DIRECT>(a.buf + a.line_off[row], len, r, &bytes, PASS == 1 && a.nl_check,
                                               &nlhit, &deferred, VCFCD_GT0_NONE);
        if (PASS == 2) {
            if (l == 0 && (!ok || bytes != size))   // (cannot happen: the sizes are exact)
                atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | VCFCD_E_INTERNAL));
            continue;
        }
        if (ok && bytes == size && !capx) continue;
        miss();   // (a wrong size, another fate, or the cap: pass 2 on exact offsets)
        if (ok) {   // the exact size (a predicted one may have been wrong)
            if (l == 0) a.rec_size[row] = bytes | VCFCD_DEFER;
            continue;
        }
        bool nl = nlhit;
        if (!nl && a.nl_check) nl = row_has_nl(a.buf + a.line_off[row], len);
        if (nl) {   // (as k_encode_var: the caller indexes the lines again)
            if (l == 0) {
                atomicAdd(a.defer_fallback, 1u);
                a.rec_size[row] = 0;
                atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | VCFCD_E_NEWLINE));
            }
            continue;
        }
        // another shape after its first chunk: the general path, staged (as k_encode_var)
        if (l == 0) atomicAdd(a.defer_fallback, 1u);
        if (!row_setup(a, row, lds + wave * RING_STRIDE, r)) continue;
        const uint32_t st = encode_general(a.buf + a.line_off[row], len, r, &bytes);
        if (l == 0) {
            a.rec_size[row] = st == VCFCD_OK ? bytes : 0u;
            if (st != VCFCD_OK) atomicMin((unsigned long long *)a.err, (unsigned long long)((row << 8) | st));
        }
    }
}

constexpr uint32_t DEFER_BLOCKS = 1280;   // 5 waves per SIMD over 256 CUs, 4 waves per block (640: law 2 +1.6 %)

// blocks of k_encode_var to launch for m rows
static uint64_t var_blocks(uint64_t m, uint32_t rows_per_wave = VAR_ROWS) {
    const uint64_t per_block = (uint64_t)K1_WAVES * rows_per_wave;
    return (m + per_block - 1) / per_block;
}

// ---------------------------------------------------------------------------
// Compaction: staging -> out[rec_off[row]] with aligned 16-byte stores.
// realign16: bytes [sh, sh + 16) of the 32 bytes (lo, hi).
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

// ---------------------------------------------------------------------------
// Output-ordered compaction: the output is cut into 4 KiB tiles;
// a grid of waves strides over the tiles, and within a tile lane l writes the
// 16-byte blocks l, l + 64, l + 128, l + 192, so every store instruction
// covers 1 KiB of the output contiguously and every output line is written
// once, by one wave.  A block's bytes come from the record holding its first
// byte (an unaligned 16-B load from that record's staging), merged with the
// overflow slot's first bytes where the block crosses record byte
// prim_bytes, and with the next record's first bytes where it crosses a
// record end (records hold >= 26 bytes, so a block meets at most two).
// The size scan (k_scan_lb<0, true>) gives each tile the row holding its
// first byte.  (4 KiB tiles: 2 KiB the same, 8 KiB +45 %, ab_compact_tile.txt;
// the round-1 row-ordered kernel was 12 % slower, ab_compact_out.txt.)
constexpr uint32_t CTB = 4;                // 16-B blocks per lane per tile
// tile_first flag: the tile lies inside a deferred record.  It shares the
// word with the row index, so deferral needs rows < 2^31 (vcfc_encode_device
// turns it off for larger batches; without it the bound is 2^32 rows)
constexpr uint32_t TILE_DEFERRED = 0x80000000u;
constexpr uint32_t CT = 1024 * CTB;        // output bytes per tile

// bytes [0, s) of a, then b's first 16 - s bytes (0 < s < 16)
__device__ __forceinline__ uint4 merge16(uint4 a, uint4 b, uint32_t s) {
    const uint4 sh = realign16(make_uint4(0, 0, 0, 0), b, 16u - s);
    auto m = [&](uint32_t d) {
        return s >= 4 * d + 4 ? ~0u : s <= 4 * d ? 0u : (1u << (8 * (s - 4 * d))) - 1u;
    };
    const uint32_t m0 = m(0), m1 = m(1), m2 = m(2), m3 = m(3);
    return make_uint4((a.x & m0) | (sh.x & ~m0), (a.y & m1) | (sh.y & ~m1), (a.z & m2) | (sh.z & ~m2),
                      (a.w & m3) | (sh.w & ~m3));
}

// Tiles wholly inside a deferred record (VCFCD_DEFER; the size scan flags
// them in tile_first) are skipped: k_encode_defer writes those records
// afterwards (a tile shared with a staged record is written here with
// whatever the deferred record's staging holds, and k_encode_defer then
// rewrites the deferred record's bytes of it).
__global__ __launch_bounds__(256) void k_compact_out(const uint8_t *__restrict__ prims,
                                                     const uint8_t *__restrict__ slots,
                                                     const uint64_t *__restrict__ slot_off,
                                                     const uint64_t *__restrict__ rec_off, uint64_t n,
                                                     const uint32_t *__restrict__ tile_first,
                                                     uint8_t *__restrict__ out, uint64_t out_cap, uint32_t pb,
                                                     const uint32_t *gate, const uint32_t *__restrict__ rec_size,
                                                     const uint32_t *defer_count) {
    if (gate && *gate == 0) return;   // (the second compaction: only after a misprediction)
    // (round 6: with deferred records in the batch, a 16-byte block whose
    // bytes all belong to deferred records is neither loaded nor stored --
    // k_encode_defer writes it; blocks shared with a staged record are
    // copied whole as before, their deferred bytes rewritten by k_encode_defer)
    const bool anyd = defer_count && vw::readfirst(*defer_count) != 0;
    const uint32_t l = vw::lane_id();
    const uint64_t g = (uint64_t)blockIdx.x * 4 + vw::readfirst(threadIdx.x >> 6);
    const uint64_t G = (uint64_t)gridDim.x * 4;
    const uint32_t pbs = 31u - (uint32_t)__builtin_clz(pb);   // prim_bytes is a power of two (vcfc_prim_bytes)
    const uint64_t total = rec_off[n];
    const uint64_t lim = total < out_cap ? total : out_cap;
    const uint64_t ntile = (lim + CT - 1) / CT;
    for (uint64_t t = g; t < ntile; t += G) {
        const uint64_t o0 = t * CT;
        const uint32_t tfr = tile_first[t];
        if (tfr & TILE_DEFERRED) continue;   // inside one deferred record (k_encode_defer's)
        const uint64_t r0 = tfr;
        // rows r0 .. r0 + 63: their starts (lane j holds row r0 + j); rows
        // past n start "at infinity"
        const uint64_t ro = r0 + l <= n ? rec_off[r0 + l] : ~0ull;
        const uint64_t so = r0 + l < n ? slot_off[r0 + l] : 0;
        // deferred rows of the batch as a 64-bit lane mask (anyd only)
        uint64_t dmask = anyd ? vw::ballot(r0 + l < n && (rec_size[r0 + l] & VCFCD_DEFER)) : 0ull;
        // rows that start before the tile ends; a tile over more than 63
        // rows (records of < 64 B on average) takes the rows in batches
        uint64_t base = r0;   // row of lane 0's values
        uint64_t rov = ro, sov = so;
        // per block: the row holding its first byte (start, end, slot) and
        // the row holding its last byte (a block meets at most two non-empty
        // records; empty rows -- failed lines -- start where the next begins)
        uint32_t idx[CTB], idx2[CTB];
        uint64_t st[CTB], en[CTB], sl[CTB];
        uint32_t skm = 0;   // (anyd) bit k: every record touching block k is deferred
#pragma unroll
        for (int k = 0; k < (int)CTB; k++) { idx[k] = 0; idx2[k] = 0; st[k] = 0; en[k] = 0; sl[k] = 0; }
        for (;;) {
            const uint64_t bnd = vw::ballot(rov < o0 + CT);   // rows (of this batch) starting before the tile end
            const uint32_t nr = (uint32_t)vw::popc64(bnd);    // a prefix of the lanes (starts are sorted)
            const uint32_t nu = nr < 63 ? nr : 63;            // lane j + 1 holds row j's end
            for (uint32_t j = 0; j < nu; j++) {
                const uint64_t rj = ((uint64_t)vw::readlane((uint32_t)(rov >> 32), j) << 32) | vw::readlane((uint32_t)rov, j);
                const uint64_t ej = ((uint64_t)vw::readlane((uint32_t)(rov >> 32), j + 1) << 32) | vw::readlane((uint32_t)rov, j + 1);
                const uint64_t sj = ((uint64_t)vw::readlane((uint32_t)(sov >> 32), j) << 32) | vw::readlane((uint32_t)sov, j);
                const uint32_t ij = (uint32_t)(base - r0) + j;
                const bool dj = (dmask >> j) & 1u;
#pragma unroll
                for (int k = 0; k < (int)CTB; k++) {
                    const uint64_t o = o0 + 16u * (l + 64u * k);
                    if (o >= rj) { idx[k] = ij; st[k] = rj; en[k] = ej; sl[k] = sj; }
                    if (o + 15 >= rj) idx2[k] = ij;
                    if (anyd) {
                        const uint32_t b = 1u << k;
                        skm = o >= rj ? (dj ? skm | b : skm & ~b) : (o + 15 >= rj && !dj ? skm & ~b : skm);
                    }
                }
            }
            if (nr < 64) break;
            // lane 63's row starts inside the tile too: next batch from row base + 63
            base += 63;
            rov = base + l <= n ? rec_off[base + l] : ~0ull;
            sov = base + l < n ? slot_off[base + l] : 0;
            dmask = anyd ? vw::ballot(base + l < n && (rec_size[base + l] & VCFCD_DEFER)) : 0ull;
        }
#pragma unroll
        for (int k = 0; k < (int)CTB; k++) {
            const uint64_t o = o0 + 16u * (l + 64u * k);
            if (o >= lim) continue;
            if ((skm >> k) & 1u) continue;   // (k_encode_defer's bytes)
            const uint64_t r = r0 + idx[k];
            const uint64_t x = o - st[k];   // offset in the record
            const uint8_t *prim = prims + (r << pbs);
            const uint8_t *slot = slots + sl[k];
            uint4 v = x + 16 <= pb ? vw::uload16(prim + x) : x >= pb ? vw::uload16(slot + (x - pb)) : vw::uload16(prim + x);
            if (x < pb && x + 16 > pb) v = merge16(v, vw::uload16(slot), (uint32_t)(pb - x));
            if (o + 16 > en[k] && en[k] < lim)   // the next non-empty record starts at en
                v = merge16(v, vw::uload16(prims + ((r0 + idx2[k]) << pbs)), (uint32_t)(en[k] - o));
            if (o + 16 <= lim) {
                // non-temporal: the records leave the chip (D2H, a file, the
                // next stage), and the next batch's encode keeps L2 / MALL to
                // itself (-0.8 % per step in an A/B, ab_compact_nt.txt; round 3
                // again: plain stores +1 % k_compact on law 1, +5 % on law 2,
                // profiles/r03/ab/ab_compact_plain.txt)
                vw::gstore16_nt(out, o, v);
            } else {
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                for (uint32_t i = 0; o + i < lim; i++) out[o + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Exclusive scan u32 -> u64 (n + 1 outputs).  MODE 0: identity, MODE 1:
// vcfc_slot_bytes(len), MODE 2: record sizes (VCFCD_DEFER masked), MODE 3:
// line kinds, two counts in one word (bit 0 -> the low half, bit 1 -> the
// high half: both stay below 2^32 for a chunk's < 2^32 - 1 lines).  4096
// items per 256-thread block.

template <int MODE> __device__ __forceinline__ uint64_t scan_xf(uint32_t v) {
    return MODE == 1   ? vcfc_slot_bytes(v)
           : MODE == 2 ? (uint64_t)(v & ~VCFCD_DEFER)
           : MODE == 3 ? (uint64_t)(v & 1u) | ((uint64_t)((v >> 1) & 1u) << 32)
                       : (uint64_t)v;
}

// Exclusive block scan of u64 values: each wave scans four 16-bit limbs with
// DPP add-scans (exact: 64 x 0xFFFF < 2^22), the four wave totals go through
// LDS (one barrier), instead of an 8-step LDS scan with 16 barriers.
__device__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t *sh, uint64_t *total) {
    static_assert(SCAN_THREADS == 256, "four waves per block");
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint64_t inc = (uint64_t)vw::scan_add(lo & 0xFFFFu) + ((uint64_t)vw::scan_add(lo >> 16) << 16) +
                         ((uint64_t)vw::scan_add(hi & 0xFFFFu) << 32) + ((uint64_t)vw::scan_add(hi >> 16) << 48);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 63u) sh[w] = inc;   // wave totals
    __syncthreads();
    const uint64_t t0 = sh[0], t1 = sh[1], t2 = sh[2], t3 = sh[3];
    __syncthreads();   // (sh is reused by the caller's next scan)
    *total = t0 + t1 + t2 + t3;
    const uint64_t before = (w > 0 ? t0 : 0) + (w > 1 ? t1 : 0) + (w > 2 ? t2 : 0);
    return before + inc - v;
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

// ---------------------------------------------------------------------------
// Single-pass exclusive scan u32 -> u64 (n + 1 outputs) with decoupled
// look-back over tiles of SCAN_TILE items: the encoder's two scans in one
// launch each instead of three.  Tiles take a ticket in launch order, so a
// tile only ever waits for tiles whose blocks are already running.  A tile's
// state is one 8-byte word {status:2, value:62} written by a single
// agent-scope store and polled with agent-scope loads (one naturally aligned
// word: no payload to order; MI355X_MICROARCH.md, inter-workgroup
// visibility).  MODE as launch_scan; TILES (the size scan) also gives every
// 4 KiB output tile its first row (k_compact_out) and flags records that end
// past out_cap.  State (tickets, flags) zeroed before the launch.
constexpr uint64_t LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = LB_AGG - 1;

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// gate (the size scan's second launch, after k_encode_defer<1>): nothing
// to redo unless *gate -- then block 0 merges the first scan's out_cap
// report (*merge) into err and every block returns.
template <int MODE, bool TILES>
__global__ __launch_bounds__(256) void k_scan_lb(const uint32_t *__restrict__ in, uint64_t n, uint32_t *ticket,
                                                 uint64_t *flags, uint64_t *__restrict__ out,
                                                 uint32_t *__restrict__ tile_first, uint64_t out_cap, uint64_t *err,
                                                 const uint32_t *gate, const uint64_t *merge) {
    __shared__ uint64_t sh[SCAN_THREADS];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_excl;
    if (gate && *gate == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && merge && *merge != ~0ull)
            atomicMin((unsigned long long *)err, (unsigned long long)*merge);
        return;
    }
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t base = tile * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t vals[SCAN_ITEMS];
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; i++) {
        vals[i] = base + i < n ? scan_xf<MODE>(in[base + i]) : 0;
        sum += vals[i];
    }
    uint64_t agg;
    const uint64_t texcl = block_excl_scan_u64(sum, sh, &agg);
    if (threadIdx.x < 64) {   // wave 0: publish the aggregate, look back
        const uint32_t l = threadIdx.x;
        if (l == 0) lb_store(flags + tile, (tile == 0 ? LB_INC : LB_AGG) | agg);
        uint64_t excl = 0;
        if (tile > 0) {
            int64_t p = (int64_t)tile - 1;   // the window covers tiles p, p - 1, ..., p - 63
            for (;;) {
                const int64_t q = p - (int64_t)l;
                const uint64_t f = q >= 0 ? lb_load(flags + q) : LB_INC;   // (before tile 0: an inclusive 0)
                const uint64_t inc = vw::ballot((f >> 62) == 2);
                const uint32_t k = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;   // nearest inclusive prefix
                const uint64_t ready = vw::ballot((f >> 62) != 0);
                const uint64_t need = k < 64 ? (k == 63 ? ~0ull : ((2ull << k) - 1)) : ~0ull;
                if ((ready & need) != need) {   // a tile before it has not published yet
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const uint64_t v = l <= k ? (f & LB_VAL) : 0;
                // wave total of v, exact: four 16-bit limbs (64 x 0xFFFF fits 32 bits)
                const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
                const uint64_t tlo = (uint64_t)vw::readlane(vw::scan_add(lo & 0xFFFFu), 63) +
                                     ((uint64_t)vw::readlane(vw::scan_add(lo >> 16), 63) << 16);
                const uint64_t thi = (uint64_t)vw::readlane(vw::scan_add(hi & 0xFFFFu), 63) +
                                     ((uint64_t)vw::readlane(vw::scan_add(hi >> 16), 63) << 16);
                excl += tlo + (thi << 32);
                if (k < 64) break;
                p -= 64;
            }
            if (l == 0) lb_store(flags + tile, LB_INC | (excl + agg));
        }
        if (l == 0) s_excl = excl;
    }
    __syncthreads();
    uint64_t run = s_excl + texcl;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; i++) {
        const uint64_t r = base + i;
        if (r < n) {
            out[r] = run;
            if (TILES) {
                const uint64_t b = run + vals[i];
                if (b > out_cap) atomicMin((unsigned long long *)err, (unsigned long long)((r << 8) | VCFCD_E_NOSPACE));
                // (a tile whose bytes all belong to deferred records: flagged,
                // the compaction skips it -- k_encode_defer writes those
                // bytes.  The tile a deferred record ends in is followed
                // into the next records while they are deferred or empty;
                // records end past the batch's last byte count as covered.
                // Round 5: kind-1 law 2, every record deferred, k_compact
                // copied one 4 KiB tile of staging garbage per record)
                const bool dr = MODE == 2 && (in[r] & VCFCD_DEFER);
                for (uint64_t t = (run + CT - 1) / CT; t * CT < b; t++) {
                    const uint64_t te = (t + 1) * CT;
                    bool skip = dr && te <= b;
                    if (dr && te > b) {
                        uint64_t e = b, q = r + 1;
                        for (int k = 0; k < 4 && q < n && e < te; k++, q++) {
                            const uint32_t v = in[q];
                            if (v != 0 && !(v & VCFCD_DEFER)) break;
                            e += v & ~VCFCD_DEFER;
                        }
                        skip = e >= te || q >= n;
                    }
                    tile_first[t] = (uint32_t)r | (skip ? TILE_DEFERRED : 0u);
                }
            }
            if (r + 1 == n) out[n] = run + vals[i];
        }
        run += vals[i];
    }
}

// Per-call state of one encode: the look-back tickets and tile flags zeroed,
// the first-error word set to "none".  A kernel rather than two
// hipMemsetAsync calls: replays of a HIP graph captured around
// vcfc_encode_device spun in the look-back on the second replay
// (tools/dbg/graph_probe.py).  Round 4 pinned the cause
// (tools/dbg/memset_graph_probe.py, profiles/r04/memset_graph_probe.txt):
// memset nodes of 4 and 8 bytes replay correctly, but a 24-byte node writes
// garbage into its first 16 bytes from the second replay on, consistent
// with the hang (the ticket array's memset, far more than 8 bytes, did not
// leave zeros).  A kernel node is replayed like every other launch.
__global__ __launch_bounds__(256) void k_encode_reset(uint64_t *lb, uint64_t words, uint64_t *err, uint64_t *nospace) {
    for (uint64_t i = threadIdx.x; i < words; i += 256) lb[i] = 0;
    if (threadIdx.x == 0) {
        *err = ~0ull;
        *nospace = ~0ull;
    }
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
    // look-back scan state, zeroed by one memset per encode: the two scans'
    // tickets, the retry counter, the two scans' tile flags
    const uint64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE + 1;
    L.lb = o;
    L.retry_count = o + 8;
    L.defer_count = o + 12;
    // after both scans' flags: the misprediction word, the fallback count, the first scan's out_cap report
    L.mispredict = o + 16 + 16 * nt;
    L.defer_fallback = L.mispredict + 4;
    L.nospace = L.mispredict + 8;
    L.lb_bytes = 32 + 16 * nt;
    o = al(o + L.lb_bytes);
    L.defer_list = o; o = al(o + 4 * n);
    L.tile_first = o; o = al(o + 4 * (vcfc_record_bound(n, total_line_bytes) / CT + 2));
    L.prim_bytes = vcfc_prim_bytes(n, total_line_bytes);
    L.prim = o; o = al(o + (uint64_t)L.prim_bytes * n);
    L.slots = o; o = al(o + total_line_bytes + total_line_bytes / 2 + 64 * (n + 1));
    L.dbg = o;
    o += VCFC_DIAG_WS_BYTES(n);
    L.total = o;
    return L;
}

hipError_t vcfc_encode_device(const VcfcEncodeArgs &a, hipStream_t s, hipEvent_t *ev) {
    hipError_t e;
    if (a.n == 0) {
        if ((e = hipMemsetAsync(a.err, 0xFF, 8, s)) != hipSuccess) return e;
        return hipMemsetAsync(a.rec_off, 0, 8, s);
    }
    // Deferred records need the row index below TILE_DEFERRED (tile_first
    // carries both): batches of 2^31 rows or more encode without deferral.
    if (a.defer_records && a.n >= (uint64_t)TILE_DEFERRED) {
        VcfcEncodeArgs b = a;
        b.defer_records = 0;
        return vcfc_encode_device(b, s, ev);
    }
    const uint64_t nt = (a.n + SCAN_TILE - 1) / SCAN_TILE;   // scan tiles
    // lb: tickets (slot scan, size scan), retry counter, slot-scan flags
    // (nt + 1), size-scan flags (nt + 1)
    uint32_t *tickets = reinterpret_cast<uint32_t *>(a.lb);
    uint64_t *flags_a = reinterpret_cast<uint64_t *>(a.lb + 16), *flags_b = flags_a + nt + 1;
    // (the tickets and counters, both scans' flags, the misprediction word and the fallback count)
    hipLaunchKernelGGL(k_encode_reset, dim3(1), dim3(256), 0, s, reinterpret_cast<uint64_t *>(a.lb),
                       (uint64_t)(2 + 2 * (nt + 1) + 1), a.err, a.nospace);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[0], s);
    hipLaunchKernelGGL((k_scan_lb<1, false>), dim3((unsigned)nt), dim3(SCAN_THREADS), 0, s, a.line_len, a.n, tickets,
                       flags_a, a.slot_off, nullptr, 0, nullptr, nullptr, nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[1], s);
    hipLaunchKernelGGL(k_encode_fast, dim3((unsigned)((a.n + K1_WAVES - 1) / K1_WAVES)), dim3(64 * K1_WAVES), 0, s, a,
                       (uint64_t)0, a.n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.defer_records)
        hipLaunchKernelGGL(k_encode_var<VAR_DEFER>, dim3((unsigned)var_blocks(a.n)), dim3(64 * K1_WAVES), 0, s, a,
                           (uint64_t)0, a.n);
    else
        hipLaunchKernelGGL(k_encode_var<VAR_PLAIN>, dim3((unsigned)var_blocks(a.n)), dim3(64 * K1_WAVES), 0, s, a,
                           (uint64_t)0, a.n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[2], s);
    // (deferred records: sizes flagged VCFCD_DEFER masked, their tiles
    // flagged for the compaction, and the out_cap report held back -- some
    // sizes may be predictions)
    if (a.defer_records)
        hipLaunchKernelGGL((k_scan_lb<2, true>), dim3((unsigned)nt), dim3(SCAN_THREADS), 0, s, a.rec_size, a.n,
                           tickets + 1, flags_b, a.rec_off, a.tile_first, a.out_cap, a.nospace, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_scan_lb<0, true>), dim3((unsigned)nt), dim3(SCAN_THREADS), 0, s, a.rec_size, a.n,
                           tickets + 1, flags_b, a.rec_off, a.tile_first, a.out_cap, a.err, nullptr, nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[3], s);
    // a grid of 8 waves per SIMD striding over the output tiles (uniform work)
    const uint64_t tiles = vcfc_record_bound(a.n, a.line_bytes_hint) / CT + 1;
    const uint64_t cblocks = tiles < 8192 ? (tiles + 3) / 4 : 2048;
    hipLaunchKernelGGL(k_compact_out, dim3((unsigned)cblocks), dim3(256), 0, s, a.prim, a.slots, a.slot_off,
                       a.rec_off, a.n, a.tile_first, a.out, a.out_cap, a.prim_bytes, nullptr, a.rec_size,
                       a.defer_records ? a.defer_count : nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[4], s);
    // the deferred rows' records, straight into out (a resident grid; exits
    // at once when k_encode_var deferred none)
    if (a.defer_records) {
        const uint64_t dblocks = (a.n + K1_WAVES - 1) / K1_WAVES;
        const dim3 dgrid((unsigned)(dblocks < DEFER_BLOCKS ? dblocks : DEFER_BLOCKS));
        hipLaunchKernelGGL(k_encode_defer<1>, dgrid, dim3(64 * K1_WAVES), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // after a misprediction: the layout again on exact sizes (three
        // launches that return at once otherwise)
        hipLaunchKernelGGL((k_scan_lb<2, true>), dim3((unsigned)nt), dim3(SCAN_THREADS), 0, s, a.rec_size, a.n,
                           tickets + 1, flags_b, a.rec_off, a.tile_first, a.out_cap, a.err, a.mispredict, a.nospace);
        hipLaunchKernelGGL(k_compact_out, dim3((unsigned)cblocks), dim3(256), 0, s, a.prim, a.slots, a.slot_off,
                           a.rec_off, a.n, a.tile_first, a.out, a.out_cap, a.prim_bytes, a.mispredict, a.rec_size,
                           a.defer_count);
        hipLaunchKernelGGL(k_encode_defer<2>, dgrid, dim3(64 * K1_WAVES), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (ev) (void)hipEventRecord(ev[5], s);
    return hipSuccess;
}

hipError_t vcfc_scan_u32(const uint32_t *in, uint64_t n, uint64_t *partials, uint64_t *out, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(out, 0, 8, s);
    return launch_scan<0>(in, n, partials, out, s);
}

hipError_t vcfc_scan_kinds(const uint32_t *in, uint64_t n, uint64_t *partials, uint64_t *out, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(out, 0, 8, s);
    return launch_scan<3>(in, n, partials, out, s);
}
