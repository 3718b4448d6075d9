// vcfc_ingest.hip -- GPU line index of an input chunk (the
// device counterpart of compress()'s getline loop, reference
// src/compress.cpp:218-238).
//
// A chunk is a run of whole lines resident in HBM (every line ends with
// '\n'; the host appends one after an unterminated last line of the file, as
// getline still returns it).  The index gives, in line order:
//   data lines   (non-empty, first byte not '#'): offset, length, line number
//                -- exactly the encoder's input arrays;
//   pass lines   (first byte '#'): offset, length, line number and the count
//                of data lines before it (where it sits in the output);
// empty lines are skipped (compress.cpp:219-221) but still counted.
//
//   k_nl_scan     one wave per 16 KiB segment, the only pass over the bytes:
//                 '\n' count, and the first NL_SLOT positions in order into
//                 the segment's slot (per-lane masks, a wave prefix sum of
//                 their popcounts)
//   k_nl_hop      (instead, when the header gives the sample count: line ends
//                 guessed and checked, ~0.5 KiB read per line; see below)
//   scan          segment bases (the encoder's exclusive scan)
//   k_nl_place    one lane per segment: its positions from the slot to their
//                 place, and the kind of the line after each (its first
//                 byte: data, '#' or empty); a segment with more than
//                 NL_SLOT lines (average line < 64 bytes: header lines) scans
//                 its bytes again
//   scan          data and '#' line ranks, two counts in one word
//   k_line_place  one lane per line: scatter into the output arrays (the
//                 last lane: the counts)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

// Diagnostic builds (tests/simt_emu) pass -DVCFC_DIAG='"hooks.h"'; the
// product build defines the hook empty.
#ifdef VCFC_DIAG
#include VCFC_DIAG
#endif
#ifndef VCFC_DIAG_HOP_READ
#define VCFC_DIAG_HOP_READ(bytes)   // bytes a walker loads in one round (emulator diagnostics)
#endif

namespace {

constexpr uint32_t SEG = 16384;          // bytes per wave
constexpr uint32_t WIN = 1024;           // bytes per wave step (16 per lane)
constexpr uint32_t IX_WAVES = 4;
constexpr uint32_t NL_SLOT = 128;        // '\n' positions kept per segment by k_nl_scan
// A slot entry's top bits (the hop index): 1 + the kind of the line after
// that '\n' when the walker saw its first byte, else 0 (k_nl_place reads it)
constexpr uint32_t SLOT_KIND = 62;
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// bit j: byte j of x is '\n' (exact per byte)
__device__ __forceinline__ uint32_t nl_bits(uint32_t x) {
    const uint32_t t = x ^ 0x0A0A0A0Au;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// 16-bit '\n' mask of bytes [p, p + 16) (bytes at or past n count as none)
__device__ __forceinline__ uint32_t nl_mask16(const uint8_t *buf, uint64_t n, uint64_t p) {
    if (p + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + p);
        return nl_bits(v.x) | nl_bits(v.y) << 4 | nl_bits(v.z) << 8 | nl_bits(v.w) << 12;
    }
    uint32_t m = 0;
    for (uint32_t j = 0; j < 16 && p + j < n; j++) m |= (buf[p + j] == '\n' ? 1u : 0u) << j;
    return m;
}

// kind of the line starting at byte x (phase 2): 1 data, 2 '#', 0 empty (or none: x = n)
__device__ __forceinline__ uint32_t line_kind_at(const uint8_t *buf, uint64_t n, uint64_t x) {
    const uint32_t c = x < n ? buf[x] : '\n';
    return c == '\n' ? 0u : c == '#' ? 2u : 1u;
}

// positions of the '\n' bytes of one 1 KiB window (lane l: bytes [p, p + 16))
// at out[o0 + rank] for ranks below `lim`; returns the window's count.
// kind (phase 2): kind[rank + 1] = the kind of the line after each.
__device__ __forceinline__ uint32_t nl_window(const uint8_t *buf, uint64_t n, uint64_t p, uint64_t *out, uint64_t o0,
                                              uint64_t lim, uint32_t *kind = nullptr) {
    uint32_t m = nl_mask16(buf, n, p);
    const uint32_t c = __builtin_popcount(m);
    const uint32_t inc = vw::scan_add(c);
    uint64_t o = o0 + inc - c;
    while (m && o < lim) {
        const uint64_t x = p + (uint64_t)__builtin_ctz(m);
        if (kind) kind[o + 1] = line_kind_at(buf, n, x + 1);
        out[o++] = x;
        m &= m - 1;
    }
    return vw::readlane(inc, 63);
}

// '\n' mask of a lane's 16 bytes already loaded
__device__ __forceinline__ uint32_t nl_mask_v(uint4 v) {
    return nl_bits(v.x) | nl_bits(v.y) << 4 | nl_bits(v.z) << 8 | nl_bits(v.w) << 12;
}

// One pass over the segment: all its loads are issued before the first
// window is processed (16 x 16 B per lane in flight), except in the chunk's
// last segment, whose bytes past n must not be read as 16-byte blocks.
__global__ __launch_bounds__(256) void k_nl_scan(const uint8_t *buf, uint64_t n, uint64_t n_seg, uint32_t *seg_cnt,
                                                 uint64_t *slot) {
    const uint64_t seg = (uint64_t)blockIdx.x * IX_WAVES + vw::readfirst(threadIdx.x >> 6);
    if (seg >= n_seg) return;
    const uint32_t l = vw::lane_id();
    uint64_t *sl = slot + seg * NL_SLOT;
    uint32_t c = 0;
    if ((seg + 1) * SEG > n) {
        for (uint32_t w = 0; w < SEG; w += WIN) c += nl_window(buf, n, seg * SEG + w + 16 * l, sl, c, NL_SLOT);
    } else {
        constexpr uint32_t NW = SEG / WIN;
        uint4 v[NW];
        const uint4 *src = reinterpret_cast<const uint4 *>(buf + seg * SEG) + l;
#pragma unroll
        for (uint32_t k = 0; k < NW; k++) v[k] = src[k * (WIN / 16)];
#pragma unroll
        for (uint32_t k = 0; k < NW; k++) {
            uint32_t m = nl_mask_v(v[k]);
            const uint32_t cnt = __builtin_popcount(m);
            const uint32_t inc = vw::scan_add(cnt);
            uint32_t o = c + inc - cnt;
            const uint64_t p = seg * SEG + k * WIN + 16 * l;
            while (m && o < NL_SLOT) {
                sl[o++] = p + (uint64_t)__builtin_ctz(m);
                m &= m - 1;
            }
            c += vw::readlane(inc, 63);
        }
    }
    if (l == 0) seg_cnt[seg] = c;
}

// ---------------------------------------------------------------------------
// Hop index (compress_device when the header gives the sample count S): the
// same per-segment output as k_nl_scan without reading every byte.  A wave
// holds HOPW walkers of 16 lanes; walker w walks the lines that end in its
// span of `wseg` segments, one round trip per line:
//   LINE    the line's first MW bytes (256..1024: the previous line's prefix
//           length + 96, rounded up) and a 256-byte guess window around where
//           the line would end if its prefix were as long as the previous
//           line's.  A '\n' in the first window is the end.  Else the 9th TAB
//           gives gt0 (the first sample byte) and the end is predicted at
//           e = gt0 + 4 S - 1 (every token 3 bytes + TAB): taken when byte e
//           is '\n' and the 31 bytes 4, 8, ..., 124 before it are TABs; if
//           the guess window missed e, VERIFY loads the 256 bytes ending at e
//           next round.  No 9th TAB in MW < 1024 bytes: the line again with
//           1 KiB.  '#' lines, prefixes over 1 KiB, a failed check: TRY, or
//           FIND when there is nothing to try.
//   TRY     (round 4) genotype regions of other lengths: the walker keeps
//           HOP_K learned candidates -- a region length G and the TAB mask of
//           the 256 bytes ending at that line's '\n' -- and tries them in
//           turn: taken when the window ending at gt0 + G holds exactly that
//           TAB mask and its only '\n' is the last byte.  Rows whose token
//           lengths are a per-column trait (haploid males, '.' for the same
//           samples) or fixed-width (GT:DP:GQ with two-digit DP/GQ) repeat
//           one G per row kind, so a law-2 file is hopped too.
//   FIND    the next 1 KiB scanned for its first '\n'.  (The walker's
//           start, the first '\n' at or after its span's first byte - 1,
//           comes from k_nl_hop_start, round 6: a wave per walker scanning
//           4 KiB a step, ahead of the walk.)
//   LEARN   after FIND ended a data line whose region is >= 256 bytes: the
//           256 bytes ending at its '\n' become a candidate (round robin).
//   GUESS   (round 6; walkers without TRY / LEARN, the chr22-shaped files)
//           after a data line of L >= 512 bytes found by LINE / VERIFY: the
//           next HOP_G lines (HOP_GL when every walker of the wave guesses:
//           a lean round with nothing else in it) are guessed to be L bytes
//           long, L the mean of the lines guessed so far, and one 256-byte
//           window around each guessed end is loaded in one round -- no
//           prefix, no 9th TAB.  Window k's line is taken when the
//           window holds exactly one '\n', at least 64 bytes in, with TABs
//           at the 15 places 4, 8, ..., 60 before it, and its line is a
//           data line (its first byte, from the round's head load or the
//           previous window, is neither '#' nor '\n'); the first window that
//           fails ends the round and its line goes to LINE.  Lines whose
//           lengths vary by less than ~100 bytes from one to the next (a
//           chr22 prefix varies by tens) take one round per HOP_G lines.
// A walker whose TRYs keep failing (HOP_TRUST misses more than hits) stops
// trying and learning: lines of random lengths cost what they did before.
// Loads are 16 B per lane over contiguous 256-byte rows (coalesced).  A
// chr22-shaped file is read for ~0.5 KiB per line instead of every byte.
// A line predicted across a '\n' it did not see (a shorter line whose guessed
// end lands on a later line's '\n' with TABs at the checked places) is
// caught by the encoder (VcfcEncodeArgs::nl_check), and the chunk is indexed
// again by k_nl_scan.
constexpr uint32_t HOPW = 4;                   // walkers per wave
// (devfile step: 16384 +1.2 %, 8192 +4.6 %; round 6: 65536 +1.9 %, 131072 +3.0 %,
// profiles/r06/ab/ab_r6dev_law1.txt -- more walkers, more FIND starts)
#ifndef VCFC_HOP_WALKERS
#define VCFC_HOP_WALKERS 32768
#endif
constexpr uint64_t HOP_WALKERS = VCFC_HOP_WALKERS;
constexpr uint32_t GW = 256;                   // guess window (16 B per lane)
constexpr uint32_t HOP_LINE = 0, HOP_VERIFY = 1, HOP_FIND = 2, HOP_DONE = 3, HOP_TRY = 4, HOP_LEARN = 5, HOP_GUESS = 6;
constexpr uint32_t HOP_G = 4;                  // lines guessed per GUESS round (one window each) ...
#ifndef VCFC_HOP_GL
#define VCFC_HOP_GL 4
#endif
constexpr uint32_t HOP_GL = VCFC_HOP_GL;       // ... in a lean round (every walker of the wave guessing)
constexpr uint32_t GUESS_MIN = 512;            // line length below which GUESS is not used
constexpr uint32_t GUESS_LEAD = 160;           // a guessed end's window starts this far before it
constexpr uint32_t HOP_K = 3;                  // learned candidates per walker
constexpr uint32_t HOP_TRUST = 8;              // TRY credit: +1 per hit (capped), -1 per all-miss

// 16 bytes at p (bytes at or past n read as 0)
__device__ __forceinline__ uint4 load16(const uint8_t *buf, uint64_t n, uint64_t p) {
    if (p + 16 <= n) return *reinterpret_cast<const uint4 *>(buf + p);
    uint4 v = make_uint4(0, 0, 0, 0);
    for (uint32_t j = 0; j < 16 && p + j < n; j++)
        (j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w) |= (uint32_t)buf[p + j] << (8 * (j & 3));
    return v;
}
__device__ __forceinline__ uint32_t tab_mask_v(uint4 v) {   // ('\t' = '\n' ^ 0x03)
    return nl_bits(v.x ^ 0x03030303u) | nl_bits(v.y ^ 0x03030303u) << 4 | nl_bits(v.z ^ 0x03030303u) << 8 |
           nl_bits(v.w ^ 0x03030303u) << 12;
}
// byte j (0..15) of a lane's 16 bytes
__device__ __forceinline__ uint32_t byte16(uint4 v, uint32_t j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3u))) & 0xFFu;
}
// inclusive sum over the lane's 16-lane walker
__device__ __forceinline__ uint32_t walker_scan(uint32_t v) {
    const uint32_t l = vw::lane_id();
#pragma unroll
    for (uint32_t d = 1; d < 16; d <<= 1) {
        const uint32_t y = vw::shfl(v, (l - d) & 63u);
        if ((l & 15u) >= d) v += y;
    }
    return v;
}

// Each walker's first line end: the first '\n' at or after its span's first
// byte - 1 (walker 0: none, it starts at byte 0), or ~0 when there is none
// before the span's end.  One wave per walker, 4 KiB per step (64 lanes x
// 4 x 16 B): lines of ~10 KB cost ~2 steps here instead of ~5 of the walk's
// 1 KiB FIND rounds at the start of every span (the walk's own layout, four
// walkers of 16 lanes a wave at 4 KiB a step, was slower: 89 against 60 us
// on the config-2 file).
__global__ __launch_bounds__(256) void k_nl_hop_start(const uint8_t *buf, uint64_t n, uint64_t n_seg, uint32_t wseg,
                                                      uint64_t walkers, uint64_t *wstart) {
    const uint32_t l = vw::lane_id();
    const uint64_t walker = (uint64_t)blockIdx.x * IX_WAVES + vw::readfirst(threadIdx.x >> 6);
    if (walker >= walkers) return;
    const uint64_t sg0 = walker * wseg, lo = sg0 * SEG, hi = umin64((sg0 + wseg) * SEG, n);
    if (sg0 >= n_seg || lo == 0) {
        if (l == 0) wstart[walker] = ~0ull;
        return;
    }
    uint64_t found = ~0ull;
    for (uint64_t c = lo - 1; c < hi && found == ~0ull; c += 4096) {
        uint32_t m[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) m[j] = nl_mask_v(load16(buf, n, c + 1024u * j + 16u * l));
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint64_t b = vw::ballot(m[j] != 0);
            if (b && found == ~0ull) {
                const uint32_t f = (uint32_t)__builtin_ctzll(b);
                found = c + 1024u * j + 16u * f + (uint32_t)__builtin_ctz(vw::readlane(m[j], f));
            }
        }
    }
    if (l == 0) wstart[walker] = found < hi ? found : ~0ull;
}

// LEARN (TRY / LEARN compiled in) is chosen by the host when the first data
// lines of the file are not all 3-byte-token lines: the candidate state puts
// the walker at 116 VGPRs (4 waves per SIMD; pinned to 5 it spills 16
// dwords) and costs the configs[1] device file +3.7 %, while law-2 files go
// 16.5 -> 13.7 ms (profiles/r04/ab/ab_tall_law*.txt); without it the walker
// is round 3's (86 VGPRs, 5 waves).
template <bool LEARN, bool NOSTORE = false>   // (NOSTORE: VCFC_DIAG_HOP_TWICE's timing copy)
// (round 6: pinned to 6 waves per SIMD, 80 VGPRs and a 12-byte spill, the
// same speed; to 8, 64 VGPRs and 72 bytes spilled, +4 %:
// profiles/r06/ab/ab_r6hop_devfile_law1.txt)
__global__ __launch_bounds__(256) void k_nl_hop(const uint8_t *buf, uint64_t n, uint64_t n_seg, uint32_t S,
                                                uint32_t wseg, const uint64_t *wstart, uint32_t *seg_cnt,
                                                uint64_t *slot, uint32_t L0, VcfcHopCands hc) {
    const uint32_t l = vw::lane_id(), wl = l & 15u, w0 = l & ~15u, sh = l & 48u;   // w0: the walker's first lane
    const uint64_t walker = ((uint64_t)blockIdx.x * IX_WAVES + (threadIdx.x >> 6)) * HOPW + (l >> 4);
    const uint64_t sg0 = walker * wseg;                              // the walker's first segment
    const uint64_t lo = sg0 * SEG, hi = umin64((sg0 + wseg) * SEG, n);
    const uint32_t nseg = sg0 >= n_seg ? 0u : (uint32_t)umin64(wseg, n_seg - sg0);
    uint32_t mode = nseg == 0 ? HOP_DONE : HOP_LINE;
    uint64_t p = 0, q = 0, e = 0;
    uint32_t pl = 0, rows = 4;          // previous prefix length; 256-byte rows of the next LINE window
    uint32_t L = 0;                     // GUESS: the guessed line length ('\n' included)
    uint64_t gs0 = 0;                   // GUESS: the streak's first line start ...
    uint32_t gn = 0;                    // ... and its lines so far
    uint32_t cur = 0, cc = 0;           // current segment (in the span) and its count
    // learned candidates (walker-uniform lengths; this lane's 16-bit TAB mask of each)
    // (round 6: seeded with the host's candidates from the file's first
    // lines, so a wave need not FIND and LEARN each row kind first)
    uint32_t cg[HOP_K] = {hc.g[0], hc.g[1], hc.g[2]};
    uint32_t csig[HOP_K] = {hc.sig[0][wl], hc.sig[1][wl], hc.sig[2][wl]};
    uint32_t ins = (hc.g[0] != 0) + (hc.g[1] != 0) + (hc.g[2] != 0), trust = HOP_TRUST;
    ins = ins == HOP_K ? 0u : ins;
    uint64_t gt = 0;                    // the current data line's gt0 (lrn: it may be learned)
    bool lrn = false, tdef = false;     // tdef: the TRY round also checks the 3-byte end e (VERIFY's job)
    // (the walker's lanes; lo <= x < hi, in order).  kh: the kind of the
    // line after x when the walker saw its first byte (SLOT_KIND), else 0
    uint64_t nsacc = 0;                 // (NOSTORE: the positions' checksum, the walk's only output)
    auto record = [&](uint64_t x, uint32_t kh = 0) {
        const uint32_t k = (uint32_t)((x - lo) / SEG);
        if (NOSTORE) nsacc = nsacc * 31u + x + kh + cur + cc;
        for (; cur < k; cur++, cc = 0)
            if (!NOSTORE && l == w0) seg_cnt[sg0 + cur] = cc;
        if (!NOSTORE && l == w0 && cc < NL_SLOT) slot[(sg0 + cur) * NL_SLOT + cc] = x | ((uint64_t)kh << SLOT_KIND);
        cc++;
    };
    auto wbits = [&](bool pr) { return (uint32_t)(vw::ballot(pr) >> sh) & 0xFFFFu; };
    // the walker's first line end (k_nl_hop_start): the walk starts after it,
    // guessing from L0 (the host's first data line; as if a line of that
    // length ended at p - 1) when there is one
    if (mode != HOP_DONE && lo != 0) {
        const uint64_t e0 = wstart[walker];
        if (e0 == ~0ull) mode = HOP_DONE;
        else {
            if (e0 >= lo) record(e0);
            p = e0 + 1;
            const bool g = !LEARN && L0 >= GUESS_MIN;
            L = g ? L0 : L;
            gs0 = p - L0;   // (mod 2^64: s - gs0 stays exact)
            gn = 1;
            mode = p >= hi ? HOP_DONE : g ? HOP_GUESS : HOP_LINE;
        }
    }
    // learned candidates to try (trusted walkers, data lines only)
    auto have_cand = [&]() { return LEARN && lrn && trust != 0 && (cg[0] | cg[1] | cg[2]) != 0; };
    // a failed prediction: the candidates, else FIND from fq
    auto to_try = [&](uint64_t fq) {
        q = fq;
        tdef = false;
        mode = have_cand() ? HOP_TRY : HOP_FIND;
    };
    // GUESS steps of one round (wave-uniform call; act: the walker was
    // guessing at the round's start, v / hd its windows and head byte):
    // the windows in order while they hold (collectives for every window; a
    // walker takes its lines up to the first window that fails)
    auto guess_round = [&](auto ng, const uint4 *v, uint32_t hd, bool act) {
        constexpr uint32_t NG = decltype(ng)::value;   // windows this round
        bool go = act && hd != '#' && hd != '\n';   // the line at p is a data line
        uint32_t nextm = go ? HOP_GUESS : HOP_LINE;   // the mode after this round
        uint64_t s = p;          // the current line's start
        const uint32_t Lw = L;   // the windows' line length
#pragma unroll
        for (uint32_t k = 0; k < NG; k++) {
            const uint64_t ws = p - 1 + (uint64_t)(k + 1) * Lw - GUESS_LEAD;   // (mode0 GUESS: L >= 512, p >= 1)
            const uint32_t m = nl_mask_v(v[k]);
            const uint32_t b = wbits(m != 0);
            const uint32_t f = b ? (uint32_t)__builtin_ctz(b) : 0u;
            const uint32_t mf = vw::shfl(m, w0 + f);
            const uint32_t jf = 16u * f + (uint32_t)__builtin_ctz(mf | 0x10000u);   // the '\n', window-relative
            const bool one = b != 0 && (b & (b - 1)) == 0 && (mf & (mf - 1)) == 0 && jf >= 64;
            // TABs at jf - 4 i (i = 1..15): this lane's bytes [16 wl, 16 wl + 16) inside [jf - 60, jf)
            const int32_t r0 = (int32_t)jf - 60 - (int32_t)(16u * wl), r1 = (int32_t)jf - (int32_t)(16u * wl);
            const uint32_t lo4 = (uint32_t)(r0 < 0 ? 0 : r0 > 16 ? 16 : r0), hi4 = (uint32_t)(r1 < 0 ? 0 : r1 > 16 ? 16 : r1);
            const uint32_t rm = ((1u << hi4) - 1u) & ~((1u << lo4) - 1u);
            const uint32_t want = (0x1111u << ((uint32_t)r1 & 3u)) & rm;
            const bool tabs_ok = (tab_mask_v(v[k]) & want) == want;
            const uint32_t tbad = wbits(!tabs_ok);   // (collectives stay wave-uniform)
            const bool hit = one && tbad == 0;
            // the next line's first byte (window byte jf + 1; none past the window)
            const uint32_t jn = jf + 1;
            const uint32_t nb = vw::shfl(byte16(v[k], jn & 15u), w0 + ((jn >> 4) & 15u));
            const uint64_t e = ws + jf;
            if (go) {
                if (!hit || e <= s) {   // the guess failed: this line by LINE
                    nextm = HOP_LINE;
                    go = false;
                } else if (e >= hi) {
                    nextm = HOP_DONE;
                    go = false;
                } else {
                    // (the next line's kind, when its first byte is in the window)
                    record(e, jn < GW ? (nb == '\n' ? 1u : nb == '#' ? 3u : 2u) : 0u);
                    s = e + 1;
                    gn++;
                    // the next line: past the span, its first byte not in
                    // this window (the next round's head load checks it),
                    // a '#' or empty line (LINE), or a data line (go on)
                    if (s >= hi) { nextm = HOP_DONE; go = false; }
                    else if (jn >= GW) go = false;
                    else if (nb == '#' || nb == '\n') { nextm = HOP_LINE; go = false; }
                }
            }
        }
        if (act) {
            mode = nextm;
            p = s;
            // the next windows: the mean length of the streak's lines (a
            // chr22 prefix varies by ~9 bytes from line to line: guessed from
            // the last line alone, 8 lines ahead drift past the window's
            // +-96 bytes in 5 % of rounds, from the mean in 0.1 %)
            L = (uint32_t)((float)(s - gs0) / (float)gn + 0.5f);
        }
    };
    while (vw::ballot(mode != HOP_DONE)) {
        if (!LEARN) {
            // every walker of the wave guessing or done: lean rounds -- the
            // windows, the head byte and the GUESS steps, nothing else
            while (vw::ballot(mode != HOP_GUESS && mode != HOP_DONE) == 0 && vw::ballot(mode == HOP_GUESS) != 0) {
                const bool act = mode == HOP_GUESS;
                uint4 w[HOP_GL];
#pragma unroll
                for (uint32_t k = 0; k < HOP_GL; k++)
                    w[k] = act ? load16(buf, n, p - 1 + (uint64_t)(k + 1) * L - GUESS_LEAD + 16u * wl) : make_uint4(0, 0, 0, 0);
                const uint32_t hd = act && p < n ? buf[p] : 0u;
                if (l == w0 && act) VCFC_DIAG_HOP_READ(256u * HOP_GL + 1u);
                guess_round(std::integral_constant<uint32_t, HOP_GL>(), w, hd, act);
            }
            if (vw::ballot(mode != HOP_DONE) == 0) break;
        }
        const uint32_t mode0 = mode;   // (the round's mode: the steps below may switch it for the next round)
        // ---- loads: the main window (LINE: `rows` rows, FIND: 4), the guess window ----
        const uint64_t base = mode == HOP_FIND ? q : p;
        const uint32_t nr = mode == HOP_FIND ? 4u : mode == HOP_LINE ? rows : 0u;
        // (TRY: rows 0..2 hold the 256 bytes ending at each learned
        // candidate's end gt0 + G_k, all tried in one round)
        // (GUESS: rows 0..3 are the windows of the next HOP_G guessed ends,
        // window k from p - 1 + (k + 1) L - GUESS_LEAD; hd = the line's first byte)
        const bool gm = !LEARN && mode == HOP_GUESS;
        uint4 v[4];
        uint32_t cvalid = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t G = k == 0 ? cg[0] : k == 1 ? cg[1] : cg[2];
            const bool cv = LEARN && k < 3 && mode == HOP_TRY && G != 0 && gt + G + 1 >= GW && gt + G < n;
            cvalid |= cv ? 1u << k : 0u;
            v[k] = k < nr ? load16(buf, n, base + 256u * k + 16u * wl)
                   : gm   ? load16(buf, n, p - 1 + (uint64_t)(k + 1) * L - GUESS_LEAD + 16u * wl)
                   : cv ? *reinterpret_cast<const uint4 *>(buf + gt + G + 1 - GW + 16u * wl) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t hd = gm && p < n ? buf[p] : 0u;
        uint64_t g0 = 0;
        bool gok = true;   // (VERIFY / TRY / LEARN: the window ends at e = g0 + GW - 1)
        if (mode == HOP_LINE) {
            const uint64_t x = p + pl + 4ull * S - 1;   // the end if the prefix is as long as the last one
            g0 = x >= GW / 2 + 62 ? x - (GW / 2 + 62) : 0;
        } else if (mode == HOP_VERIFY || mode == HOP_LEARN || (mode == HOP_TRY && tdef)) {
            gok = e + 1 >= GW;
            g0 = gok ? e + 1 - GW : 0;
        } else {
            gok = false;
        }
        const bool gv = mode != HOP_FIND && mode != HOP_DONE && g0 + GW <= n && gok;
        const uint4 ga = gv ? *reinterpret_cast<const uint4 *>(buf + g0 + 16u * wl) : make_uint4(0, 0, 0, 0);
        if (l == w0 && mode != HOP_DONE)
            VCFC_DIAG_HOP_READ(256u * nr + (gv ? GW : 0u) + GW * (uint32_t)__builtin_popcount(cvalid) + (gm ? 256u * HOP_G + 1u : 0u));
        // ---- the first '\n' of the main window (row-major: row k, then lane) ----
        uint64_t first = ~0ull;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t m = nl_mask_v(v[k]);
            const uint32_t b = wbits(m != 0);
            const uint32_t f = b ? (uint32_t)__builtin_ctz(b) : 0u;
            const uint32_t mf = vw::shfl(m, w0 + f);   // (collectives stay wave-uniform)
            if (b && first == ~0ull) first = base + 256u * k + 16u * f + (uint32_t)__builtin_ctz(mf | 0x10000u);
        }
        bool found = false, check = false;
        if (mode == HOP_FIND) {
            if (first != ~0ull) { e = first; found = true; }
            else if (q + 1024 >= n) { e = n - 1; found = true; }   // (buf[n - 1] is '\n')
            else q += 1024;
            // a data line the candidates did not know: learn its region
            if (LEARN && found && lrn && trust && e >= gt + GW - 1) { found = false; mode = HOP_LEARN; }
        }
        // ---- TRY / LEARN (wave-uniform branches: a wave of 3-byte-token
        // lines pays nothing for them).  TRY: candidate k holds when the
        // window ending at gt0 + G_k has exactly its TAB mask and its only
        // '\n' is the last byte ----
        uint32_t chit = 0;   // the region length of the first candidate that holds (0: none)
        if (LEARN && vw::ballot(mode0 == HOP_TRY || mode0 == HOP_LEARN)) {
            const uint32_t gtm = tab_mask_v(ga);
#pragma unroll
            for (uint32_t k = 0; k < 3; k++) {
                const uint32_t sg = k == 0 ? csig[0] : k == 1 ? csig[1] : csig[2];
                const bool tok = ((cvalid >> k) & 1u) && tab_mask_v(v[k]) == sg &&
                                 nl_mask_v(v[k]) == (wl == 15 ? 0x8000u : 0u);
                const bool hk = wbits(!tok) == 0;   // (collectives stay wave-uniform)
                // (the length itself: a LEARN below may replace the slot this round)
                const uint32_t G = k == 0 ? cg[0] : k == 1 ? cg[1] : cg[2];
                if (hk && chit == 0 && mode0 == HOP_TRY) chit = G;
            }
            // LEARN: every walker of the wave takes the lowest learner's
            // candidate (a law-2 row kind is learned once per wave, not once
            // per walker), a learner also its own; a length already held is
            // not taken again
            auto insert = [&](uint32_t G, uint32_t sg) {
                if (G == cg[0] || G == cg[1] || G == cg[2]) return;
                if (ins == 0) { cg[0] = G; csig[0] = sg; }
                else if (ins == 1) { cg[1] = G; csig[1] = sg; }
                else { cg[2] = G; csig[2] = sg; }
                ins = ins + 1 == HOP_K ? 0u : ins + 1;
            };
            const uint64_t lm = vw::ballot(mode0 == HOP_LEARN && gv);
            if (lm) {
                const uint32_t sw0 = (uint32_t)__builtin_ctzll(lm) & ~15u;
                const uint32_t Gown = (uint32_t)(e - gt);
                const uint32_t Gs = vw::shfl(Gown, sw0), ss = vw::shfl(gtm, sw0 + wl);
                insert(Gs, ss);
                if (mode0 == HOP_LEARN && gv) insert(Gown, gtm);
            }
        }
        if (mode0 == HOP_LEARN) found = true;
        // ---- LINE: the 9th TAB, the predicted end ----
        uint32_t t9 = ~0u, acc = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const bool act = k < nr && mode == HOP_LINE && first == ~0ull && t9 == ~0u;
            if (vw::ballot(act)) {   // (wave-uniform: walkers without work compute and drop)
                const uint32_t tm = act ? tab_mask_v(v[k]) : 0u;
                const uint32_t c = (uint32_t)__builtin_popcount(tm);
                const uint32_t inc = walker_scan(c) + acc;
                const bool has9 = act && inc - c < 9 && inc >= 9;
                uint32_t mm = tm;
                for (uint32_t r = inc - c; has9 && r < 8; r++) mm &= mm - 1;
                const uint32_t hb = wbits(has9);
                const uint32_t tl = 256u * k + 16u * wl + (uint32_t)__builtin_ctz(mm | 0x10000u);
                const uint32_t t9n = vw::shfl(tl, w0 + (hb ? (uint32_t)__builtin_ctz(hb) : 0u));
                if (hb) t9 = t9n;
                acc = vw::shfl(inc, w0 + 15);
            }
        }
        const uint32_t b0 = vw::shfl(v[0].x & 0xFFu, w0);
        if (mode == HOP_LINE) {
            lrn = false;
            if (first != ~0ull) { e = first; found = true; }
            else if (S == 0 || b0 == '#') { mode = HOP_FIND; q = p + 256u * rows; }
            else if (t9 == ~0u) {
                if (rows < 4) rows = 4;                              // the line again with 1 KiB
                else { mode = HOP_FIND; q = p + 1024; }
            } else {
                pl = t9 + 1;
                const uint32_t want = pl + 96;
                rows = want <= 256 ? 1u : want <= 512 ? 2u : 4u;
                gt = p + t9 + 1;
                lrn = true;
                e = p + t9 + 4ull * S;   // gt0 + 4 S - 1
                if (e >= n) to_try(p + 256u * nr);
                else if (gv && e >= g0 + 124 && e < g0 + GW) check = true;
                else if (have_cand()) {   // (the TRY round checks e too: VERIFY's window)
                    mode = HOP_TRY;
                    tdef = true;
                    q = p + 256u * nr;
                } else mode = HOP_VERIFY;
            }
        } else if (mode == HOP_VERIFY) {
            if (gv && e >= g0 + 124) check = true;
            else to_try(p);
        } else if (mode == HOP_TRY && tdef && gv) {
            check = true;
        }
        // ---- the check: byte e is '\n', bytes e - 4 i (i = 1..31) TABs ----
        bool bad = false;
        if (check) {
            const uint32_t s8 = 8u * (uint32_t)((e - g0) & 3u);
            const uint32_t gw[4] = {ga.x, ga.y, ga.z, ga.w};
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t a = g0 + 16u * wl + 4u * j + ((e - g0) & 3u);
                const uint32_t want = a == e ? 0x0Au : 0x09u;
                bad |= a + 124 >= e && a <= e && ((gw[j] >> s8) & 0xFFu) != want;
            }
        }
        const bool bw = wbits(bad) != 0;
        if (check) {
            if (!bw) found = true;
            else if (mode0 != HOP_TRY) to_try(p + 256u * nr);   // (past the first window: no '\n' there)
        }
        if (mode0 == HOP_TRY && !found) {   // the 3-byte end failed: the first candidate that holds
            if (chit) {
                e = gt + chit;
                found = true;
                trust = trust < HOP_TRUST ? trust + 1 : trust;
            } else {
                mode = HOP_FIND;   // (q: where the prediction left it)
                trust = trust ? trust - 1 : 0;
            }
        }
        // ---- the line end: record, next line ----
        if (found) {
            if (e >= hi) mode = HOP_DONE;
            else {
                if (e >= lo) record(e);
                // a data line found by LINE / VERIFY: guess the next ones from its length
                const uint64_t Ln = e + 1 - p;
                const bool g = !LEARN && ((mode0 == HOP_LINE && b0 != '#') || mode0 == HOP_VERIFY) && Ln >= GUESS_MIN &&
                               Ln < (1ull << 30);
                L = g ? (uint32_t)Ln : L;
                gs0 = g ? p : gs0;
                gn = g ? 1u : gn;
                p = e + 1;
                mode = p >= hi ? HOP_DONE : g ? HOP_GUESS : HOP_LINE;
            }
        }
        if (!LEARN && vw::ballot(mode0 == HOP_GUESS)) guess_round(std::integral_constant<uint32_t, HOP_G>(), v, hd, mode0 == HOP_GUESS);
    }
    for (; cur < nseg; cur++, cc = 0)
        if (!NOSTORE && l == w0) seg_cnt[sg0 + cur] = cc;
    if (NOSTORE && l == w0 && nsacc == 0x5EED5EED5EED5EEDull) seg_cnt[sg0] = 0;   // (keeps the walk alive)
}

// One wave per 64 segments, one lane per segment (most hold a few lines:
// a wave per segment spent ~0.1 ms launching 622k waves for 8 MB of
// positions); a segment with more lines than its slot holds is scanned
// again by the whole wave, one such segment after the other.
// A line's kind is its first byte, the byte after the previous line's '\n':
// each placed position gives the kind of the line after it, so no lane
// needs another segment's positions (line 0: byte 0, by segment 0's lane).
__global__ __launch_bounds__(256) void k_nl_place(const uint8_t *buf, uint64_t n, uint64_t n_seg, const uint32_t *seg_cnt,
                                                  const uint64_t *slot, const uint64_t *seg_base, uint64_t *nl,
                                                  uint32_t *kind, uint64_t *counts) {
    const uint32_t l = vw::lane_id();
    const uint64_t seg0 = ((uint64_t)blockIdx.x * IX_WAVES + vw::readfirst(threadIdx.x >> 6)) * 64;
    if (seg0 >= n_seg) return;
    const uint64_t seg = seg0 + l;
    const uint32_t c = seg < n_seg ? seg_cnt[seg] : 0u;
    if (seg == 0) kind[0] = line_kind_at(buf, n, 0);
    if (c <= NL_SLOT) {
        const uint64_t *sl = slot + seg * NL_SLOT;
        const uint64_t b = seg < n_seg ? seg_base[seg] : 0;
        uint64_t *dst = nl + b;
        for (uint32_t k = 0; k < c; k++) {
            const uint64_t xs = sl[k], x = xs & ((1ull << SLOT_KIND) - 1);
            const uint32_t kh = (uint32_t)(xs >> SLOT_KIND);
            dst[k] = x;
            kind[b + k + 1] = kh ? kh - 1u : line_kind_at(buf, n, x + 1);
        }
    }
    // more lines than the slot holds: scan the segment again, keeping at
    // most the c positions the count scan made room for.  The hop index may
    // have counted fewer than there are (a guessed end across a line it did
    // not see); the positions kept would then be the segment's first c, and
    // the line after them would swallow a real '\n' -- a '#' line placed
    // verbatim if it starts with '#', which the encoder never checks.  So a
    // count that differs from the scan's marks the index as wrong
    // (counts[3] = 2: the driver indexes the chunk again from every byte).
    for (uint64_t m = vw::ballot(c > NL_SLOT); m; m &= m - 1) {
        const uint32_t f = (uint32_t)__builtin_ctzll(m);
        const uint64_t sf = seg0 + f;
        const uint32_t cf = vw::readlane(c, f);
        uint64_t *dst = nl + seg_base[sf];
        uint32_t o = 0;
        for (uint32_t w = 0; w < SEG; w += WIN) o += nl_window(buf, n, sf * SEG + w + 16 * l, dst, o, cf, kind + seg_base[sf]);
        if (o != cf && l == 0) atomicMax((unsigned long long *)(counts + 3), 2ull);
    }
}

// rank[i] = data lines before line i | '#' lines before it << 32
__global__ __launch_bounds__(256) void k_line_place(const uint64_t *nl, uint64_t n_lines, const uint64_t *rank,
                                                    VcfcLineIndex x) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lines) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0u;
    const uint64_t r0 = rank[i], r1 = rank[i + 1];
    const uint64_t d = (uint32_t)r0, q = r0 >> 32;
    if (i + 1 == n_lines) {   // the counts: data and '#' lines
        x.counts[1] = (uint32_t)r1;
        x.counts[2] = r1 >> 32;
    }
    if (nl[i] - s > 0xFFFFFFFFull) atomicMax((unsigned long long *)(x.counts + 3), 1ull);   // line lengths are 32-bit
    if ((uint32_t)r1 > d) {
        x.line_off[d] = s;
        x.line_len[d] = (uint32_t)(nl[i] - s);
        x.line_no[d] = (uint32_t)i;
    }
    if ((r1 >> 32) > q) {
        x.pass_off[q] = s;
        x.pass_len[q] = (uint32_t)(nl[i] - s);
        x.pass_no[q] = (uint32_t)i;
        x.pass_before[q] = d;
    }
}

// counts[0] = the line count (the segment scan's total), counts[3] = 0 (the
// flags phase 2 raises), in one launch instead of a copy and a memset
__global__ void k_index_counts(const uint64_t *total, uint64_t *counts) {
    if (threadIdx.x == 0) {
        counts[0] = *total;
        counts[3] = 0;
    }
}

}  // namespace

// Phase 1 workspace depends on the chunk size only (every byte may be a
// '\n'); phase 2 on the line count phase 1 found.
VcfcLineIndexLayout vcfc_line_index_layout(uint64_t chunk_bytes, uint64_t n_lines) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t seg = (chunk_bytes + SEG - 1) / SEG + 1;
    VcfcLineIndexLayout L;
    uint64_t o = 0;
    L.seg_cnt = o; o = al(o + 4 * seg);
    L.seg_base = o; o = al(o + 8 * (seg + 1));
    L.slot = o; o = al(o + 8ull * NL_SLOT * seg);
    L.wstart = o; o = al(o + 8 * (seg / 2 + 2));   // hop walkers (each over >= 2 segments)
    L.partials1 = o; o = al(o + 8 * ((seg + 4095) / 4096 + 1));
    L.total1 = o;
    o = 0;
    L.nl = o; o = al(o + 8 * (n_lines + 1));
    L.kind = o; o = al(o + 4 * (n_lines + 1));
    L.rank = o; o = al(o + 8 * (n_lines + 1));
    L.partials2 = o; o = al(o + 8 * ((n_lines + 4095) / 4096 + 1));
    L.total2 = o;
    return L;
}

// Phase 1: '\n' count of buf[0, n) (n <= chunk_bytes of the layout; the
// last byte must be '\n') and the kept positions; x.counts[0] = lines.  Phase 2 needs that count on
// the host (its grids), as the encoder needs the data line count.  The
// output arrays of `x` hold up to n / 2 data lines (a data line has at least
// one byte and its '\n') and n pass lines.
hipError_t vcfc_line_index(const uint8_t *buf, uint64_t n, uint8_t *ws, const VcfcLineIndexLayout &L,
                           const VcfcLineIndex &x, hipStream_t s, uint32_t S_hint, uint64_t hop_walkers,
                           bool hop_learn, uint32_t len_hint, const VcfcHopCands *cands) {
    // ws: phase 1 workspace (L.total1 bytes)
    uint32_t *seg_cnt = reinterpret_cast<uint32_t *>(ws + L.seg_cnt);
    uint64_t *seg_base = reinterpret_cast<uint64_t *>(ws + L.seg_base);
    uint64_t *slot = reinterpret_cast<uint64_t *>(ws + L.slot);
    uint64_t *partials = reinterpret_cast<uint64_t *>(ws + L.partials1);
    hipError_t e;
    if (n == 0) return hipMemsetAsync(x.counts, 0, 24, s);
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    const dim3 sg((unsigned)((n_seg + IX_WAVES - 1) / IX_WAVES)), blk(64 * IX_WAVES);
    if (S_hint >= 32) {
        // spans of wseg segments: about HOP_WALKERS walkers, each over at
        // least 2 segments
        const uint64_t hw = hop_walkers ? hop_walkers : HOP_WALKERS;
        const uint64_t wseg = std::max<uint64_t>(2, (n_seg + hw - 1) / hw);
        const uint64_t walkers = (n_seg + wseg - 1) / wseg;
        const uint64_t per_block = (uint64_t)HOPW * IX_WAVES;
        const dim3 hg((unsigned)((walkers + per_block - 1) / per_block));
        uint64_t *wstart = reinterpret_cast<uint64_t *>(ws + L.wstart);
        hipLaunchKernelGGL(k_nl_hop_start, dim3((unsigned)((walkers + IX_WAVES - 1) / IX_WAVES)), blk, 0, s, buf, n, n_seg,
                           (uint32_t)wseg, walkers, wstart);
        VcfcHopCands hc;
        memset(&hc, 0, sizeof hc);
        if (cands && hop_learn) hc = *cands;
        if (hop_learn)
            hipLaunchKernelGGL(k_nl_hop<true>, hg, blk, 0, s, buf, n, n_seg, S_hint, (uint32_t)wseg, wstart, seg_cnt, slot,
                               0u, hc);
        else {
#ifdef VCFC_DIAG_HOP_TWICE   // (diagnostic timing: the walk once without its stores, then the real one)
            hipLaunchKernelGGL((k_nl_hop<false, true>), hg, blk, 0, s, buf, n, n_seg, S_hint, (uint32_t)wseg, wstart,
                               seg_cnt, slot, len_hint, hc);
#endif
            hipLaunchKernelGGL(k_nl_hop<false>, hg, blk, 0, s, buf, n, n_seg, S_hint, (uint32_t)wseg, wstart, seg_cnt, slot,
                               len_hint, hc);
        }
    }
    else
        hipLaunchKernelGGL(k_nl_scan, sg, blk, 0, s, buf, n, n_seg, seg_cnt, slot);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = vcfc_scan_u32(seg_cnt, n_seg, partials, seg_base, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_index_counts, dim3(1), dim3(64), 0, s, seg_base + n_seg, x.counts);
    return hipGetLastError();
}

// Phase 2, once the host knows the line count (counts[0]): the '\n'
// positions in order, then the data / pass tables; ws1 = phase 1's
// workspace, ws2 = L.total2 bytes for vcfc_line_index_layout(chunk, n_lines).
// The host's view of an index in one D2H (compress_device): counts[0..3],
// then the first pk entries of the '#' line tables -- pass_off, pass_before
// (u64), pass_len, pass_no (u32).  Consecutive small D2H copies each cost
// the GPU ~12 us of idle time on this runtime (profiles/r06/devfile_trace_*).
namespace {
__global__ __launch_bounds__(256) void k_index_summary(const uint64_t *counts, const uint64_t *po, const uint64_t *pb,
                                                       const uint32_t *pl, const uint32_t *pn, uint64_t pk,
                                                       uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t *o64 = reinterpret_cast<uint64_t *>(out);
    if (i < 4) o64[i] = counts[i];
    if (i < pk) {
        o64[4 + i] = po[i];
        o64[4 + pk + i] = pb[i];
        uint32_t *o32 = reinterpret_cast<uint32_t *>(o64 + 4 + 2 * pk);
        o32[i] = pl[i];
        o32[pk + i] = pn[i];
    }
}
}  // namespace

hipError_t vcfc_index_summary(const VcfcLineIndex &x, uint64_t pk, uint8_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_index_summary, dim3((unsigned)((std::max<uint64_t>(pk, 4) + 255) / 256)), dim3(256), 0, s,
                       x.counts, x.pass_off, x.pass_before, x.pass_len, x.pass_no, pk, out);
    return hipGetLastError();
}

hipError_t vcfc_line_index_place(const uint8_t *buf, uint64_t n, uint64_t n_lines, const uint8_t *ws1, uint8_t *ws2,
                                 const VcfcLineIndexLayout &L, const VcfcLineIndex &x, hipStream_t s) {
    const uint32_t *seg_cnt = reinterpret_cast<const uint32_t *>(ws1 + L.seg_cnt);
    const uint64_t *seg_base = reinterpret_cast<const uint64_t *>(ws1 + L.seg_base);
    const uint64_t *slot = reinterpret_cast<const uint64_t *>(ws1 + L.slot);
    uint64_t *nl = reinterpret_cast<uint64_t *>(ws2 + L.nl);
    uint32_t *kind = reinterpret_cast<uint32_t *>(ws2 + L.kind);
    uint64_t *rank = reinterpret_cast<uint64_t *>(ws2 + L.rank);
    uint64_t *partials = reinterpret_cast<uint64_t *>(ws2 + L.partials2);
    hipError_t e;
    if (n_lines == 0) return hipMemsetAsync(x.counts + 1, 0, 24, s);
    // (counts[3] was zeroed by phase 1)
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    hipLaunchKernelGGL(k_nl_place, dim3((unsigned)((n_seg + 64 * IX_WAVES - 1) / (64 * IX_WAVES))), dim3(64 * IX_WAVES), 0,
                       s, buf, n, n_seg, seg_cnt, slot, seg_base, nl, kind, x.counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = vcfc_scan_kinds(kind, n_lines, partials, rank, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_line_place, dim3((unsigned)((n_lines + 255) / 256)), dim3(256), 0, s, nl, n_lines, rank, x);
    return hipGetLastError();
}
