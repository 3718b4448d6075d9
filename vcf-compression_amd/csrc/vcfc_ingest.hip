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
//   scan          segment bases (the encoder's exclusive scan)
//   k_nl_place    one wave per segment: its positions from the slot to their
//                 place; a segment with more than NL_SLOT lines (average
//                 line < 64 bytes: header lines) scans its bytes again
//   k_line_kind   one lane per line: data / pass flags
//   scan x2       data and pass ranks
//   k_line_place  one lane per line: scatter into the output arrays
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

namespace {

constexpr uint32_t SEG = 16384;          // bytes per wave
constexpr uint32_t WIN = 1024;           // bytes per wave step (16 per lane)
constexpr uint32_t IX_WAVES = 4;
constexpr uint32_t NL_SLOT = 128;        // '\n' positions kept per segment by k_nl_scan

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

// positions of the '\n' bytes of one 1 KiB window (lane l: bytes [p, p + 16))
// at out[o0 + rank] for ranks below `lim`; returns the window's count
__device__ __forceinline__ uint32_t nl_window(const uint8_t *buf, uint64_t n, uint64_t p, uint64_t *out, uint64_t o0,
                                              uint64_t lim) {
    uint32_t m = nl_mask16(buf, n, p);
    const uint32_t c = __builtin_popcount(m);
    const uint32_t inc = vw::scan_add(c);
    uint64_t o = o0 + inc - c;
    while (m && o < lim) {
        out[o++] = p + (uint64_t)__builtin_ctz(m);
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
// same per-segment output as k_nl_scan without reading every byte.  One wave
// walks the lines that start in a group of HOPG segments.  A data line whose
// first 1 KiB holds its 9th TAB and no '\n' is predicted to end at
// gt0 + 4 S - 1 (every token 3 bytes + TAB, gt0 = its first sample byte):
// one 256-byte window loaded beside the first (at the previous line's prefix
// length) checks that this byte is '\n' and the 31 bytes 4, 8, ..., 124
// before it are TABs.  Every other line (header and '#' lines, empty lines,
// other token lengths, a failed check) is scanned for its '\n'.  A group
// finds its first line start by scanning from the byte before it.  So a
// chr22-shaped file is read for ~1.2 KiB per line instead of every byte.
// A line predicted across a '\n' it did not see (one that is shorter than
// predicted and whose end lands on another line's '\n', with TABs at the 31
// checked places) is caught by the encoder (k_encode_fast<true> rejects '\n'
// in its tokens, k_nl_verify scans the rows it rejects), and the chunk is
// indexed again by k_nl_scan.
constexpr uint32_t HOPG = 8;          // 16 KiB segments per walker (128 KiB)
constexpr uint32_t GW = 256;          // guess window (4 bytes per lane)

// first '\n' at or after q (q < n, buf[n - 1] == '\n'), 4 KiB per round
__device__ uint64_t find_nl(const uint8_t *buf, uint64_t n, uint64_t q) {
    const uint32_t l = vw::lane_id();
    for (;;) {
        if (q >= n) return n - 1;   // (buf[n - 1] is '\n')
        uint32_t m[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) m[k] = nl_mask16(buf, n, q + 1024u * k + 16u * l);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint64_t b = vw::ballot(m[k] != 0);
            if (b) {
                const uint32_t f = (uint32_t)__builtin_ctzll(b);
                return q + 1024u * k + 16u * f + (uint32_t)__builtin_ctz(vw::readlane(m[k], f));
            }
        }
        q += 4096;
    }
}

// end ('\n') of the line starting at p (p < n); pl: the previous predicted
// line's prefix length (updated)
__device__ uint64_t line_end(const uint8_t *buf, uint64_t n, uint64_t p, uint32_t S, uint32_t &pl) {
    const uint32_t l = vw::lane_id();
    const uint64_t x = p + pl + 4ull * S - 1;      // the end if the prefix is as long as the last one
    const uint64_t g0 = x >= GW / 2 ? x - GW / 2 : 0;
    // the line's first 1 KiB and the guess window, both in flight
    const uint32_t nm = nl_mask16(buf, n, p + 16u * l);
    uint4 v = make_uint4(0, 0, 0, 0);
    const uint64_t q = p + 16u * l;
    if (q + 16 <= n) v = *reinterpret_cast<const uint4 *>(buf + q);
    uint32_t gw = 0;
    const uint64_t gq = g0 + 4u * l;
    if (gq + 4 <= n) __builtin_memcpy(&gw, buf + gq, 4);
    const uint32_t b0 = vw::readlane(v.x & 0xFFu, 0);
    // the first '\n' in the window is the line end (an empty line: p itself)
    const uint64_t nb = vw::ballot(nm != 0);
    if (nb) {
        const uint32_t f = (uint32_t)__builtin_ctzll(nb);
        return p + 16u * f + (uint32_t)__builtin_ctz(vw::readlane(nm, f));
    }
    if (S == 0 || b0 == '#' || p + 1024 > n) return find_nl(buf, n, p + 1024);
    // the 9th TAB of the window
    const uint32_t tm = (p + 16u * l + 16 <= n) ? (nl_bits(v.x ^ 0x03030303u) | nl_bits(v.y ^ 0x03030303u) << 4 |
                                                   nl_bits(v.z ^ 0x03030303u) << 8 | nl_bits(v.w ^ 0x03030303u) << 12)
                                                : 0u;   // ('\t' = '\n' ^ 0x03)
    const uint32_t c = (uint32_t)__builtin_popcount(tm);
    const uint32_t inc = vw::scan_add(c);
    const bool has9 = inc - c < 9 && inc >= 9;
    const uint64_t hb = vw::ballot(has9);
    if (!hb) return find_nl(buf, n, p + 1024);      // prefix longer than 1 KiB: scan
    const uint32_t k9 = (uint32_t)__builtin_ctzll(hb);
    uint32_t mm = tm;
    for (uint32_t k = inc - c; k < 8; k++) mm &= mm - 1;   // (lane k9 only; others' values unused)
    const uint32_t t9 = vw::readlane(16u * l + (uint32_t)__builtin_ctz(mm | 0x10000u), k9);
    const uint64_t gt0 = p + t9 + 1;
    const uint64_t e = gt0 + 4ull * S - 1;
    pl = (uint32_t)(gt0 - p);
    if (e >= n) return find_nl(buf, n, p + 1024);
    // the predicted end and the TABs before it, from the guess window (or one more load)
    bool ok;
    if (e >= g0 + 124 && e < g0 + GW && g0 + GW <= n) {
        // lane j's dword holds bytes [g0 + 4 j, + 4): byte e - 4 i is byte ((e - g0) & 3) of lane (e - g0) / 4 - i
        const uint32_t le = (uint32_t)(e - g0) >> 2, sh = 8u * ((uint32_t)(e - g0) & 3u);
        const uint32_t byte = (gw >> sh) & 0xFFu;
        const bool mine = l <= le && l + 31 >= le;       // lanes le - 31 .. le
        const uint32_t want = l == le ? 0x0Au : 0x09u;
        ok = vw::ballot(mine && byte != want) == 0;
    } else {
        uint32_t w = 0;
        const bool mine = l < 32;
        const uint64_t a = e - 4ull * l;                 // lane i: byte e - 4 i
        if (mine && a < n && a >= gt0) w = buf[a];
        const uint32_t want = l == 0 ? 0x0Au : 0x09u;
        ok = S >= 32 && vw::ballot(mine && w != want) == 0;
    }
    if (ok) return e;
    return find_nl(buf, n, p + 1024);
}

__global__ __launch_bounds__(256) void k_nl_hop(const uint8_t *buf, uint64_t n, uint64_t n_seg, uint32_t S,
                                                uint32_t *seg_cnt, uint64_t *slot) {
    const uint64_t g = (uint64_t)blockIdx.x * IX_WAVES + vw::readfirst(threadIdx.x >> 6);
    const uint64_t seg0 = g * HOPG;
    if (seg0 >= n_seg) return;
    const uint32_t l = vw::lane_id();
    const uint64_t lo = seg0 * SEG, hi = (seg0 + HOPG) * SEG < n ? (seg0 + HOPG) * SEG : n;
    uint32_t cnt = 0;   // lane k < HOPG: '\n' count of segment seg0 + k
    auto record = [&](uint64_t e) {   // lo <= e < hi, in order
        const uint32_t k = (uint32_t)((e - lo) / SEG);
        const uint32_t c = vw::readlane(cnt, k);
        if (l == 0 && c < NL_SLOT) slot[(seg0 + k) * NL_SLOT + c] = e;
        cnt += l == k ? 1u : 0u;
    };
    uint64_t p = 0;
    if (lo > 0) {
        const uint64_t e = find_nl(buf, n, lo - 1);
        if (e >= lo && e < hi) record(e);
        p = e + 1;
    }
    uint32_t pl = 0;
    while (p < hi) {
        const uint64_t e = line_end(buf, n, p, S, pl);   // (wave-uniform)
        if (e >= hi) break;
        record(e);
        p = e + 1;
    }
    if (l < HOPG && seg0 + l < n_seg) seg_cnt[seg0 + l] = cnt;
}

__global__ __launch_bounds__(256) void k_nl_place(const uint8_t *buf, uint64_t n, uint64_t n_seg, const uint32_t *seg_cnt,
                                                  const uint64_t *slot, const uint64_t *seg_base, uint64_t *nl) {
    const uint64_t seg = (uint64_t)blockIdx.x * IX_WAVES + vw::readfirst(threadIdx.x >> 6);
    if (seg >= n_seg) return;
    const uint32_t l = vw::lane_id();
    const uint32_t c = seg_cnt[seg];
    uint64_t *dst = nl + seg_base[seg];
    if (c <= NL_SLOT) {
        const uint64_t *sl = slot + seg * NL_SLOT;
        for (uint32_t k = l; k < c; k += 64) dst[k] = sl[k];
        return;
    }
    // more lines than the slot holds: scan the segment again (at most c
    // positions: the hop index may have counted fewer than there are, and
    // the encoder then rejects the chunk's index)
    uint32_t o = 0;
    for (uint32_t w = 0; w < SEG; w += WIN) o += nl_window(buf, n, seg * SEG + w + 16 * l, dst, o, c);
}

__global__ __launch_bounds__(256) void k_line_kind(const uint8_t *buf, const uint64_t *nl, uint64_t n_lines,
                                                   uint32_t *is_data, uint32_t *is_pass) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lines) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0u;
    const bool nonempty = nl[i] > s;
    const bool hash = nonempty && buf[s] == '#';
    is_data[i] = nonempty && !hash;
    is_pass[i] = hash;
}

__global__ __launch_bounds__(256) void k_line_place(const uint64_t *nl, uint64_t n_lines, const uint64_t *data_rank,
                                                    const uint64_t *pass_rank, VcfcLineIndex x) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lines) return;
    const uint64_t s = i ? nl[i - 1] + 1 : 0u;
    const uint64_t d = data_rank[i];
    if (nl[i] - s > 0xFFFFFFFFull) atomicMax((unsigned long long *)(x.counts + 3), 1ull);   // line lengths are 32-bit
    if (data_rank[i + 1] > d) {
        x.line_off[d] = s;
        x.line_len[d] = (uint32_t)(nl[i] - s);
        x.line_no[d] = (uint32_t)i;
    }
    const uint64_t q = pass_rank[i];
    if (pass_rank[i + 1] > q) {
        x.pass_off[q] = s;
        x.pass_len[q] = (uint32_t)(nl[i] - s);
        x.pass_no[q] = (uint32_t)i;
        x.pass_before[q] = d;
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
    L.partials1 = o; o = al(o + 8 * ((seg + 4095) / 4096 + 1));
    L.total1 = o;
    o = 0;
    L.nl = o; o = al(o + 8 * (n_lines + 1));
    L.is_data = o; o = al(o + 4 * (n_lines + 1));
    L.is_pass = o; o = al(o + 4 * (n_lines + 1));
    L.data_rank = o; o = al(o + 8 * (n_lines + 1));
    L.pass_rank = o; o = al(o + 8 * (n_lines + 1));
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
                           const VcfcLineIndex &x, hipStream_t s, uint32_t S_hint) {
    // ws: phase 1 workspace (L.total1 bytes)
    uint32_t *seg_cnt = reinterpret_cast<uint32_t *>(ws + L.seg_cnt);
    uint64_t *seg_base = reinterpret_cast<uint64_t *>(ws + L.seg_base);
    uint64_t *slot = reinterpret_cast<uint64_t *>(ws + L.slot);
    uint64_t *partials = reinterpret_cast<uint64_t *>(ws + L.partials1);
    hipError_t e;
    if (n == 0) return hipMemsetAsync(x.counts, 0, 24, s);
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    const dim3 sg((unsigned)((n_seg + IX_WAVES - 1) / IX_WAVES)), blk(64 * IX_WAVES);
    if (S_hint)
        hipLaunchKernelGGL(k_nl_hop, dim3((unsigned)((n_seg + HOPG * IX_WAVES - 1) / (HOPG * IX_WAVES))), blk, 0, s, buf,
                           n, n_seg, S_hint, seg_cnt, slot);
    else
        hipLaunchKernelGGL(k_nl_scan, sg, blk, 0, s, buf, n, n_seg, seg_cnt, slot);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = vcfc_scan_u32(seg_cnt, n_seg, partials, seg_base, s)) != hipSuccess) return e;
    return hipMemcpyAsync(x.counts, seg_base + n_seg, 8, hipMemcpyDeviceToDevice, s);
}

// Phase 2, once the host knows the line count (counts[0]): the '\n'
// positions in order, then the data / pass tables; ws1 = phase 1's
// workspace, ws2 = L.total2 bytes for vcfc_line_index_layout(chunk, n_lines).
hipError_t vcfc_line_index_place(const uint8_t *buf, uint64_t n, uint64_t n_lines, const uint8_t *ws1, uint8_t *ws2,
                                 const VcfcLineIndexLayout &L, const VcfcLineIndex &x, hipStream_t s) {
    const uint32_t *seg_cnt = reinterpret_cast<const uint32_t *>(ws1 + L.seg_cnt);
    const uint64_t *seg_base = reinterpret_cast<const uint64_t *>(ws1 + L.seg_base);
    const uint64_t *slot = reinterpret_cast<const uint64_t *>(ws1 + L.slot);
    uint64_t *nl = reinterpret_cast<uint64_t *>(ws2 + L.nl);
    uint32_t *is_data = reinterpret_cast<uint32_t *>(ws2 + L.is_data);
    uint32_t *is_pass = reinterpret_cast<uint32_t *>(ws2 + L.is_pass);
    uint64_t *data_rank = reinterpret_cast<uint64_t *>(ws2 + L.data_rank);
    uint64_t *pass_rank = reinterpret_cast<uint64_t *>(ws2 + L.pass_rank);
    uint64_t *partials = reinterpret_cast<uint64_t *>(ws2 + L.partials2);
    hipError_t e;
    if (n_lines == 0) return hipMemsetAsync(x.counts + 1, 0, 24, s);
    if ((e = hipMemsetAsync(x.counts + 3, 0, 8, s)) != hipSuccess) return e;
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    hipLaunchKernelGGL(k_nl_place, dim3((unsigned)((n_seg + IX_WAVES - 1) / IX_WAVES)), dim3(64 * IX_WAVES), 0, s, buf,
                       n, n_seg, seg_cnt, slot, seg_base, nl);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const dim3 g((unsigned)((n_lines + 255) / 256)), blk(256);
    hipLaunchKernelGGL(k_line_kind, g, blk, 0, s, buf, nl, n_lines, is_data, is_pass);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = vcfc_scan_u32(is_data, n_lines, partials, data_rank, s)) != hipSuccess) return e;
    if ((e = vcfc_scan_u32(is_pass, n_lines, partials, pass_rank, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_line_place, g, blk, 0, s, nl, n_lines, data_rank, pass_rank, x);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(x.counts + 1, data_rank + n_lines, 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    return hipMemcpyAsync(x.counts + 2, pass_rank + n_lines, 8, hipMemcpyDeviceToDevice, s);
}
