// stream_probe.hip -- read-bandwidth ceiling of the access patterns the
// encoder could use (not product code; a measurement tool).  Every pattern
// reads the same ~10.2 GB (1M rows of 10,192 B, the config-2 line size) and
// XOR-folds it into one word per wave so the loads stay live.
//   p0  grid-stride 16-B loads over the whole buffer (copy-kernel pattern)
//   p1  one wave per row, 2 KiB chunks (32 B per lane as two 16-B loads at
//       stride 32) + a 4-B look-ahead load, three chunks in flight: the
//       encoder's genotype stream
//   p2  as p1 without the look-ahead load
//   p3  one wave per row, 1 KiB chunks (one contiguous 16-B load per lane),
//       six in flight
//   p4  one wave per row, 4 KiB chunks (four 16-B loads per lane, each 1 KiB
//       contiguous), two in flight
//   p5  p1 with the look-ahead load issued by lane 63 only
//   p6  the encoder's dependency chain per row: line_off[row] (scalar load),
//       then the line's first 1 KiB (prefix phase), a genotype start x9
//       derived from those bytes, then p5's stream from x9 (three dependent
//       latencies per row); V dependent VALU per 2 KiB chunk (0 / 96)
//   p8  line_off[row], then p5's stream from the line start (two latencies:
//       the prefix read as part of the first chunk); V as p6
//   p6 V=192 / 288, and p6 at 6 waves per SIMD (26 KB of LDS per block, the
//       encoder's occupancy) with V = 96 / 192 / 288
// Build: hipcc --offload-arch=gfx950 -O3 -o build/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint64_t ROW = 10192, NROW = 1000000;

__device__ __forceinline__ v4u ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t fold(v4u v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ __launch_bounds__(256) void p0(const v4u *buf, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) acc ^= fold(buf[i]);
    if (acc == 0x12345678u) sink[0] = acc;
}

// LOOK 0: no look-ahead load; 1: every lane; 2: lane 63 only (the others'
// offsets past the range: no memory request)
template <int LOOK>
__global__ __launch_bounds__(256) void p1(const uint8_t *buf, uint32_t *sink) {
    const uint32_t l = threadIdx.x & 63;
    const uint32_t yo = LOOK == 2 ? (l == 63 ? 0u : 0x40000000u) : 0u;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NROW) return;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf + row * ROW), (short)0, (int)ROW, 0x00020000);
    const uint32_t nch = (ROW + 2047) / 2048;
    uint32_t acc = 0;
    v4u a0 = ld16(rs, 32 * l), b0 = ld16(rs, 32 * l + 16);
    uint32_t y0 = LOOK ? ld4(rs, 32 * l + 32 + yo) : 0;
    v4u a1 = ld16(rs, 2048 + 32 * l), b1 = ld16(rs, 2048 + 32 * l + 16);
    uint32_t y1 = LOOK ? ld4(rs, 2048 + 32 * l + 32 + yo) : 0;
    v4u a2 = ld16(rs, 4096 + 32 * l), b2 = ld16(rs, 4096 + 32 * l + 16);
    uint32_t y2 = LOOK ? ld4(rs, 4096 + 32 * l + 32 + yo) : 0;
    for (uint32_t c = 0; c < nch; c += 3) {
        acc ^= fold(a0) ^ fold(b0) ^ y0;
        a0 = ld16(rs, (c + 3) * 2048 + 32 * l); b0 = ld16(rs, (c + 3) * 2048 + 32 * l + 16);
        if (LOOK) y0 = ld4(rs, (c + 3) * 2048 + 32 * l + 32 + yo);
        acc ^= fold(a1) ^ fold(b1) ^ y1;
        a1 = ld16(rs, (c + 4) * 2048 + 32 * l); b1 = ld16(rs, (c + 4) * 2048 + 32 * l + 16);
        if (LOOK) y1 = ld4(rs, (c + 4) * 2048 + 32 * l + 32 + yo);
        acc ^= fold(a2) ^ fold(b2) ^ y2;
        a2 = ld16(rs, (c + 5) * 2048 + 32 * l); b2 = ld16(rs, (c + 5) * 2048 + 32 * l + 16);
        if (LOOK) y2 = ld4(rs, (c + 5) * 2048 + 32 * l + 32 + yo);
        asm volatile("" ::: "memory");
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void p3(const uint8_t *buf, uint32_t *sink) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NROW) return;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf + row * ROW), (short)0, (int)ROW, 0x00020000);
    uint32_t acc = 0;
    v4u v[6];
#pragma unroll
    for (int k = 0; k < 6; k++) v[k] = ld16(rs, 1024 * k + 16 * l);
    for (uint32_t c = 0; c < (ROW + 1023) / 1024; c += 6) {
#pragma unroll
        for (int k = 0; k < 6; k++) {
            acc ^= fold(v[k]);
            v[k] = ld16(rs, 1024 * (c + 6 + k) + 16 * l);
        }
        asm volatile("" ::: "memory");
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void p4(const uint8_t *buf, uint32_t *sink) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NROW) return;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(buf + row * ROW), (short)0, (int)ROW, 0x00020000);
    uint32_t acc = 0;
    v4u v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = ld16(rs, 1024 * k + 16 * l);
    for (uint32_t c = 0; c < (ROW + 4095) / 4096; c++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            acc ^= fold(v[k]);
            v[k] = v[k + 4];
            v[k + 4] = ld16(rs, 4096 * (c + 2) + 1024 * k + 16 * l);
        }
        asm volatile("" ::: "memory");
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// V dependent VALU on the chunk's words (models the encoder's per-chunk work)
template <int V>
__device__ __forceinline__ uint32_t work(uint32_t acc, v4u a, v4u b) {
    uint32_t x = acc ^ fold(a) ^ fold(b);
#pragma unroll
    for (int i = 0; i < V / 2; i++) {
        x = (x ^ (x << 7)) + (uint32_t)i;
    }
    return x;
}

template <bool PREFIX, int V, bool OCC6 = false>
__global__ __launch_bounds__(256) void p6(const uint8_t *buf, const uint64_t *line_off, uint32_t *sink) {
    const uint32_t l = threadIdx.x & 63;
    if (OCC6) {   // 26 KB of LDS per block: 6 blocks = 6 waves per SIMD
        __shared__ uint32_t occ[6656];
        if (sink[1] == 0x12345678u) { occ[threadIdx.x] = l; sink[2] = occ[(threadIdx.x + 1) & 255]; }
    }
    const uint32_t yo = l == 63 ? 0u : 0x40000000u;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NROW) return;
    // (uint32_t) casts: readfirstlane returns int, which would sign-extend
    // offsets of 2 GiB and more into the upper word (a faulting address)
    const uint64_t off = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)line_off[row]) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(line_off[row] >> 32)) << 32);
    const uint8_t *line = buf + off;
    uint32_t acc = 0, x9 = 0;
    if (PREFIX) {
        auto rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(line), (short)0, 1024, 0x00020000);
        const v4u pv = ld16(rp, 16 * l);
        acc = fold(pv);
        x9 = ((uint32_t)__builtin_amdgcn_readfirstlane(acc) & 0x7Fu) + 64u;   // data-dependent genotype start
    }
    const uint8_t *g = line + x9;
    const uint32_t glen = (uint32_t)ROW - x9;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(g), (short)0, (int)glen, 0x00020000);
    const uint32_t nch = (glen + 2047) / 2048;
    v4u a0 = ld16(rs, 32 * l), b0 = ld16(rs, 32 * l + 16);
    uint32_t y0 = ld4(rs, 32 * l + 32 + yo);
    v4u a1 = ld16(rs, 2048 + 32 * l), b1 = ld16(rs, 2048 + 32 * l + 16);
    uint32_t y1 = ld4(rs, 2048 + 32 * l + 32 + yo);
    v4u a2 = ld16(rs, 4096 + 32 * l), b2 = ld16(rs, 4096 + 32 * l + 16);
    uint32_t y2 = ld4(rs, 4096 + 32 * l + 32 + yo);
    for (uint32_t c = 0; c < nch; c += 3) {
        acc = work<V>(acc ^ y0, a0, b0);
        a0 = ld16(rs, (c + 3) * 2048 + 32 * l); b0 = ld16(rs, (c + 3) * 2048 + 32 * l + 16);
        y0 = ld4(rs, (c + 3) * 2048 + 32 * l + 32 + yo);
        acc = work<V>(acc ^ y1, a1, b1);
        a1 = ld16(rs, (c + 4) * 2048 + 32 * l); b1 = ld16(rs, (c + 4) * 2048 + 32 * l + 16);
        y1 = ld4(rs, (c + 4) * 2048 + 32 * l + 32 + yo);
        acc = work<V>(acc ^ y2, a2, b2);
        a2 = ld16(rs, (c + 5) * 2048 + 32 * l); b2 = ld16(rs, (c + 5) * 2048 + 32 * l + 16);
        y2 = ld4(rs, (c + 5) * 2048 + 32 * l + 32 + yo);
        asm volatile("" ::: "memory");
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t bytes = ROW * NROW;
    uint8_t *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, bytes + 65536));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(sink, 0, 64));
    CK(hipMemset(buf, 0x5A, bytes + 65536));
    uint64_t *line_off;
    {
        std::vector<uint64_t> lo(NROW);
        for (uint64_t i = 0; i < NROW; i++) lo[i] = i * ROW;
        CK(hipMalloc(&line_off, 8 * NROW));
        CK(hipMemcpy(line_off, lo.data(), 8 * NROW, hipMemcpyHostToDevice));
    }
    const char *pname[15] = {"p0", "p1", "p2", "p3", "p4", "p5", "p6 V=0", "p6 V=96", "p8 V=0", "p8 V=96",
                             "p6 V=192", "p6 V=288", "p6 occ6 V=96", "p6 occ6 V=192", "p6 occ6 V=288"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned rowsg = (unsigned)((NROW + 3) / 4);
    for (int pat = 0; pat < 15; pat++) {
        float best = 1e9f, tot = 0;
        for (int rep = 0; rep < 8; rep++) {
            CK(hipEventRecord(e0, 0));
            if (pat == 0) hipLaunchKernelGGL(p0, dim3(256 * 32), dim3(256), 0, 0, (const v4u *)buf, bytes / 16, sink);
            if (pat == 1) hipLaunchKernelGGL(p1<1>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 2) hipLaunchKernelGGL(p1<0>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 3) hipLaunchKernelGGL(p3, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 4) hipLaunchKernelGGL(p4, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 5) hipLaunchKernelGGL(p1<2>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 6) hipLaunchKernelGGL((p6<true, 0>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 7) hipLaunchKernelGGL((p6<true, 96>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 8) hipLaunchKernelGGL((p6<false, 0>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 9) hipLaunchKernelGGL((p6<false, 96>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 10) hipLaunchKernelGGL((p6<true, 192>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 11) hipLaunchKernelGGL((p6<true, 288>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 12) hipLaunchKernelGGL((p6<true, 96, true>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 13) hipLaunchKernelGGL((p6<true, 192, true>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            if (pat == 14) hipLaunchKernelGGL((p6<true, 288, true>), dim3(rowsg), dim3(256), 0, 0, buf, line_off, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0) { best = ms < best ? ms : best; tot += ms; }
        }
        printf("%s best %.3f ms (%.0f GB/s), mean %.3f ms\n", pname[pat], best, bytes / (best * 1e-3) / 1e9, tot / 7);
    }
    return 0;
}
