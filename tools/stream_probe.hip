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

int main() {
    const uint64_t bytes = ROW * NROW;
    uint8_t *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, bytes + 65536));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0x5A, bytes + 65536));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned rowsg = (unsigned)((NROW + 3) / 4);
    for (int pat = 0; pat < 6; pat++) {
        float best = 1e9f, tot = 0;
        for (int rep = 0; rep < 8; rep++) {
            CK(hipEventRecord(e0, 0));
            if (pat == 0) hipLaunchKernelGGL(p0, dim3(256 * 32), dim3(256), 0, 0, (const v4u *)buf, bytes / 16, sink);
            if (pat == 1) hipLaunchKernelGGL(p1<1>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 2) hipLaunchKernelGGL(p1<0>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 3) hipLaunchKernelGGL(p3, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 4) hipLaunchKernelGGL(p4, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            if (pat == 5) hipLaunchKernelGGL(p1<2>, dim3(rowsg), dim3(256), 0, 0, buf, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0) { best = ms < best ? ms : best; tot += ms; }
        }
        printf("p%d best %.3f ms (%.0f GB/s), mean %.3f ms\n", pat, best, bytes / (best * 1e-3) / 1e9, tot / 7);
    }
    return 0;
}
