// store_probe.hip -- write-bandwidth of the decoder's output pattern (not
// product code; a measurement tool).  1M lines of 10,190 B (the config-2
// line size) are written by one wave each as 16-B stores per lane, 1 KiB per
// wave store instruction:
//   s0  lines packed back to back (line starts at any byte: every 16-B store
//       is unaligned, as k_dec_write's token stores)
//   s1  the same lines with every line start rounded up to 16 B
//   s2  packed lines, stores aligned to 16 B inside each line (head and tail
//       bytes stored singly)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
constexpr uint64_t LINE = 10190, NLINE = 1000000;

__global__ __launch_bounds__(256) void s_lines(uint8_t *out, const uint64_t *off, int aligned_inside) {
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= NLINE) return;
    const uint32_t l = threadIdx.x & 63;
    uint8_t *dst = out + off[r];
    const v4u v = {(uint32_t)r, l, 0x09307C30u, 0x09307C30u};
    if (!aligned_inside) {
        for (uint32_t b = 16 * l; b + 16 <= LINE; b += 1024)
            *(g_v4u *)((__attribute__((address_space(1))) uint8_t *)dst + b) = v;
        if (l < (LINE & 15)) dst[(LINE & ~15ull) + l] = 0x0A;
        return;
    }
    const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
    const uint32_t body = (uint32_t)((LINE - head) & ~15ull);
    for (uint32_t b = head + 16 * l; b < head + body; b += 1024)
        *(g_v4u *)((__attribute__((address_space(1))) uint8_t *)dst + b) = v;
    if (l < head) dst[l] = 0x30;
    if (l < LINE - head - body) dst[head + body + l] = 0x0A;
}

int main() {
    std::vector<uint64_t> packed(NLINE), rounded(NLINE);
    uint64_t p = 0, q = 0;
    for (uint64_t i = 0; i < NLINE; i++) {
        packed[i] = p;
        rounded[i] = q;
        p += LINE + (i * 7919) % 13;   // line lengths vary a little, as real lines
        q = (q + LINE + (i * 7919) % 13 + 15) & ~15ull;
    }
    uint8_t *out;
    uint64_t *d_off;
    CK(hipMalloc(&out, q + 65536));
    CK(hipMalloc(&d_off, 8 * NLINE));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int pat = 0; pat < 3; pat++) {
        CK(hipMemcpy(d_off, pat == 1 ? rounded.data() : packed.data(), 8 * NLINE, hipMemcpyHostToDevice));
        float best = 1e9f, tot = 0;
        for (int rep = 0; rep < 8; rep++) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(s_lines, dim3((unsigned)((NLINE + 3) / 4)), dim3(256), 0, 0, out, d_off, pat == 2);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0) { best = ms < best ? ms : best; tot += ms; }
        }
        printf("s%d best %.3f ms (%.0f GB/s), mean %.3f ms\n", pat, best, LINE * NLINE / (best * 1e-3) / 1e9, tot / 7);
    }
    return 0;
}
