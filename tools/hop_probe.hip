// hop_probe.hip -- latency of the hop line index's walk (not product code; a
// measurement tool): 32 768 walkers of 16 lanes (4 a wave, as k_nl_hop),
// walker w starting at w x 311 KB of a 10.19 GB buffer, R rounds each of G
// 256-byte windows G lines apart (a line = 10 189 B), the next round's
// address depending on the loaded bytes (the walk's chain).  Compared: the
// stride of a config-2 line, a 256-byte stride (one page region), and G.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/hop_probe tools/hop_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr uint64_t TOTAL = 10189ull * 1000000ull;
constexpr uint64_t ALLOC = TOTAL + (64ull << 20);   // walker starts run past TOTAL by ~1.5 MB (checked per case)

template <uint32_t G>
__global__ __launch_bounds__(256) void walk(const uint8_t *buf, uint64_t span, uint64_t stride, uint32_t rounds,
                                            uint64_t walkers, uint32_t *out) {
    const uint32_t l = threadIdx.x & 63, wl = l & 15;
    const uint64_t w = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (l >> 4);
    if (w >= walkers) return;
    uint64_t p = w * span;
    uint32_t acc = 0;
    for (uint32_t r = 0; r < rounds; r++) {
        uint4 v[G];
#pragma unroll
        for (uint32_t k = 0; k < G; k++) v[k] = *reinterpret_cast<const uint4 *>(buf + p + k * stride + 16 * wl);
        uint32_t x = 0;
#pragma unroll
        for (uint32_t k = 0; k < G; k++) x |= v[k].x | v[k].w;
        acc += x;
        p += G * stride + (x & 1);   // (the buffer is zero: a dependence, no change)
    }
    if (acc == 12345) out[0] = acc;
}

int main() {
    uint8_t *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, ALLOC));
    CK(hipMemset(buf, 0, ALLOC));
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Case { const char *name; uint32_t g; uint64_t walkers, span, stride; uint32_t rounds; };
    const Case cases[] = {
        {"32768 walkers, 30 rounds, 1 window/round, line stride", 1, 32768, 311000, 10189, 30},
        {"32768 walkers, 8 rounds, 4 windows/round, line stride", 4, 32768, 311000, 10189, 8},
        {"32768 walkers, 30 rounds, 1 window/round, 256-B stride", 1, 32768, 311000, 256, 30},
        {"32768 walkers, 8 rounds, 4 windows/round, 256-B stride", 4, 32768, 311000, 256, 8},
        {"16384 walkers, 60 rounds, 1 window/round, line stride", 1, 16384, 622000, 10189, 60},
        {"16384 walkers, 15 rounds, 4 windows/round, line stride", 4, 16384, 622000, 10189, 15},
        {"65536 walkers, 4 rounds, 4 windows/round, line stride", 4, 65536, 155500, 10189, 4},
        {"32768 walkers, 1 round, 1 window", 1, 32768, 311000, 10189, 1},
    };
    for (const Case &c : cases) {
        // every load inside the buffer: the last walker's last window
        const uint64_t last = (c.walkers - 1) * c.span + (uint64_t)c.rounds * c.g * c.stride + c.rounds + 256;
        if (last > ALLOC) { printf("case %s reads past the buffer (%llu)\n", c.name, (unsigned long long)last); return 1; }
        float best = 1e9;
        const dim3 grid((unsigned)((c.walkers + 15) / 16));
        for (int it = 0; it < 8; it++) {
            CK(hipEventRecord(e0));
            if (c.g == 1) hipLaunchKernelGGL(walk<1>, grid, dim3(256), 0, 0, buf, c.span, c.stride, c.rounds, c.walkers, out);
            else hipLaunchKernelGGL(walk<4>, grid, dim3(256), 0, 0, buf, c.span, c.stride, c.rounds, c.walkers, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 2 && ms < best) best = ms;
        }
        printf("{\"case\": \"%s\", \"us\": %.1f, \"us_per_round\": %.2f}\n", c.name, best * 1000, best * 1000 / c.rounds);
    }
    return 0;
}
