// write_probe.hip -- write-bandwidth ceiling for the decoder's output shape
// (not product code; a measurement tool).  Every pattern writes the same
// 10.19 GB (1M lines of 10,189 B, the config-2 decode output):
//   w0  grid-stride 16-B plain stores over the whole buffer
//   w1  grid-stride 16-B non-temporal stores
//   w2  one wave per line, 1 KiB per store instruction (16 B per lane),
//       non-temporal -- the decoder's tile stores, lines back to back
//   w3  as w2, plain stores
//   w4  as w3, each line's stores at its own (unaligned) start -- the
//       decoder's tile stores at line + REQ' (any byte alignment)
//   w5  as w4 with 4-B stores (a lane's four dwords one by one)
//   w6  as w4 from a resident grid: wave g writes lines g, g + G, g + 2G, ...
//       (G = 4 x blocks; blocks 1024 / 2048 / 4096 / 8192)
//   w7  as w4 with a block per line: wave w of the block writes the line's
//       1 KiB pieces w, w + 4, w + 8, ... (4x fewer lines written at once)
//   w8  as w3 with every store instruction's 1 KiB aligned to 128 B (the
//       line's bytes from its first 128-B boundary: no partial 128-B line
//       inside a line, only at its two ends)
//   w9  as w3 with 64-B aligned store windows
//   w10 output-ordered chunks (round 6): the buffer (from byte 37) cut into
//       C-byte chunks, a resident grid taking chunks g, g + G, ... (each
//       wave-iteration writes C contiguous bytes, 1 KiB per instruction),
//       C = 1 / 2 / 4 KiB; "+load" first reads one dword per lane of a
//       680 MB input at the chunk (and uses it), as a tile writer reads
//       its record window -- on gfx9 that load's wait also waits for the
//       wave's earlier stores
// Build: hipcc --offload-arch=gfx950 -O3 -o build/write_probe tools/write_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint64_t LINE = 10189, NLINE = 1000000, TOTAL = LINE * NLINE;

template <bool NT>
__global__ __launch_bounds__(256) void w_grid(v4u *buf, uint64_t n16) {
    const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store(v, buf + i); else buf[i] = v;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void w_line(uint8_t *buf) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NLINE) return;
    const uint64_t o0 = row * LINE, a0 = (o0 + 15) & ~15ull, e = o0 + LINE;
    const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
    for (uint64_t o = a0 + 16 * l; o + 16 <= e; o += 1024) {
        v4u *p = reinterpret_cast<v4u *>(buf + o);
        if (NT) __builtin_nontemporal_store(v, p); else *p = v;
    }
}

template <bool DW>
__global__ __launch_bounds__(256) void w_line_u(uint8_t *buf) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NLINE) return;
    const uint64_t o0 = row * LINE + 37, e = o0 + LINE - 64;
    for (uint64_t o = o0 + 16 * l; o + 16 <= e; o += 1024) {
        if (DW) {
            uint32_t *p = reinterpret_cast<uint32_t *>(buf + o);
            p[0] = 0x09307C30u; p[1] = 0x09307C30u; p[2] = 0x09307C30u; p[3] = 0x09307C30u;
        } else {
            const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
            __builtin_memcpy(buf + o, &v, 16);
        }
    }
}

__global__ __launch_bounds__(256) void w_line_persist(uint8_t *buf) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t G = (uint64_t)gridDim.x * 4;
    for (uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < NLINE; row += G) {
        const uint64_t o0 = row * LINE + 37, e = o0 + LINE - 64;
        for (uint64_t o = o0 + 16 * l; o + 16 <= e; o += 1024) {
            const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
            __builtin_memcpy(buf + o, &v, 16);
        }
    }
}

__global__ __launch_bounds__(256) void w_line_block(uint8_t *buf) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t row = blockIdx.x;
    const uint64_t o0 = row * LINE + 37, e = o0 + LINE - 64;
    for (uint64_t o = o0 + 1024 * w + 16 * l; o + 16 <= e; o += 4096) {
        const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
        __builtin_memcpy(buf + o, &v, 16);
    }
}

template <uint32_t A>
__global__ __launch_bounds__(256) void w_line_al(uint8_t *buf) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t row = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= NLINE) return;
    const uint64_t o0 = row * LINE, a0 = (o0 + A - 1) & ~(uint64_t)(A - 1), e = o0 + LINE;
    const v4u v = {0x09307C30u, 0x09307C30u, 0x09307C30u, 0x09307C30u};
    for (uint64_t o = a0 + 16 * l; o + 16 <= e; o += 1024) *reinterpret_cast<v4u *>(buf + o) = v;
}

template <uint32_t C, bool LOAD>
__global__ __launch_bounds__(256) void w_chunk(uint8_t *buf, const uint32_t *src, uint64_t nsrc) {
    const uint32_t l = threadIdx.x & 63;
    const uint64_t G = (uint64_t)gridDim.x * 4, nchunk = (TOTAL - 64) / C;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += G) {
        uint32_t x = 0x09307C30u;
        if (LOAD) x |= src[(c * 64 + l) % nsrc];   // the input is zero
        const v4u v = {x, x, x, x};
        const uint64_t o0 = 37 + c * C;
        for (uint64_t o = o0 + 16 * l; o < o0 + C; o += 1024) __builtin_memcpy(buf + o, &v, 16);
    }
}

int main() {
    uint8_t *buf;
    CK(hipMalloc(&buf, TOTAL + 64));
    const uint64_t NSRC = 680000000ull / 4;
    uint32_t *src;
    CK(hipMalloc(&src, NSRC * 4));
    CK(hipMemset(src, 0, NSRC * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[27] = {"w0 grid plain", "w1 grid nt", "w2 line nt", "w3 line plain", "w4 line plain unaligned",
                             "w5 line plain unaligned dwords", "w6 resident 1024 blocks", "w6 resident 2048 blocks",
                             "w6 resident 4096 blocks", "w6 resident 8192 blocks", "w7 block per line", "w8 line 128-B aligned", "w9 line 64-B aligned",
                             "w10 chunk 1K g2048", "w10 chunk 2K g2048", "w10 chunk 4K g2048",
                             "w10 chunk 1K g2048 +load", "w10 chunk 2K g2048 +load", "w10 chunk 4K g2048 +load",
                             "w10 chunk 1K g4096", "w10 chunk 2K g4096", "w10 chunk 4K g4096",
                             "w10 chunk 1K g4096 +load", "w10 chunk 2K g4096 +load", "w10 chunk 4K g4096 +load",
                             "w10 chunk 8K g2048 +load", "w10 chunk 8K g4096 +load"};
    for (int p = 0; p < 27; p++) {
        float best = 1e9;
        for (int it = 0; it < 12; it++) {
            CK(hipEventRecord(e0));
            if (p == 0) hipLaunchKernelGGL(w_grid<false>, dim3(8192), dim3(256), 0, 0, (v4u *)buf, TOTAL / 16);
            if (p == 1) hipLaunchKernelGGL(w_grid<true>, dim3(8192), dim3(256), 0, 0, (v4u *)buf, TOTAL / 16);
            if (p == 2) hipLaunchKernelGGL(w_line<true>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            if (p == 3) hipLaunchKernelGGL(w_line<false>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            if (p == 4) hipLaunchKernelGGL(w_line_u<false>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            if (p == 5) hipLaunchKernelGGL(w_line_u<true>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            if (p >= 6 && p < 10) hipLaunchKernelGGL(w_line_persist, dim3(1024u << (p - 6)), dim3(256), 0, 0, buf);
            if (p == 10) hipLaunchKernelGGL(w_line_block, dim3(NLINE), dim3(256), 0, 0, buf);
            if (p == 11) hipLaunchKernelGGL(w_line_al<128>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            if (p == 12) hipLaunchKernelGGL(w_line_al<64>, dim3(NLINE / 4), dim3(256), 0, 0, buf);
            const dim3 g(p >= 19 && p < 25 ? 4096 : p == 26 ? 4096 : 2048);
            if (p == 13 || p == 19) hipLaunchKernelGGL((w_chunk<1024, false>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 14 || p == 20) hipLaunchKernelGGL((w_chunk<2048, false>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 15 || p == 21) hipLaunchKernelGGL((w_chunk<4096, false>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 16 || p == 22) hipLaunchKernelGGL((w_chunk<1024, true>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 17 || p == 23) hipLaunchKernelGGL((w_chunk<2048, true>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 18 || p == 24) hipLaunchKernelGGL((w_chunk<4096, true>), g, dim3(256), 0, 0, buf, src, NSRC);
            if (p == 25 || p == 26) hipLaunchKernelGGL((w_chunk<8192, true>), g, dim3(256), 0, 0, buf, src, NSRC);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it >= 2 && ms < best) best = ms;
        }
        printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GB/s\": %.1f}\n", names[p], best, TOTAL / (best * 1e6));
    }
    return 0;
}
