// vcfc_synth.hip -- synthetic genotype rows generated directly in HBM for the
// benchmark and the large parity cases (config 2/4 inputs do not fit on disk
// comfortably; the reference's own generator other/random_vcf.py needs ~40 min
// for 2504 x 1M in Python).  Not on the encode path.
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>
#include "vcfc_device.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// allele from a 32-bit uniform
__device__ __forceinline__ uint32_t allele(uint32_t u, int law, float af) {
    if (law == 0) {
        // p(0) = .90, p(1) = .08, p(2) = .02  (reference other/random_vcf.py:66-67)
        return u < 3865470566u ? 0u : (u < 4209067950u ? 1u : 2u);
    }
    const float x = (float)(u >> 8) * (1.0f / 16777216.0f);
    if (af <= 1.0f) return x < af ? 1u : 0u;
    const float a1 = af - 1.0f;           // multi-allelic row: second ALT at 0.5 %
    return x < a1 ? 1u : (x < a1 + 0.005f ? 2u : 0u);
}

// law 2 ("general shapes"): per-column sample traits, the
// same for every row (as sex and coverage are in a real VCF)
__device__ __forceinline__ bool col_male(uint32_t j) { return (mix64(0xC0FFEEull ^ j) & 1ull) != 0; }
__device__ __forceinline__ bool col_missing(uint32_t j) { return (mix64(0xBADC0DEull ^ j) >> 32) < 858993459ull; }
// token bytes of sample j in a law-2 row of `kind` (see workload.py)
__device__ __forceinline__ uint32_t law2_len(uint32_t kind, uint32_t j) {
    return kind == 0 ? (col_male(j) ? 1u : 3u) : kind == 1 ? 9u : kind == 4 ? (col_missing(j) ? 1u : 3u) : 3u;
}

// one wave per row: prefix copy + S tokens separated by TABs + '\n'.
// laws 0/1: every token "a|b"; law 2: row_af[row] = kind + allele frequency;
// law 3 (the RLE worst case): row_af[row] = kind, 0 = the
// classes 0|0 0|1 1|0 1|1 cycling (every token starts a run), 1 = alleles
// i.i.d. at frequency 1/2 (het-heavy: runs of 4/3 tokens on average).
// Genotypes hash (seed, row_base + row, sample): a batch generated as row
// slices with their row_base equals the batch generated whole.
__global__ __launch_bounds__(256) void k_synth(uint8_t *buf, const uint64_t *line_off, uint64_t n,
                                               const uint8_t *prefix, const uint64_t *prefix_off,
                                               const float *row_af, uint32_t S, int law, uint64_t seed,
                                               uint64_t row_base) {
    const uint64_t lrow = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (lrow >= n) return;
    const uint64_t row = row_base + lrow;   // (the genotype hash's row)
    const uint32_t l = vw::lane_id();
    uint8_t *dst = buf + line_off[lrow];
    const uint64_t p0 = prefix_off[lrow], p1 = prefix_off[lrow + 1];
    const uint32_t P = (uint32_t)(p1 - p0);
    for (uint32_t i = l; i < P; i += 64) dst[i] = prefix[p0 + i];
    uint8_t *g = dst + P;
    float af = row_af ? row_af[lrow] : 0.0f;
    if (law == 2) {
        const uint32_t kind = (uint32_t)af;
        af -= (float)kind;
        uint32_t base = 0;   // byte offset of the current 64-sample block's first token
        for (uint32_t j0 = 0; j0 < S; j0 += 64) {
            const uint32_t j = j0 + l;
            const uint32_t len = j < S ? law2_len(kind, j) : 0u;
            const uint32_t inc = vw::scan_add(j < S ? len + 1u : 0u);
            if (j < S) {
                uint8_t *t = g + base + inc - (len + 1u);
                const uint64_t h = mix64(seed ^ mix64(row * 0x100000001B3ull + j));
                const uint32_t a1 = allele((uint32_t)h, 1, af), a2 = allele((uint32_t)(h >> 32), 1, af);
                if (len == 1) {
                    t[0] = kind == 4 ? (uint8_t)'.' : (uint8_t)('0' + a1);
                } else if (kind == 2 && ((h >> 40) & 0xFFu) < 77u) {   // ~30 % "./."
                    t[0] = '.'; t[1] = '/'; t[2] = '.';
                } else {
                    t[0] = (uint8_t)('0' + a1);
                    t[1] = kind == 3 ? (uint8_t)'/' : (uint8_t)'|';
                    t[2] = (uint8_t)('0' + a2);
                    if (len == 9) {
                        const uint32_t dp = 10u + (uint32_t)((h >> 48) % 90u), gq = 10u + (uint32_t)((h >> 56) % 90u);
                        t[3] = ':'; t[4] = (uint8_t)('0' + dp / 10); t[5] = (uint8_t)('0' + dp % 10);
                        t[6] = ':'; t[7] = (uint8_t)('0' + gq / 10); t[8] = (uint8_t)('0' + gq % 10);
                    }
                }
                t[len] = (uint8_t)(j + 1 == S ? '\n' : '\t');
            }
            base += vw::readlane(inc, 63);
        }
        return;
    }
    const uint32_t cyc = law == 3 && af < 0.5f ? (uint32_t)(row & 3u) : 4u;   // law 3 kind 0: the phase
    if (law == 3) af = 0.5f;
    for (uint32_t j = l; j < S; j += 64) {
        const uint64_t h = mix64(seed ^ mix64(row * 0x100000001B3ull + j));
        uint32_t a1 = allele((uint32_t)h, law == 3 ? 1 : law, af), a2 = allele((uint32_t)(h >> 32), law == 3 ? 1 : law, af);
        if (cyc < 4u) {   // 0|0 0|1 1|0 1|1 0|0 ...
            const uint32_t c = (cyc + j) & 3u;
            a1 = c >> 1;
            a2 = c & 1u;
        }
        g[4 * j + 0] = (uint8_t)('0' + a1);
        g[4 * j + 1] = (uint8_t)'|';
        g[4 * j + 2] = (uint8_t)('0' + a2);
        g[4 * j + 3] = (uint8_t)(j + 1 == S ? '\n' : '\t');
    }
}

}  // namespace

hipError_t vcfc_synth_device(uint8_t *buf, const uint64_t *line_off, uint64_t n, const uint8_t *prefix,
                             const uint64_t *prefix_off, const float *row_af, uint32_t S, int law,
                             uint64_t seed, uint64_t row_base, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, buf, line_off, n, prefix,
                       prefix_off, row_af, S, law, seed, row_base);
    return hipGetLastError();
}
