// vcfc_check.hip -- per-record 64-bit digests of an encoded batch on the GPU.
//
// Full-size parity (2504 x 1M rows, the biobank shards) compares every
// record without moving the records: the device digests each record in
// place, the checker digests its own CPU encode of the same rows, and the
// two digest arrays (8 B per row) are compared.  Digest (order-sensitive,
// word-parallel):
//   h = n * G + sum_k mix(w_k ^ (k * K1 + K2))   (mod 2^64),   digest = mix(h)
// w_k = record bytes [8k, 8k + 8) little-endian, zero-padded; mix = the
// splitmix64 finaliser.  One wave per record, lane l takes words l, l + 64, ...
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

constexpr int HASH_WAVES = 4;

__global__ __launch_bounds__(256) void k_record_hash(const uint8_t *__restrict__ recs,
                                                     const uint64_t *__restrict__ rec_off, uint64_t n,
                                                     uint64_t *__restrict__ out) {
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    const uint64_t i = (uint64_t)blockIdx.x * HASH_WAVES + wave;
    if (i >= n) return;
    const uint32_t l = vw::lane_id();
    const uint64_t a = rec_off[i], b = rec_off[i + 1];
    const uint64_t len = b - a;
    // buffer resource over the record's dwords: loads past it read 0
    const uint32_t lead = (uint32_t)(a & 3u);
    const vw::brsrc rs = vw::make_rsrc(recs + (a - lead), (uint32_t)((lead + len + 3u) & ~3ull));
    uint64_t h = 0;
    const uint64_t nw = (len + 7) / 8;
    for (uint64_t k0 = 0; k0 < nw; k0 += 64) {
        const uint64_t k = k0 + l;
        if (k < nw) {
            const uint32_t o = (uint32_t)(8 * k);   // record byte o is resource byte o + lead
            const uint32_t d0 = vw::bload4(rs, o), d1 = vw::bload4(rs, o + 4u), d2 = vw::bload4(rs, o + 8u);
            uint32_t lo = vw::alignbyte(d1, d0, lead), hi = vw::alignbyte(d2, d1, lead);
            const uint64_t valid = len - 8 * k;   // >= 1
            if (valid < 8) {
                const uint64_t m = (1ull << (8 * valid)) - 1ull;
                lo &= (uint32_t)m;
                hi &= (uint32_t)(m >> 32);
            }
            const uint64_t w = ((uint64_t)hi << 32) | lo;
            h += mix64(w ^ (k * 0xD1B54A32D192ED03ull + 0x8CB92BA72F3D8DD7ull));
        }
    }
    // wave sum (mod 2^64)
    for (uint32_t o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = vw::shfl((uint32_t)h, l ^ o), hi = vw::shfl((uint32_t)(h >> 32), l ^ o);
        h += ((uint64_t)hi << 32) | lo;
    }
    if (l == 0) out[i] = mix64(len * 0x9E3779B97F4A7C15ull + h);
}

}  // namespace

hipError_t vcfc_record_hash(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_record_hash, dim3((unsigned)((n + HASH_WAVES - 1) / HASH_WAVES)), dim3(64 * HASH_WAVES), 0, s,
                       recs, rec_off, n, out);
    return hipGetLastError();
}
