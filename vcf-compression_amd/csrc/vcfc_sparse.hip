// vcfc_sparse.hip -- sparse-file layout of `.vcfc` records (reference
// sparsify_file, src/sparse.cpp:290-580; offsets compute_sparse_offset,
// src/sparse.cpp:18-51).
//
// Each record i goes to file offset  data_start + (L + POS_i) * F * B  with
// L = 300,000,000, F = 4, B = 4096 (src/sparse.hpp:29-32; CHROM ignored because
// VCFC_SPARSE_MULTIPLE_REF_PER_FILE is false, :15), prefixed by 16 bytes:
// BE(dist_to_prev) BE(dist_to_next).  k_sparse_plan computes, one thread per
// record, POS (strtoul of the 2nd column), the file offset and the 16-byte
// prefix from the neighbours' offsets, and flags any layout where records
// overlap or are out of order (the host then replays the reference's exact
// write sequence).  The bytes themselves are written by the host (pwritev).
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>
#include "vcfc_device.h"

namespace {

constexpr uint64_t SPARSE_L = 300000000ull, SPARSE_STRIDE = 4ull * 4096ull;

// POS of record r (body = bytes after its 8 header bytes); false = the
// reference throws (empty CHROM/POS, POS not a whole strtoul number)
__device__ bool record_pos(const uint8_t *rec, uint64_t body, uint64_t *pos) {
    const uint8_t *b = rec + 8;
    uint64_t p = 0;
    while (p < body && b[p] != '\t') p++;
    *pos = 0;
    if (p >= body) return true;          // CHROM never terminated: POS stays 0
    if (p == 0) return false;            // empty CHROM
    const uint64_t ps = ++p;
    while (p < body && b[p] != '\t') p++;
    if (p >= body) return true;          // POS never terminated: stays 0
    if (p == ps) return false;           // empty POS
    uint64_t i = ps;
    while (i < p && (b[i] == ' ' || (b[i] >= '\t' && b[i] <= '\r'))) i++;
    bool neg = false;
    if (i < p && (b[i] == '+' || b[i] == '-')) { neg = b[i] == '-'; i++; }
    if (i >= p || b[i] < '0' || b[i] > '9') return false;
    uint64_t v = 0;
    bool ovf = false;
    for (; i < p && b[i] >= '0' && b[i] <= '9'; i++) {
        const uint64_t d = b[i] - '0';
        if (v > (~0ull - d) / 10) ovf = true;
        v = v * 10 + d;
    }
    if (i != p) return false;
    *pos = ovf ? ~0ull : (neg ? 0 - v : v);
    return true;
}

__device__ __forceinline__ void be64(uint8_t *o, uint64_t v) {
    for (int k = 0; k < 8; k++) o[k] = (uint8_t)(v >> (56 - 8 * k));
}

__global__ __launch_bounds__(256) void k_sparse_plan(const uint8_t *recs, const uint64_t *rec_off, uint64_t n,
                                                     uint64_t data_start, uint64_t *file_off, uint8_t *prefix,
                                                     uint64_t *status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t off[3];
    bool ok = true;
    for (int k = 0; k < 3; k++) {
        const int64_t j = (int64_t)i + k - 1;
        off[k] = 0;
        if (j < 0 || (uint64_t)j >= n) continue;
        uint64_t pos = 0;
        const uint64_t body = rec_off[j + 1] - rec_off[j] - 8;
        if (!record_pos(recs + rec_off[j], body, &pos)) { if (j == (int64_t)i) ok = false; continue; }
        off[k] = (SPARSE_L + pos) * SPARSE_STRIDE + data_start;
    }
    if (!ok) {
        atomicMin((unsigned long long *)&status[0], (unsigned long long)((i << 8) | 8u /* VCFC_E_FORMAT */));
        return;
    }
    file_off[i] = off[1];
    const uint64_t prev = i == 0 ? data_start : off[0];
    const uint64_t next = i + 1 < n ? off[2] - off[1] : 0;   // the last record's stays 0
    be64(prefix + 16 * i, off[1] - prev);
    be64(prefix + 16 * i + 8, next);
    // anomaly: the straight "one write per record" plan equals the reference's
    // sequential writes only if records do not overlap each other or the
    // first-offset slot and appear in increasing offset order
    const uint64_t len = 16 + (rec_off[i + 1] - rec_off[i]);
    bool anomaly = off[1] < data_start;
    if (i + 1 < n) anomaly |= off[2] <= off[1] || off[1] + len > off[2];
    if (anomaly) atomicOr((unsigned long long *)&status[1], 1ull);
}

}  // namespace

hipError_t vcfc_sparse_plan_launch(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t data_start,
                                   uint64_t *file_off, uint8_t *prefix, uint64_t *status, hipStream_t s) {
    hipError_t e = hipMemsetAsync(status, 0xFF, 8, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(status + 1, 0, 8, s)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sparse_plan, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, recs, rec_off, n,
                       data_start, file_off, prefix, status);
    return hipGetLastError();
}
