// vcfc_device.h -- device-side launch interface shared by the C-ABI
// (vcfc_api.cpp) and the kernels (vcfc_encode.hip).  Plain pointers only.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

// status codes (identical to include/vcfc.h)
#define VCFCD_OK 0
#define VCFCD_E_LT8COLS 1
#define VCFCD_E_8COLS 2
#define VCFCD_E_NOSPACE 4

// error word: min over failing rows of (row << 8 | code); ~0 = no error
#define VCFCD_NO_ERROR (~0ull)

struct VcfcEncodeArgs {
    // input: concatenated VCF data lines (device memory)
    const uint8_t *buf;
    const uint64_t *line_off;  // byte offset of line i in buf
    const uint32_t *line_len;  // length of line i, without '\n'
    uint64_t n;                // rows
    // output
    uint8_t *out;              // records, concatenated in row order
    uint64_t out_cap;
    uint64_t *rec_off;         // n + 1 exclusive offsets; rec_off[n] = total
    // workspace (see vcfc_encode_workspace_layout)
    uint64_t *slot_off;        // n + 1
    uint32_t *rec_size;        // n
    uint64_t *partials;        // scan partials
    uint64_t *err;             // 1 word
    uint32_t *retry;           // rows the fast kernel hands to the general one
    uint32_t *retry_count;
    uint8_t *slots;            // per-row staging slots
    uint64_t slots_cap;
};

struct VcfcWorkspaceLayout {
    uint64_t slot_off, rec_size, partials, err, retry, retry_count, slots, total;
};

// Bytes of per-row staging for a line of `len` bytes: covers the worst-case
// record (8 + len + (len+1)/2 + 2) plus the 16-byte flush granule.
__host__ __device__ inline uint64_t vcfc_slot_bytes(uint32_t len) {
    return ((uint64_t)len + (len >> 1) + 48 + 15) & ~15ull;
}

// Workspace layout for n rows whose line lengths sum to <= total_line_bytes.
VcfcWorkspaceLayout vcfc_encode_workspace_layout(uint64_t n, uint64_t total_line_bytes);

// Enqueue the whole encode on `stream` (no host synchronisation, capturable).
// If `ev` is non-null, ev[0..4] are recorded before the slot scan, after it,
// after k_encode, after the size scan and after k_compact.
hipError_t vcfc_encode_device(const VcfcEncodeArgs &a, hipStream_t stream, hipEvent_t *ev = nullptr);
