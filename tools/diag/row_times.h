// Diagnostic hooks (tools/row_times.py): per-row start/end wall clock of
// k_encode_fast into the workspace's dbg region.  Build a separate library:
//   make -C vcf-compression_amd B=$PWD/build_rt EXTRA='-DVCFC_DIAG="\"$PWD/tools/diag/row_times.h\""'
#pragma once
#define VCFC_DIAG_ROW_BEGIN() const uint64_t vcfc_diag_t0 = wall_clock64()
#define VCFC_DIAG_ROW_END(a, row)                                                             \
    if (vw::lane_id() == 0) {                                                                 \
        (a).dbg[2 * (row)] = vcfc_diag_t0;                                                    \
        (a).dbg[2 * (row) + 1] = wall_clock64();                                              \
    }
#define VCFC_DIAG_GENERAL_ROW(a)
#define VCFC_DIAG_WS_BYTES(n) (16ull * (n))
