// TEST INFRASTRUCTURE ONLY: diagnostic hooks for the emulator build -- count
// the rows that take the general path (emu_api.cpp reads it).
#pragma once
#define VCFC_DIAG_ROW_BEGIN()
#define VCFC_DIAG_ROW_END(a, row)
#define VCFC_DIAG_GENERAL_ROW(a) \
    if (vw::lane_id() == 0) atomicAdd((a).retry_count, 1u)
#define VCFC_DIAG_WS_BYTES(n) 0ull
// bytes the hop line index's walkers load (k_nl_hop), summed per process
void emu_diag_hop_read(unsigned long long bytes);
#define VCFC_DIAG_HOP_READ(bytes) emu_diag_hop_read((unsigned long long)(bytes))
