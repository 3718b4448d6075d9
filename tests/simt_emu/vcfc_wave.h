// TEST INFRASTRUCTURE ONLY: emulated twin of
// vcf-compression_amd/csrc/vcfc_wave.h (same API, fiber-emulated wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace vw {
inline uint32_t lane_id() { return emu::lane(); }
inline uint64_t ballot(bool p) { return emu::collective(emu::OP_BALLOT, p ? 1 : 0, 0, 0); }
inline uint64_t lanemask_lt() { uint32_t l = lane_id(); return l == 0 ? 0ull : (~0ull >> (64 - l)); }
inline uint32_t shfl(uint32_t v, uint32_t src) { return (uint32_t)emu::collective(emu::OP_SHFL, v, src & 63, 0); }
inline uint32_t readlane(uint32_t v, uint32_t l) { return shfl(v, l); }
inline uint32_t readfirst(uint32_t v) { return (uint32_t)emu::collective(emu::OP_READFIRST, v, 0, 0); }
inline uint32_t dpp(uint32_t old, uint32_t src, int ctrl, int rm, int bm, bool bc) {
    uint64_t c = (uint64_t)ctrl | ((uint64_t)rm << 16) | ((uint64_t)bm << 20) | ((uint64_t)(bc ? 1 : 0) << 24);
    return (uint32_t)emu::collective(emu::OP_DPP, old, src, c);
}
inline uint32_t shr1(uint32_t v, uint32_t fill) { return dpp(fill, v, 0x138, 0xf, 0xf, false); }
inline uint32_t shr1z(uint32_t v) { return shr1(v, 0u); }
inline uint32_t shl1(uint32_t v, uint32_t fill) { return dpp(fill, v, 0x130, 0xf, 0xf, false); }
inline uint32_t row_shl1(uint32_t v) { return dpp(0u, v, 0x101, 0xf, 0xf, false); }
inline uint32_t scan_add(uint32_t v) {
    v += dpp(0u, v, 0x111, 0xf, 0xf, false);
    v += dpp(0u, v, 0x112, 0xf, 0xf, false);
    v += dpp(0u, v, 0x114, 0xf, 0xf, false);
    v += dpp(0u, v, 0x118, 0xf, 0xf, false);
    v += dpp(0u, v, 0x142, 0xa, 0xf, false);
    v += dpp(0u, v, 0x143, 0xc, 0xf, false);
    return v;
}
inline uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
inline uint32_t scan_max(uint32_t v) {
    v = umax(v, dpp(0u, v, 0x111, 0xf, 0xf, false));
    v = umax(v, dpp(0u, v, 0x112, 0xf, 0xf, false));
    v = umax(v, dpp(0u, v, 0x114, 0xf, 0xf, false));
    v = umax(v, dpp(0u, v, 0x118, 0xf, 0xf, false));
    v = umax(v, dpp(0u, v, 0x142, 0xa, 0xf, false));
    v = umax(v, dpp(0u, v, 0x143, 0xc, 0xf, false));
    return v;
}
inline uint32_t last_nz(uint32_t v, uint32_t t) { return v ? v : t; }
inline uint32_t scan_last_nz(uint32_t v) {
    v = last_nz(v, dpp(0u, v, 0x111, 0xf, 0xf, false));
    v = last_nz(v, dpp(0u, v, 0x112, 0xf, 0xf, false));
    v = last_nz(v, dpp(0u, v, 0x114, 0xf, 0xf, false));
    v = last_nz(v, dpp(0u, v, 0x118, 0xf, 0xf, false));
    v = last_nz(v, dpp(0u, v, 0x142, 0xa, 0xf, false));
    v = last_nz(v, dpp(0u, v, 0x143, 0xc, 0xf, false));
    return v;
}
inline uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (s & 3)));
}
inline uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t k = (sel >> (8 * i)) & 0xFFu;
        uint32_t b;
        if (k < 8) b = (uint32_t)(v >> (8 * k)) & 0xFFu;
        else if (k == 8) b = (s1 >> 15) & 1 ? 0xFFu : 0u;
        else if (k == 9) b = (s1 >> 31) & 1 ? 0xFFu : 0u;
        else if (k == 10) b = (s0 >> 15) & 1 ? 0xFFu : 0u;
        else if (k == 11) b = (s0 >> 31) & 1 ? 0xFFu : 0u;
        else if (k == 12) b = 0u;
        else b = 0xFFu;
        r |= b << (8 * i);
    }
    return r;
}
inline uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
inline int32_t sext24(int32_t v) { return (int32_t)((uint32_t)v << 8) >> 8; }
inline int32_t mad24(int32_t a, int32_t b, int32_t x) { return (int32_t)((uint32_t)x + (uint32_t)(sext24(a) * sext24(b))); }
inline uint32_t umul24(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)(a & 0xFFFFFFu) * (b & 0xFFFFFFu)); }
inline int32_t mulsel(int32_t f, int32_t x) { return (int32_t)((uint32_t)sext24(f) * (uint32_t)sext24(x)); }
inline uint32_t dot4u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r = c;
    for (int i = 0; i < 4; i++) r += ((a >> (8 * i)) & 0xFFu) * ((b >> (8 * i)) & 0xFFu);
    return r;
}
struct ldsp { uint8_t *a; };
inline ldsp lds_sel(uint8_t *lds, int32_t f, int32_t x, int32_t dm) { return ldsp{lds + mad24(f, x, dm)}; }
template <int OFF, bool HI> inline void lds_st8(ldsp p, uint32_t v) { p.a[OFF] = (uint8_t)(HI ? (v >> 16) : v); }
inline void lds_st32(ldsp p, uint32_t v) { memcpy(p.a, &v, 4); }
inline uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
inline int32_t sbit(uint32_t x, uint32_t bit) { return ((x >> bit) & 1u) ? -1 : 0; }
inline void wave_sync() { emu::collective(emu::OP_WAVESYNC, 0, 0, 0); }
// lowest set bit index; value unspecified for 0 (v_ffbl_b32: callers must not use it)
inline uint32_t ffbl(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
inline int popc64(uint64_t m) { return __builtin_popcountll(m); }
inline int hibit64(uint64_t m) { return 63 - __builtin_clzll(m); }
inline uint32_t mulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
inline uint4 gload16(const void *base, uint32_t idx) { return ((const uint4 *)base)[idx]; }
inline uint4 uload16(const void *p) { uint4 v; memcpy(&v, p, 16); return v; }
inline uint32_t gload4(const void *base, uint32_t idx) { return ((const uint32_t *)base)[idx]; }
inline void gstore16(void *base, uint64_t byte_off, uint4 v) { *(uint4 *)((uint8_t *)base + byte_off) = v; }
inline void gstore16_nt(void *base, uint64_t byte_off, uint4 v) { gstore16(base, byte_off, v); }
struct brsrc { const uint8_t *base; uint32_t bytes; };
inline brsrc make_rsrc(const void *base, uint32_t bytes) { return brsrc{(const uint8_t *)base, bytes}; }
inline uint32_t bload_dw(brsrc r, uint32_t off) {
    if ((uint64_t)off + 4 > r.bytes) return 0u;   // per-dword range check
    uint32_t v; memcpy(&v, r.base + off, 4); return v;
}
inline uint4 bload16(brsrc r, uint32_t off, int = 0) {   // (cache policy: no effect here)
    return make_uint4(bload_dw(r, off), bload_dw(r, off + 4), bload_dw(r, off + 8), bload_dw(r, off + 12));
}
inline uint32_t bload4(brsrc r, uint32_t off, int = 0) { return bload_dw(r, off); }
inline void pin_loads() {}
}  // namespace vw
