// vcfc_wave.h -- wave64 primitives for the gfx950 kernels.
//
// Everything the kernels need from the CDNA4 wave: lane id, ballot, DPP
// scans, cross-lane shifts, alignbyte.  Scans are built from DPP row_shr /
// row_bcast so they cost VALU slots only (no LDS round trip).
//
// tests/simt_emu/ provides a drop-in header of the same name that emulates
// these primitives on the CPU (64 fibers per wave) so the kernel source can be
// exercised without a GPU; this file is the only implementation the product
// library is built with.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vw {

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return __builtin_amdgcn_readlane(v, l);
}
__device__ __forceinline__ uint32_t readfirst(uint32_t v) {
    return __builtin_amdgcn_readfirstlane(v);
}
// lane i receives lane i-1's value; lane 0 receives `fill` (DPP wave_shr:1)
__device__ __forceinline__ uint32_t shr1(uint32_t v, uint32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false);
}
// lane i receives lane i-1's value; lane 0 receives 0 (one v_mov_b32_dpp)
__device__ __forceinline__ uint32_t shr1z(uint32_t v) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xf, 0xf, true);
}
// lane i receives lane i+1's value; lane 63 receives `fill` (DPP wave_shl:1)
__device__ __forceinline__ uint32_t shl1(uint32_t v, uint32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false);
}
// lane i receives lane i+1's value within its row of 16 lanes; the last
// lane of each row receives 0 (DPP row_shl:1)
__device__ __forceinline__ uint32_t row_shl1(uint32_t v) {
    return __builtin_amdgcn_update_dpp(0u, v, 0x101, 0xf, 0xf, false);
}
// generic lane gather (ds_bpermute)
__device__ __forceinline__ uint32_t shfl(uint32_t v, uint32_t src) {
    return __builtin_amdgcn_ds_bpermute(src << 2, v);
}
// inclusive add scan over the wave.  Written out in asm: hipcc does not
// always fold the update_dpp + add pairs into v_add_u32_dpp (3 VALU per step
// instead of 1).  s_nop 1 covers the VALU-write -> DPP-read hazard (2 wait
// states), including the producer of v before the block.
__device__ __forceinline__ uint32_t scan_add(uint32_t v) {
    asm volatile(
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
// inclusive unsigned-max scan over the wave (identity 0)
__device__ __forceinline__ uint32_t scan_max(uint32_t v) {
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false));
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false));
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false));
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false));
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false));
    v = umax(v, __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false));
    return v;
}
// inclusive "last non-zero" scan: lane l gets the value of the highest lane
// <= l whose v is non-zero (0 if none); DPP steps as scan_max
// Written out in asm as scan_add: one compare and one v_cndmask_b32 with the
// DPP source per step (v stays where it is non-zero, else takes the shifted
// value; lanes outside the row read 0 / are not written), where hipcc emits
// a zeroing move, a DPP move, a compare and a select.  The compare and an
// s_nop 0 are the two wait states before each DPP read of v.
__device__ __forceinline__ uint32_t scan_last_nz(uint32_t v) {
    asm volatile(
        "s_nop 1\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "v_cmp_ne_u32 vcc, 0, %0\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_dpp %0, %0, %0, vcc row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(v)
        :
        : "vcc");
    return v;
}
// byte select: result byte i = byte sel[i] of (s0:s1) for sel 0..7, 0x0C -> 0x00
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
// ((hi:lo) >> s)[31:0], s in 0..31
__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}
// x + a*b on the low 24 bits of a and b, signed (v_mad_i32_i24)
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t x) { return x + __mul24(a, b); }
// (a & 0xFFFFFF) * (b & 0xFFFFFF), low 32 bits (v_mul_u32_u24, full rate)
__device__ __forceinline__ uint32_t umul24(uint32_t a, uint32_t b) { return __umul24(a, b); }
// sum of the byte products a_i * b_i, + c (v_dot4_u32_u8, one instruction):
// with b = 0x08040201 and bytes of a in {0, 1}, the four bytes' flags as 4 bits
__device__ __forceinline__ uint32_t dot4u(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot4(a, b, c, false);
}
// f * x for a flag f in {0, 1} and x in signed 24 bits, as one v_mul_i32_i24
// (left to itself the compiler turns some of these selects into a bit test,
// a compare, an add and a v_cndmask)
// bits of a where m is set, of b elsewhere (v_bfi_b32), m a 0 / ~0 flag:
// one instruction where the compiler's select takes a compare and a v_cndmask
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    __asm__("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// bit `bit` of x sign-extended: 0 or ~0 (v_bfe_i32)
__device__ __forceinline__ int32_t sbit(uint32_t x, uint32_t bit) { return __builtin_amdgcn_sbfe((int32_t)x, bit, 1); }
__device__ __forceinline__ int32_t mulsel(int32_t f, int32_t x) {
    int32_t r;
    __asm__("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(f), "v"(x));
    return r;
}
// LDS byte stores at lds + dm + f * x + OFF (f a flag in {0, 1}, x and dm
// signed 24-bit): the address is ONE v_mad_i32_i24 whatever the flag, shared
// by stores at offsets 0 and 1, and each store one ds_write_b8 (byte 0 of v)
// or ds_write_b8_d16_hi (byte 2).  Hand-written: left to itself the compiler
// merges the two adjacent byte stores into a ds_write_b16 at an odd address
// (misaligned) and turns some flag multiplies into v_mad_u64_u32.
struct ldsp { uint32_t a; };
__device__ __forceinline__ ldsp lds_sel(uint8_t *lds, int32_t f, int32_t x, int32_t dm) {
    const uint32_t b = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)lds + (uint32_t)dm;
    uint32_t a;
    __asm__("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(a) : "v"(f), "v"(x), "v"(b));
    return ldsp{a};
}
// one unaligned ds_write_b32 (an escape's 0xE1 and its three bytes, esc8)
__device__ __forceinline__ void lds_st32(ldsp p, uint32_t v) {
    __asm__ volatile("ds_write_b32 %0, %1" ::"v"(p.a), "v"(v) : "memory");
}
template <int OFF, bool HI>
__device__ __forceinline__ void lds_st8(ldsp p, uint32_t v) {
    if (HI) __asm__ volatile("ds_write_b8_d16_hi %0, %1 offset:%2" ::"v"(p.a), "v"(v), "i"(OFF) : "memory");
    else __asm__ volatile("ds_write_b8 %0, %1 offset:%2" ::"v"(p.a), "v"(v), "i"(OFF) : "memory");
}
// ((hi:lo) >> 8*s)[31:0]
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
// order LDS traffic between the lanes of one wave (no s_barrier needed)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// lowest set bit index; value unspecified for 0 (v_ffbl_b32: callers must not use it)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
// index of the highest set bit (m != 0)
__device__ __forceinline__ int hibit64(uint64_t m) { return 63 - __clzll(m); }

__device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }

// Global-memory accesses with the address space made explicit, so hipcc
// emits global_load/store (counted by vmcnt) instead of flat_* (whose
// out-of-order completion forces vmcnt(0)+lgkmcnt(0) waits).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cv4u;
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
__device__ __forceinline__ uint4 gload16(const void *base, uint32_t idx) {
    const v4u v = ((g_cv4u *)base)[idx];
    return make_uint4(v.x, v.y, v.z, v.w);
}
// 16 bytes at any byte address (global_load_dwordx4 takes unaligned addresses)
__device__ __forceinline__ uint4 uload16(const void *p) {
    const v4u v = *((g_cv4u *)((__attribute__((address_space(1))) const uint8_t *)p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t gload4(const void *base, uint32_t idx) {
    return ((g_cu32 *)base)[idx];
}
__device__ __forceinline__ void gstore16(void *base, uint64_t byte_off, uint4 v) {
    v4u t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    *((g_v4u *)((__attribute__((address_space(1))) uint8_t *)base + byte_off)) = t;
}
// non-temporal 16-byte store (streamed data no kernel re-reads soon)
__device__ __forceinline__ void gstore16_nt(void *base, uint64_t byte_off, uint4 v) {
    v4u t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    __builtin_nontemporal_store(t, (g_v4u *)((__attribute__((address_space(1))) uint8_t *)base + byte_off));
}
// Raw buffer resource over [base, base + bytes): loads at offsets past
// `bytes` (checked per dword) return 0 instead of touching memory, so
// prefetches past a row's end need no clamping.  The chunk offset goes in
// the VGPR offset: gfx9 leaves the SGPR offset out of the range check.
typedef __amdgpu_buffer_rsrc_t brsrc;
__device__ __forceinline__ brsrc make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
// aux: cache policy bits (0 default, 2 nt)
__device__ __forceinline__ uint4 bload16(brsrc r, uint32_t off, const int aux = 0) {
    const v4u v = aux == 2 ? __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2)
                           : __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t bload4(brsrc r, uint32_t off, const int aux = 0) {
    return aux == 2 ? __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 2)
                    : __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
// Keep just-issued prefetch loads where they are: the memory clobber stops
// LLVM from sinking them towards their (next-iteration) use, which would
// shrink the prefetch distance to zero.  Emits no instruction.
__device__ __forceinline__ void pin_loads() { asm volatile("" ::: "memory"); }
}  // namespace vw
