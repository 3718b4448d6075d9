// TEST INFRASTRUCTURE ONLY: minimal <hip/hip_runtime.h> stand-in so the
// product kernel sources compile with g++ against the fiber SIMT emulator.
#pragma once
#include <cstdint>
#include <cstring>
#include <cstddef>
#include "../emu.h"

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static
#define __restrict__

struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct uint4 { uint32_t x, y, z, w; };
struct uint2 { uint32_t x, y; };
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
inline uint2 make_uint2(uint32_t a, uint32_t b) { return uint2{a, b}; }

#define threadIdx (emu::g.cur->tid)
#define blockIdx (emu::g.bid)
#define blockDim (emu::g.block)
#define gridDim (emu::g.grid)

typedef void *hipStream_t;
typedef void *hipEvent_t;
inline int hipEventRecord(hipEvent_t, hipStream_t) { return 0; }
typedef int hipError_t;
#define hipSuccess 0
inline hipError_t hipGetLastError() { return hipSuccess; }
inline const char *hipGetErrorString(hipError_t) { return "emu"; }
inline hipError_t hipMemsetAsync(void *p, int v, size_t n, hipStream_t) { memset(p, v, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, int, hipStream_t) { memmove(d, s, n); return hipSuccess; }
#define hipMemcpyDeviceToDevice 3
#define hipMemcpyHostToDevice 1
#define hipMemcpyDeviceToHost 2
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
#define hipStreamNonBlocking 1
#define hipEventDisableTiming 2
inline hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = nullptr; return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
inline hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = nullptr; return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
#define hipDeviceAttributeMultiprocessorCount 0
inline hipError_t hipDeviceGetAttribute(int *v, int, int) { *v = 4; return hipSuccess; }
template <class F> inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int *n, F, int, size_t) { *n = 2; return hipSuccess; }

inline void __syncthreads() { emu::collective(emu::OP_SYNCTHREADS, 0, 0, 0); }

template <class T> inline T atomicAdd(T *p, T v) { T o = *p; *p = o + v; return o; }
// agent-scope relaxed loads/stores (blocks run one after the other here)
#define __HIP_MEMORY_SCOPE_AGENT 3
template <class T> inline T __hip_atomic_load(const T *p, int, int) { return *(volatile const T *)p; }
template <class T> inline void __hip_atomic_store(T *p, T v, int, int) { *(volatile T *)p = v; }
inline void __builtin_amdgcn_s_sleep(int) {}
template <class T> inline T atomicMin(T *p, T v) { T o = *p; if (v < o) *p = v; return o; }
template <class T> inline T atomicMax(T *p, T v) { T o = *p; if (v > o) *p = v; return o; }
template <class T> inline T atomicOr(T *p, T v) { T o = *p; *p = o | v; return o; }
template <class T> inline T atomicExch(T *p, T v) { T o = *p; *p = v; return o; }

inline emu::dim3v emu_dim(dim3 d) { emu::dim3v r; r.x = d.x; r.y = d.y; r.z = d.z; return r; }
#define hipLaunchKernelGGL(K, G, B, SHM, STREAM, ...) \
    emu::launch(emu_dim(dim3(G)), emu_dim(dim3(B)), [=]() { K(__VA_ARGS__); })
