// Shared helpers for libfsagg (gfx950 only).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/fsagg.h"

namespace fsagg {

// thread-local last error (fsagg_last_error)
void set_error(const char *fmt, ...);

inline hipStream_t as_stream(fsagg_stream_t s) {
  return reinterpret_cast<hipStream_t>(s);
}

inline bool aligned16(const void *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// Check the launch status once, after the kernel is enqueued.
int check_launch(const char *what);

// Compute units of the current device (cached per device; 256 if the query
// fails) — grid size of the persistent kernels.
int device_cu_count();

constexpr int kWave = 64;

// fp32 loads through a pointer read from a device table: the address space
// is stated so the compiler emits global_load (not flat_load, which also
// holds lgkmcnt); _nt marks data that is streamed once.
typedef __attribute__((address_space(1))) const float global_f32;
__device__ __forceinline__ float gload(const float *p) {
  return *(global_f32 *)(p);
}
__device__ __forceinline__ float gload_nt(const float *p) {
  return __builtin_nontemporal_load((global_f32 *)(p));
}
// Any element type.  (Why it matters: a pointer read from a table is
// generic, so a plain dereference becomes flat_load, which also counts in
// lgkmcnt — the next scalar load of a row pointer then waits for every
// HBM load in flight.)
template <typename T>
__device__ __forceinline__ T gld(const T *p) {
  typedef __attribute__((address_space(1))) const T gT;
  return *(gT *)(p);
}
template <typename T>
__device__ __forceinline__ T gld_nt(const T *p) {
  typedef __attribute__((address_space(1))) const T gT;
  return __builtin_nontemporal_load((gT *)(p));
}

// Grid size for a streaming kernel: enough workgroups to fill 256 CUs a few
// times over, never more than the work needs.
inline unsigned stream_grid(int64_t work_items, int block, int64_t cap) {
  int64_t g = (work_items + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<unsigned>(g);
}

// IEEE single ops that the compiler may not contract into an FMA.  The
// library is also compiled with -ffp-contract=off; these make the intent
// explicit at the call sites that the bit-exact contract depends on.
__device__ __forceinline__ float mul_rn(float a, float b) {
  return __fmul_rn(a, b);
}
__device__ __forceinline__ float add_rn(float a, float b) {
  return __fadd_rn(a, b);
}

// Order-preserving float <-> uint32 key (total order, -0 < +0).
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}

}  // namespace fsagg
