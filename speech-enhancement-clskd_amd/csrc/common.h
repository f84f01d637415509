// Shared device/host helpers for libclskd_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/clskd.h"

namespace clskd {

// ---- host-side error plumbing (thread-local message; no exceptions across the C ABI) ----------
void set_error(const char* fmt, ...);
// Instance name of the kernel the calling thread's last conv launch ran ("base<arg,...>", the
// template arguments rocprof shows); read back through clskd_conv_last_kernel().
void note_kernel(const char* fmt, ...);
template <typename T> inline const char* type_name();
template <> inline const char* type_name<float>() { return "float"; }
template <> inline const char* type_name<__bf16>() { return "bf16"; }

#define CLSKD_CHECK_ARG(cond, ...)                 \
  do {                                             \
    if (!(cond)) {                                 \
      ::clskd::set_error(__VA_ARGS__);             \
      return CLSKD_E_ARG;                          \
    }                                              \
  } while (0)

#define CLSKD_CHECK_SHAPE(cond, ...)               \
  do {                                             \
    if (!(cond)) {                                 \
      ::clskd::set_error(__VA_ARGS__);             \
      return CLSKD_E_SHAPE;                        \
    }                                              \
  } while (0)

#define CLSKD_LAUNCH_CHECK(name)                                                  \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::clskd::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));   \
      return CLSKD_E_HIP;                                                         \
    }                                                                             \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- device helpers ---------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD-aware tile order: the hardware places workgroup i on XCD i % 8.  Give every XCD one
// contiguous run of M-tiles (a bijection on [0, nb)), so neighbouring tiles — which read
// overlapping input rows through the conv taps — share that XCD's L2 instead of each of the
// eight L2s fetching the same rows.
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7, j = bid >> 3;
  return x * q + (x < r ? x : r) + j;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace clskd
