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
// Host function of that kernel (clskd_conv_last_kernel_fn: the executor's per-kernel timing key).
void note_kernel_fn(const void* fn);
// Dispatch knobs (capi.cpp): env read once at first use, changed only by clskd_set_knob.
enum KnobId {
  KNOB_G8, KNOB_G8_GRID, KNOB_HALO_GRID, KNOB_LSTM_NKS, KNOB_LSTM_NKS32,
  KNOB_WGRAD_WG, KNOB_NO_HALO, KNOB_BF16_WAVES, KNOB_BF16_STAGES, KNOB_BF16_TILE,
  KNOB_NO_POINTWISE, KNOB_ABF_MOMENT_DIV, KNOB_F32_WAVES, KNOB_EXEC_GATE,
  KNOB_NO_HALO32, KNOB_HALO32_SPLIT, KNOB_HALO32_MIN_N, KNOB_G8_KORDER, KNOB_G8_PP, KNOB_F32_SPLIT, KNOB_LSTM_PRIO, KNOB_SPLIT_BK, KNOB_HALOW, KNOB_SPLIT_GRID, KNOB_G8_TA, KNOB_G8_SK, KNOB_SPLIT_PD, KNOB_SPLIT_OCC, KNOB_WGRAD_DEPTH, KNOB_LSTM_BWD_WAVE, KNOB_SPLIT_NS2, KNOB_BN_PFOLD, KNOB_LSTM_PRE, KNOB_ABF_BWD_BLOCKS, KNOB_WGRAD_XCD, KNOB_LSTM_BWD_PIN,
  // timing-only experiment modes (wrong results): -DCLSKD_EXPERIMENTS builds only
  KNOB_LSTM128_TDIV, KNOB_LSTM32_TDIV, KNOB_BF16_DEBUG_MODE, KNOB_SKIP, KNOB_H32_DEBUG_MODE,
  KNOB_COUNT
};
int knob(KnobId k);
// In-place level-2 fold of a [nblk][E] fp64 partial table before a one-workgroup-per-channel
// finalize (norm.hip): returns the row count the finalize then reads (nblk when not folded).
// `bit` = 1 backward finalizes, 2 forward (CLSKD_BN_PFOLD mask).
int fold_partials(double* part, int nblk, int E, int bit, hipStream_t st);
// CLSKD_OK, or CLSKD_E_ARG (with the error message set) when `value` selects a timing-only mode
// in a product build.
int experiment_guard(const char* what, int value);
// Timing-only "what if this kernel family were free" switch (CLSKD_SKIP bit mask, experiments
// build only; always false in the product library): the entry point returns without launching.
enum SkipBit {
  SKIP_BN_FINALIZE = 1, SKIP_BN_APPLY = 2, SKIP_CONV_F32 = 4, SKIP_LSTM = 8, SKIP_ABF = 16,
  SKIP_GRAM = 32, SKIP_CONV_LOWP = 64, SKIP_CONV_DIRECT = 128, SKIP_LSTM_PRE = 256, SKIP_LSTM_BWD = 512
};
bool skip_kernel(int bit);
template <typename T> inline const char* type_name();
template <> inline const char* type_name<float>() { return "float"; }
template <> inline const char* type_name<__bf16>() { return "bf16"; }
template <> inline const char* type_name<_Float16>() { return "f16"; }
// storage-type code of a 16-bit type (clskd_compute)
template <typename T> constexpr int lowp_code() { return sizeof(T) == 4 ? CLSKD_F32 : CLSKD_BF16; }
template <> constexpr int lowp_code<_Float16>() { return CLSKD_F16; }
inline bool is_lowp(int dt) { return dt == CLSKD_BF16 || dt == CLSKD_F16; }

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

// 4 channels of fp32 / bf16 storage <-> f32x4 (8- or 16-B accesses)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ f32x4 load4(const T* p);
template <>
__device__ __forceinline__ f32x4 load4<float>(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}
template <>
__device__ __forceinline__ f32x4 load4<__bf16>(const __bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <>
__device__ __forceinline__ f32x4 load4<_Float16>(const _Float16* p) {
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  const f16x4 v = *reinterpret_cast<const f16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <typename T>
__device__ __forceinline__ void store4(T* p, f32x4 v);
template <>
__device__ __forceinline__ void store4<float>(float* p, f32x4 v) {
  *reinterpret_cast<f32x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<__bf16>(__bf16* p, f32x4 v) {
  bf16x4 o;
  o[0] = (__bf16)v[0];
  o[1] = (__bf16)v[1];
  o[2] = (__bf16)v[2];
  o[3] = (__bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = o;
}

// one v_mfma_f32_32x32x16 on 16-bit operands held as any 16-byte vector (8 lanes of bf16 or
// IEEE half bits): InT selects the bf16 or the f16 instruction (same rate on gfx950)
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
template <typename InT, typename V>
__device__ __forceinline__ f32x16 mfma16(const V& a, const V& b, const f32x16& c) {
  static_assert(sizeof(V) == 16, "8 x 16-bit operand lanes");
  if constexpr (__is_same(InT, _Float16))
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

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

// scale/shift (and batch mean/var, running stats) of one channel from its totals.
__device__ __forceinline__ void bn_channel_coeffs(int c, double S, double Q, int64_t rows,
                                                  const float* gamma, const float* beta, float eps,
                                                  float* running_mean, float* running_var,
                                                  float momentum, int n_updates, float* scale,
                                                  float* shift, float* mean_out, float* var_out) {
  const double n = (double)rows;
  const double mean = S / n;
  double var = Q / n - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float bb = beta ? beta[c] : 0.f;
  const float sc = invstd * g;
  scale[c] = sc;
  shift[c] = bb - (float)mean * sc;
  if (mean_out) mean_out[c] = (float)mean;
  if (var_out) var_out[c] = (float)var;
  if (running_mean && running_var) {
    const float unb = (float)(rows > 1 ? var * n / (n - 1.0) : var);
    float rm = running_mean[c], rv = running_var[c];
    for (int u = 0; u < n_updates; ++u) {
      rm = (1.f - momentum) * rm + momentum * (float)mean;
      rv = (1.f - momentum) * rv + momentum * unb;
    }
    running_mean[c] = rm;
    running_var[c] = rv;
  }
}


// ATen nearest_idx (UpSample.h) for F.interpolate(mode="nearest"): source index of dst.
__device__ __forceinline__ int nearest_src(int dst, int in_size, int out_size) {
  // ATen nearest_idx (UpSample.h): identity / >>1 fast paths, else floorf(dst*scale), scale in f32
  if (out_size == in_size) return dst;
  if (out_size == 2 * in_size) return dst >> 1;
  const float scale = (float)in_size / (float)out_size;
  const int s = (int)floorf((float)dst * scale);
  return s < in_size - 1 ? s : in_size - 1;
}

// masking mode 'E' (norm.hip mask_e_kernel, norm_bwd.hip mask_e_bwd_kernel): MASK_TT frames per
// block; the mask columns [256][2 * MASK_TT] staged in LDS with a padded row (MASK_LD floats: the
// bins of one wave's float2 reads fall on distinct banks)
constexpr int MASK_TT = 16;
constexpr int MASK_LD = 2 * MASK_TT + 2;
// ml[fm][r] = mcol[fm * Tm * 2 + r] for r < 2 * nt (mcol: the block's first column of bin 0)
__device__ __forceinline__ void mask_tile_load(const float* __restrict__ mcol, int Tm, int nt,
                                               float* ml) {
  for (int i = threadIdx.x; i < 256 * 2 * MASK_TT; i += blockDim.x) {
    const int fm = i / (2 * MASK_TT), r = i - fm * 2 * MASK_TT;
    if (r < 2 * nt) ml[fm * MASK_LD + r] = mcol[(int64_t)fm * Tm * 2 + r];
  }
}

}  // namespace clskd
