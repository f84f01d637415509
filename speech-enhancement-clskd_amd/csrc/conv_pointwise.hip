// Pointwise (1x1) channel lift for fp32 activations: the ReviewKD ABF conv1
// (framework.py:179-182, Cin = 8..64 student channels -> mid = 64), at every student
// resolution (up to B x 128 x T rows).
//
// With K <= 64 and N <= 64 the op moves far more bytes than it computes (K*N FMAs per row
// against 4K + N*osize bytes): the implicit-GEMM engine spends its time in per-block table
// set-up, one barrier-bound K-tile and 2-byte scatter stores (1.4 TB/s measured on the largest
// level).  Here the op is a streaming kernel:
//   * weights transposed once per block into LDS ([k][n], 16 KB at K = N = 64);
//   * TPR = N/8 threads per output row, each owning 8 output channels of 128/(256/TPR) rows:
//     the 8 weights of a k are one pair of ds_read_b128, broadcast to the lanes of the same
//     channel group and reused across the thread's rows;
//   * the input row is read 16 B at a time (all TPR threads of a row read the same bytes:
//     one cache line feeds them), fp32 FMAs in ascending k;
//   * outputs leave as one 16-B (bf16) or two 16-B (fp32) stores per row and thread, so a
//     wave writes whole rows;
//   * fused BatchNorm statistics with the engines' contract: per 128-row block, fp64 partials
//     {sum, sumsq} of the biased outputs at stats[block][N][2] (fp32 over a thread's rows,
//     fp64 across lanes and waves in a fixed order).
// Same descriptor as the engines (include/clskd.h); eligibility is decided on the host
// (pointwise_ok) and everything else runs the engines.
#include <stdlib.h>

#include "common.h"

namespace clskd {

typedef __bf16 bf16x8p __attribute__((ext_vector_type(8)));

template <int N, int C, typename OutT>
__global__ __launch_bounds__(256, 4) void conv_pointwise_kernel(const clskd_conv_desc d) {
  constexpr int TPR = N / 8;       // threads per output row
  constexpr int RPP = 256 / TPR;   // rows per pass of the block
  constexpr int NPASS = 128 / RPP; // rows per thread
  __shared__ __attribute__((aligned(16))) float wl[C * N];  // [k][n]
  __shared__ double red[4][N][2];
  const int tid = threadIdx.x;
  const float* wg = reinterpret_cast<const float*>(d.weight);
  for (int i = tid; i < C * N; i += 256) {
    const int k = i / N, n = i - (i / N) * N;
    wl[i] = wg[(int64_t)n * d.K + k];
  }
  const int cg = tid % TPR, rg = tid / TPR;
  const int n0 = cg * 8;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t m0 = (int64_t)blockIdx.x * 128;
  const int FoTo = d.Fo * d.To;
  const float* const xb = d.seg[0].ptr;
  int xo[NPASS], orow[NPASS];  // element offsets (< 2^31, checked on the host)
  bool ok[NPASS];
#pragma unroll
  for (int p = 0; p < NPASS; ++p) {
    const int64_t m = m0 + rg + p * RPP;
    ok[p] = m < M;
    const int mm = ok[p] ? (int)m : 0;
    const int b = mm / FoTo;
    const int r = mm - b * FoTo;
    const int fo = r / d.To;
    const int to = r - fo * d.To;
    xo[p] = b * (int)d.seg[0].sB + fo * (int)d.seg[0].sF + to * (int)d.seg[0].sT;
    orow[p] = b * (int)d.oB + (fo * d.of_mul + d.of_add) * (int)d.oF + to * (int)d.oT + n0;
  }
  float acc[NPASS][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float bv = d.bias ? d.bias[n0 + j] : 0.f;
#pragma unroll
    for (int p = 0; p < NPASS; ++p) acc[p][j] = bv;
  }
  __syncthreads();
  f32x4 xv[NPASS];
#pragma unroll
  for (int p = 0; p < NPASS; ++p)
    xv[p] = ok[p] ? *reinterpret_cast<const f32x4*>(xb + xo[p]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int k4 = 0; k4 < C; k4 += 4) {
    f32x4 xn[NPASS];
    if (k4 + 4 < C) {  // prefetch the next 4 channels of every row
#pragma unroll
      for (int p = 0; p < NPASS; ++p)
        xn[p] = ok[p] ? *reinterpret_cast<const f32x4*>(xb + xo[p] + k4 + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(&wl[(k4 + kk) * N + n0]);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(&wl[(k4 + kk) * N + n0 + 4]);
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const float xs = xv[p][kk];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[p][j] = fmaf(xs, w0[j], acc[p][j]);
          acc[p][4 + j] = fmaf(xs, w1[j], acc[p][4 + j]);
        }
      }
    }
    if (k4 + 4 < C) {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) xv[p] = xn[p];
    }
  }
  // ---- stores: one row segment of 8 channels per thread and row ----
  OutT* outp = reinterpret_cast<OutT*>(d.out);
#pragma unroll
  for (int p = 0; p < NPASS; ++p) {
    if (!ok[p]) continue;
    if constexpr (sizeof(OutT) == 2) {
      bf16x8p v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)acc[p][j];
      *reinterpret_cast<bf16x8p*>(outp + orow[p]) = v;
    } else {
      *reinterpret_cast<f32x4*>(outp + orow[p]) = f32x4{acc[p][0], acc[p][1], acc[p][2], acc[p][3]};
      *reinterpret_cast<f32x4*>(outp + orow[p] + 4) = f32x4{acc[p][4], acc[p][5], acc[p][6], acc[p][7]};
    }
  }
  if (!d.stats) return;
  // ---- fused BN statistics: fp32 over the thread's rows, fp64 across lanes and waves ----
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      if (ok[p]) {
        s += acc[p][j];
        q = fmaf(acc[p][j], acc[p][j], q);
      }
    }
    double ds = s, dq = q;
#pragma unroll
    for (int o = TPR; o < 64; o <<= 1) {  // lanes of the same channel group
      ds += __shfl_xor(ds, o, 64);
      dq += __shfl_xor(dq, o, 64);
    }
    if (lane < TPR) {
      red[wave][n0 + j][0] = ds;
      red[wave][n0 + j][1] = dq;
    }
  }
  __syncthreads();
  if (tid < N) {
    const double S = ((red[0][tid][0] + red[1][tid][0]) + red[2][tid][0]) + red[3][tid][0];
    const double Q = ((red[0][tid][1] + red[1][tid][1]) + red[2][tid][1]) + red[3][tid][1];
    d.stats[((int64_t)blockIdx.x * N + tid) * 2] = S;
    d.stats[((int64_t)blockIdx.x * N + tid) * 2 + 1] = Q;
  }
}

static bool pointwise_ok(const clskd_conv_desc& d) {
  const bool off = knob(KNOB_NO_POINTWISE) == 1;  // A/B switch: 1 keeps 1x1 lifts on the engine
  if (off) return false;
  if (d.compute != CLSKD_F32 || d.in_dtype != CLSKD_F32 || d.wlayout != CLSKD_WLAYOUT_NK ||
      d.accumulate)
    return false;
  if (d.ntaps != 1 || d.tap_df[0] != 0 || d.tap_dt[0] != 0 || d.nseg != 1 || d.stride_f != 1 ||
      d.stride_t != 1)
    return false;
  const int C = d.seg_c[0];
  if (C != d.ctot || !(C == 8 || C == 16 || C == 32 || C == 64) || d.K < C) return false;
  if (!(d.N == 32 || d.N == 64) || d.nlo < d.N || d.oNlo != 1) return false;
  const clskd_seg& s = d.seg[0];
  if (((uintptr_t)s.ptr & 15) || s.sB % 4 || s.sF % 4 || s.sT % 4) return false;
  const int al = d.out_dtype == CLSKD_BF16 ? 8 : 4;  // 16-B output segments
  if (((uintptr_t)d.out & 15) || d.oB % al || d.oF % al || d.oT % al) return false;
  if ((int64_t)d.B * d.Fo * d.To >= INT32_MAX) return false;
  // 32-bit element offsets of every row's input and output segment
  const int64_t xmax = (int64_t)(d.B - 1) * s.sB + (int64_t)(d.Fo - 1) * s.sF + (int64_t)(d.To - 1) * s.sT + C;
  const int64_t omax = (int64_t)(d.B - 1) * d.oB + (int64_t)((d.Fo - 1) * d.of_mul + d.of_add) * d.oF +
                       (int64_t)(d.To - 1) * d.oT + d.N;
  if (s.sB < 0 || s.sF < 0 || s.sT < 0 || d.oB < 0 || d.oF < 0 || d.oT < 0 || xmax >= INT32_MAX ||
      omax >= INT32_MAX)
    return false;
  return true;
}

template <int N, int C>
static void launch_pw(const clskd_conv_desc& d, hipStream_t st) {
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const dim3 grid((unsigned)cdiv(M, 128));
  if (d.out_dtype == CLSKD_BF16) {
    hipLaunchKernelGGL((conv_pointwise_kernel<N, C, __bf16>), grid, dim3(256), 0, st, d);
    note_kernel_fn((const void*)conv_pointwise_kernel<N, C, __bf16>);
    note_kernel("conv_pointwise_kernel<%d,%d,bf16>", N, C);
  } else {
    hipLaunchKernelGGL((conv_pointwise_kernel<N, C, float>), grid, dim3(256), 0, st, d);
    note_kernel_fn((const void*)conv_pointwise_kernel<N, C, float>);
    note_kernel("conv_pointwise_kernel<%d,%d,float>", N, C);
  }
}

template <int N>
static void launch_pw_c(const clskd_conv_desc& d, hipStream_t st) {
  switch (d.seg_c[0]) {
    case 8: launch_pw<N, 8>(d, st); break;
    case 16: launch_pw<N, 16>(d, st); break;
    case 32: launch_pw<N, 32>(d, st); break;
    default: launch_pw<N, 64>(d, st); break;
  }
}

bool conv_pointwise_takes(const clskd_conv_desc& d) { return pointwise_ok(d); }

int launch_conv_pointwise(const clskd_conv_desc& d, hipStream_t st, bool* launched) {
  *launched = false;
  if (!pointwise_ok(d)) return CLSKD_OK;
  if (d.N == 64) launch_pw_c<64>(d, st);
  else launch_pw_c<32>(d, st);
  *launched = true;
  return CLSKD_OK;
}

}  // namespace clskd
