// Backward-pass GEMMs and optimizer kernels (student training step, SURVEY.md §8 f rank 1).
//
// conv_wgrad_f32: the weight gradient of any launch of the implicit-GEMM conv engine, read
// through the SAME descriptor as the forward launch (segments, K table, output map):
//     dW[n][k] = sum_m dY(m, n) * A(m, k),   dbias[n] = sum_m dY(m, n)
// where m runs over the forward's output rows (b, fo, to), A is the forward's K-table gather and
// dY is addressed with the forward's output map.  This covers every trained GEMM of the student:
// complex Conv2d, both polyphase halves of ComplexConvTranspose2d, the LSTM input projections
// (and, with a time-shifted segment over the hidden history, the recurrent weights W_hh) and the
// complex-LSTM Linear projections.
//
// Layout: the reduction runs over M (up to B*F*T ~ 1.3 M rows), so the grid splits M into S
// row ranges; a workgroup owns a 64(n) x 64(k) tile of one range, staging 32 rows of dY and of
// the gathered A per step in LDS and issuing v_mfma_f32_32x32x2_f32 with the ROW axis as the
// MFMA reduction axis (A operand = dY^T, B operand = A).  Range partials go to a workspace
// [S][N][Kp] and a second kernel sums them in a fixed order: deterministic, no float atomics.
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace clskd {

constexpr int WG_TN = 64;   // n per workgroup tile
constexpr int WG_TK = 64;   // k per workgroup tile
constexpr int WG_RB = 32;   // rows staged per step

struct WgradArgs {
  clskd_conv_desc d;
  const float* dy;
  float* work;      // [S][N][Kp] partial dW, then [S][N] partial dbias (if bias wanted)
  int64_t rows_per_split;
  int S;
  int want_bias;
};

template <bool VEC4>
__global__ __launch_bounds__(256) void conv_wgrad_f32(const WgradArgs a) {
  const clskd_conv_desc& d = a.d;
  __shared__ __attribute__((aligned(16))) float As[2][WG_RB][WG_TK + 4];
  __shared__ __attribute__((aligned(16))) float Ds[2][WG_RB][WG_TN + 4];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int split = blockIdx.x;
  const int n0 = blockIdx.y * WG_TN;
  const int k0 = blockIdx.z * WG_TK;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t FoTo = (int64_t)d.Fo * d.To;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  const int64_t r_end = min(M, r_begin + a.rows_per_split);
  const bool ncontig = d.oNlo == 1 && d.nlo >= d.N;

  // staging roles: row lr = tid >> 3 of the 32-row step, quads q0 = tid & 7 and q0 + 8
  const int lr = tid >> 3;
  const int q0 = tid & 7;
  const int nsub = wave & 1, ksub = wave >> 1;
  // K-table entries of this thread's two 4-k quads are loop invariant
  clskd_ktab_entry ke[2][4];
  int ks_[2][4];
#pragma unroll
  for (int qq = 0; qq < 2; ++qq)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(k0 + (q0 + 8 * qq) * 4 + j, d.K - 1);
      ke[qq][j] = d.ktab[k];
      ks_[qq][j] = d.kseg[k];
      if (k0 + (q0 + 8 * qq) * 4 + j >= d.K) ke[qq][j].dF = -32768;
    }

  // one 32-row stage into registers: gathered A (2 x 4 k) and dY (2 x 4 n) of row rs + lr
  auto load_stage = [&](int64_t rs, f32x4 (&av)[2], f32x4 (&dv)[2]) {
    const int64_t m = rs + lr;
    const bool valid = m < r_end;
    int64_t b = 0, fo = 0, to = 0;
    if (valid) {
      b = m / FoTo;
      const int64_t r = m - b * FoTo;
      fo = r / d.To;
      to = r - fo * d.To;
    }
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (valid) {
        if constexpr (VEC4) {
          const clskd_ktab_entry e = ke[qq][0];
          const clskd_seg& g = d.seg[ks_[qq][0]];
          const int64_t fi = fo * d.stride_f + e.dF, ti = to * d.stride_t + e.dT;
          if (fi >= 0 && fi < g.F && ti >= 0 && ti < g.T)
            v = *reinterpret_cast<const f32x4*>(g.ptr + b * g.sB + fo * d.stride_f * g.sF +
                                                to * d.stride_t * g.sT + e.off);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const clskd_ktab_entry e = ke[qq][j];
            const clskd_seg& g = d.seg[ks_[qq][j]];
            const int64_t fi = fo * d.stride_f + e.dF, ti = to * d.stride_t + e.dT;
            if (fi >= 0 && fi < g.F && ti >= 0 && ti < g.T)
              v[j] = g.ptr[b * g.sB + fo * d.stride_f * g.sF + to * d.stride_t * g.sT + e.off];
          }
        }
      }
      av[qq] = v;
    }
    const int64_t orow = b * d.oB + (fo * d.of_mul + d.of_add) * d.oF + to * d.oT;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int nl = (q0 + 8 * qq) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (valid) {
        if (ncontig && n0 + nl + 3 < d.N && ((orow + n0 + nl) & 3) == 0) {
          v = *reinterpret_cast<const f32x4*>(a.dy + orow + n0 + nl);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = n0 + nl + j;
            if (n < d.N) v[j] = a.dy[orow + (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo];
          }
        }
      }
      dv[qq] = v;
    }
  };

  f32x16 acc = {};
  float bacc = 0.f;  // dbias partial of column n0 + tid (tid < 64, k-tile 0 only)
  f32x4 av[2], dv[2];
  if (r_begin < r_end) load_stage(r_begin, av, dv);
  int buf = 0;
  for (int64_t rs = r_begin; rs < r_end; rs += WG_RB, buf ^= 1) {
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      *reinterpret_cast<f32x4*>(&As[buf][lr][(q0 + 8 * qq) * 4]) = av[qq];
      *reinterpret_cast<f32x4*>(&Ds[buf][lr][(q0 + 8 * qq) * 4]) = dv[qq];
    }
    __syncthreads();
    if (rs + WG_RB < r_end) load_stage(rs + WG_RB, av, dv);  // in flight under the MFMAs
    // ---- 16 MFMAs (2 rows each) per wave: C[n][k] += dY^T[n][r] A[r][k] ----
    const int cl = lane & 31, rh = lane >> 5;
#pragma unroll
    for (int s = 0; s < WG_RB / 2; ++s) {
      const float x = Ds[buf][2 * s + rh][nsub * 32 + cl];
      const float y = As[buf][2 * s + rh][ksub * 32 + cl];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc, 0, 0, 0);
    }
    if (a.want_bias && blockIdx.z == 0 && tid < WG_TN) {
#pragma unroll 8
      for (int r = 0; r < WG_RB; ++r) bacc += Ds[buf][r][tid];
    }
  }
  // ---- partial tile out: work[split][n][k] ----
  const int Kp = d.K;
  float* wp = a.work + (int64_t)split * d.N * Kp;
  const int kc = k0 + ksub * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + nsub * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (n < d.N && kc < Kp) wp[(int64_t)n * Kp + kc] = acc[r];
  }
  if (a.want_bias && blockIdx.z == 0 && tid < WG_TN && n0 + tid < d.N)
    a.work[(int64_t)a.S * d.N * Kp + (int64_t)split * d.N + n0 + tid] = bacc;
}

// dw[i] (+)= sum_s work[s][i]: 16 consecutive elements x 16 split lanes per block (a wave reads
// four 64-B runs per load); split lane sl sums splits sl, sl + 16, ... (eight loads in flight per
// round), then the 16 lane sums are added in a fixed order in LDS (deterministic for a given S).
// Round 4's 32 x 8 layout read 8 splits of one element per 8 lanes (32-B pieces) and carried a
// chain of S / 8 dependent loads: 16.8 us per launch in the C3 census.  The bias partials
// ([S][N] after the weight partials) are reduced by the blocks past the weight's wblocks in the
// same launch (round 6: one launch per weight gradient instead of two).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ work, int S,
                                                          int64_t per, float* __restrict__ dw,
                                                          int accumulate, int64_t wblocks,
                                                          int64_t nbias, float* __restrict__ dbias,
                                                          int acc_bias) {
  const int e = threadIdx.x & 15, sl = threadIdx.x >> 4;
  int64_t blk = blockIdx.x;
  if (blk >= wblocks) {  // block-uniform: the bias segment
    blk -= wblocks;
    work += (int64_t)S * per;
    per = nbias;
    dw = dbias;
    accumulate = acc_bias;
  }
  const int64_t i = blk * 16 + e;
  float s = 0.f;
  if (i < per) {
    int j = sl;
    for (; j + 7 * 16 < S; j += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = work[(int64_t)(j + 16 * u) * per + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; j < S; j += 16) s += work[(int64_t)j * per + i];
  }
  __shared__ float red[16][17];
  red[sl][e] = s;
  __syncthreads();
  if (sl == 0 && i < per) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][e];
    dw[i] = accumulate ? dw[i] + t : t;
  }
}

// ------------------------------------------------------------------------------------------
// Gradient unpack: out[i] (+)= sum_{j<J} sgn[i*J+j] * src[idx[i*J+j]]  (idx < 0: skipped).
// Maps a packed GEMM-operand gradient (e.g. [[Wr,-Wi],[Wi,Wr]] blocks, polyphase taps, padded
// K) back onto the module's parameter layout; the host derives idx/sgn once per layer from
// the packing transform.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void index_gather_kernel(const float* __restrict__ src,
                                                           const int32_t* __restrict__ idx,
                                                           const float* __restrict__ sgn, int J,
                                                           int64_t n, float* __restrict__ out,
                                                           int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < J; ++j) {
      const int32_t q = idx[i * J + j];
      if (q >= 0) s = fmaf(sgn[i * J + j], src[q], s);
    }
    out[i] = accumulate ? out[i] + s : s;
  }
}

struct GatherJobsArg {
  clskd_gather_job j[CLSKD_GATHER_JOBS_MAX];
};

// one job per blockIdx.y, grid-stride over its elements (the per-element arithmetic of
// index_gather_kernel)
__global__ __launch_bounds__(256) void index_gather_jobs_kernel(const GatherJobsArg a) {
  const clskd_gather_job& jb = a.j[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < jb.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < jb.J; ++j) {
      const int32_t q = jb.idx[i * jb.J + j];
      if (q >= 0) s = fmaf(jb.sgn[i * jb.J + j], jb.src[q], s);
    }
    jb.out[i] = jb.accumulate ? jb.out[i] + s : s;
  }
}

// ------------------------------------------------------------------------------------------
// Adam (torch.optim.Adam semantics, distill.py:202-204): L2 weight decay folded into g,
// bias corrections from the step count, eps added to sqrt(v)/sqrt(bc2).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr, float beta1, float beta2,
                                                   float eps, float wd, float bc1, float bc2s,
                                                   float gscale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    const float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] = pi - (lr / bc1) * (mi / denom);
  }
}

// The same update with the step count on the device (a captured training step replays it): every
// thread derives the bias corrections of step *step + 1; step_advance_kernel then stores it.
__global__ __launch_bounds__(256) void adam_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       int64_t n, float lr, float beta1, float beta2,
                                                       float eps, float wd, const int32_t* __restrict__ step,
                                                       float gscale) {
  const float t = (float)(*step + 1);
  const float bc1 = 1.f - powf(beta1, t);
  const float bc2s = sqrtf(1.f - powf(beta2, t));
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    const float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] = pi - (lr / bc1) * (mi / denom);
  }
}

__global__ void step_advance_kernel(int32_t* step) {
  if (threadIdx.x == 0) *step += 1;
}

__global__ void fill_f32_kernel(float* p, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// y (+)= alpha * x
__global__ void axpy_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                float alpha, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = accumulate ? fmaf(alpha, x[i], y[i]) : alpha * x[i];
}

inline unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>(cdiv(n, 256), 8192); }

// splits of the row axis: about CLSKD_WGRAD_WG workgroups (default 4096), at least 256 rows
// per split.  The [S][N][K] partials are written once and re-read by wgrad_reduce_kernel, so
// S trades occupancy against partial traffic.
inline int wgrad_target() {
  const int v = knob(KNOB_WGRAD_WG);
  return v >= 64 ? v : 4096;
}
inline void wgrad_plan(const clskd_conv_desc& d, int& S, int64_t& rps) {
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t tiles = cdiv(d.N, WG_TN) * cdiv(d.K, WG_TK);
  int64_t s = cdiv(wgrad_target(), tiles);
  s = std::max<int64_t>(1, std::min<int64_t>({s, (int64_t)1024, cdiv(M, 256)}));
  rps = cdiv(cdiv(M, s), WG_RB) * WG_RB;
  S = (int)cdiv(M, rps);
}

// wgrad_x3.hip: the split-product engine for CLSKD_F32X3 descriptors (same partial layout)
bool wgrad_x3_takes(const clskd_conv_desc& d);
void wgrad_x3_plan(const clskd_conv_desc& d, int& S, int64_t& rps);
void launch_wgrad_x3(const clskd_conv_desc& d, const float* dy, float* work, int S, int64_t rps,
                     int want_bias, hipStream_t st);

}  // namespace clskd

using namespace clskd;

extern "C" int64_t clskd_conv2d_wgrad_workspace(const clskd_conv_desc* dp) {
  if (!dp) return -1;
  int S;
  int64_t rps;
  if (wgrad_x3_takes(*dp))
    wgrad_x3_plan(*dp, S, rps);
  else
    wgrad_plan(*dp, S, rps);
  return (int64_t)S * dp->N * dp->K + (int64_t)S * dp->N;
}

extern "C" int clskd_conv2d_wgrad(const clskd_conv_desc* dp, const float* dy, float* dw,
                                  float* dbias, float* work, int64_t work_elems,
                                  int32_t accumulate, void* stream) {
  CLSKD_CHECK_ARG(dp && dy && dw && work, "conv2d_wgrad: null pointer");
  const clskd_conv_desc& d = *dp;
  CLSKD_CHECK_SHAPE(d.B > 0 && d.Fo > 0 && d.To > 0 && d.N > 0 && d.K > 0, "conv2d_wgrad: empty shape");
  CLSKD_CHECK_ARG(d.in_dtype == CLSKD_F32, "conv2d_wgrad: fp32 segments only");
  CLSKD_CHECK_SHAPE(d.nseg >= 1 && d.nseg <= CLSKD_MAX_SEGS && d.K % 4 == 0, "conv2d_wgrad: nseg/K");
  int S;
  int64_t rps;
  const bool x3 = wgrad_x3_takes(d);
  if (x3)
    wgrad_x3_plan(d, S, rps);
  else
    wgrad_plan(d, S, rps);
  const int64_t need = (int64_t)S * d.N * d.K + (int64_t)S * d.N;
  CLSKD_CHECK_SHAPE(work_elems >= need, "conv2d_wgrad: workspace %lld < %lld", (long long)work_elems,
                    (long long)need);
  if (d.vec4) {
    for (int s = 0; s < d.nseg; ++s)
      CLSKD_CHECK_ARG(((uintptr_t)d.seg[s].ptr & 15) == 0 && d.seg[s].sB % 4 == 0 &&
                          d.seg[s].sF % 4 == 0 && d.seg[s].sT % 4 == 0,
                      "conv2d_wgrad: vec4 segment %d not 16-byte aligned", s);
  }
  hipStream_t st = as_stream(stream);
  if (x3) {
    launch_wgrad_x3(d, dy, work, S, rps, dbias ? 1 : 0, st);
  } else {
    WgradArgs a{d, dy, work, rps, S, dbias ? 1 : 0};
    dim3 grid(S, (unsigned)cdiv(d.N, WG_TN), (unsigned)cdiv(d.K, WG_TK));
    if (d.vec4)
      hipLaunchKernelGGL((conv_wgrad_f32<true>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv_wgrad_f32<false>), grid, dim3(256), 0, st, a);
  }
  CLSKD_LAUNCH_CHECK("conv2d_wgrad");
  const int64_t per = (int64_t)d.N * d.K;
  const int64_t wblocks = cdiv(per, 16), bblocks = dbias ? cdiv((int64_t)d.N, 16) : 0;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(wblocks + bblocks)), dim3(256), 0, st,
                     work, S, per, dw, accumulate & 1, wblocks, (int64_t)d.N, dbias,
                     (accumulate >> 1) & 1);
  CLSKD_LAUNCH_CHECK("conv2d_wgrad_reduce");
  return CLSKD_OK;
}

extern "C" int clskd_index_gather(const float* src, const int32_t* idx, const float* sgn, int32_t J,
                                  int64_t n, float* out, int32_t accumulate, void* stream) {
  CLSKD_CHECK_ARG(src && idx && sgn && out && J >= 1, "index_gather: bad argument");
  if (n <= 0) return CLSKD_OK;
  hipLaunchKernelGGL(index_gather_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), src,
                     idx, sgn, J, n, out, accumulate);
  CLSKD_LAUNCH_CHECK("index_gather");
  return CLSKD_OK;
}

extern "C" int clskd_index_gather_jobs(const clskd_gather_job* jobs, int32_t n_jobs, void* stream) {
  CLSKD_CHECK_ARG(jobs && n_jobs >= 0 && n_jobs <= CLSKD_GATHER_JOBS_MAX,
                  "index_gather_jobs: %d jobs (at most %d)", n_jobs, CLSKD_GATHER_JOBS_MAX);
  if (n_jobs == 0) return CLSKD_OK;
  GatherJobsArg a{};
  int64_t nmax = 0;
  for (int i = 0; i < n_jobs; ++i) {
    const clskd_gather_job& jb = jobs[i];
    CLSKD_CHECK_ARG(jb.src && jb.idx && jb.sgn && jb.out && jb.J >= 1 && jb.n >= 0,
                    "index_gather_jobs: bad job %d", i);
    a.j[i] = jb;
    nmax = std::max<int64_t>(nmax, jb.n);
  }
  if (nmax == 0) return CLSKD_OK;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(nmax, 256), 512);
  hipLaunchKernelGGL(index_gather_jobs_kernel, dim3(gx, (unsigned)n_jobs), dim3(256), 0,
                     as_stream(stream), a);
  CLSKD_LAUNCH_CHECK("index_gather_jobs");
  return CLSKD_OK;
}

extern "C" int clskd_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                               float beta1, float beta2, float eps, float weight_decay,
                               int32_t step, float grad_scale, void* stream) {
  CLSKD_CHECK_ARG(p && g && m && v && step >= 1, "adam: bad argument");
  if (n <= 0) return CLSKD_OK;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)step));
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, g, m, v,
                     n, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, grad_scale);
  CLSKD_LAUNCH_CHECK("adam");
  return CLSKD_OK;
}

extern "C" int clskd_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                                   float beta1, float beta2, float eps, float weight_decay,
                                   int32_t* step, float grad_scale, void* stream) {
  CLSKD_CHECK_ARG(p && g && m && v && step, "adam_dev: bad argument");
  hipStream_t st = as_stream(stream);
  if (n > 0)
    hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, m, v, n, lr, beta1,
                       beta2, eps, weight_decay, step, grad_scale);
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, st, step);
  CLSKD_LAUNCH_CHECK("adam_dev");
  return CLSKD_OK;
}

extern "C" int clskd_fill_f32(float* p, int64_t n, float value, void* stream) {
  CLSKD_CHECK_ARG(p || n == 0, "fill: null pointer");
  if (n <= 0) return CLSKD_OK;
  hipLaunchKernelGGL(fill_f32_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, n, value);
  CLSKD_LAUNCH_CHECK("fill_f32");
  return CLSKD_OK;
}

extern "C" int clskd_axpy_f32(const float* x, float* y, int64_t n, float alpha, int32_t accumulate,
                              void* stream) {
  CLSKD_CHECK_ARG((x && y) || n == 0, "axpy: null pointer");
  if (n <= 0) return CLSKD_OK;
  hipLaunchKernelGGL(axpy_f32_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, y, n,
                     alpha, accumulate);
  CLSKD_LAUNCH_CHECK("axpy_f32");
  return CLSKD_OK;
}

// ------------------------------------------------------------------------------------------
// Split-product data gradients on the bf16 engines (include/clskd.h, clskd_split_planes /
// clskd_pack_split3).  x = hi + lo + r with hi = bf16_rne(x), lo = bf16_rne(x - hi) (x - hi exact
// in fp32), |r| <= 2^-18 |x| — the split of the CLSKD_F32X3 engines (conv_split.hip), here
// materialised once so the LDS-DMA bf16 engine stages it like any bf16 map.
// ------------------------------------------------------------------------------------------
namespace clskd {

__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ src,
                                                           int64_t rows, int C,
                                                           __bf16* __restrict__ dst) {
  const int CQ = C / 4;
  const int64_t nq = rows * CQ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = q / CQ;
    const int c = (int)(q - r * CQ) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(src + r * C + c);
    bf16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hi[j] = (__bf16)v[j];
      lo[j] = (__bf16)(v[j] - (float)hi[j]);
    }
    *reinterpret_cast<bf16x4*>(dst + r * 2 * C + c) = hi;
    *reinterpret_cast<bf16x4*>(dst + r * 2 * C + C + c) = lo;
  }
}

// out[n][t*3C + s*C + c] = {hi, hi, lo}[s] of w[n][t*C + c]; zero for k >= ntaps*3C
__global__ __launch_bounds__(256) void pack_split3_kernel(const float* __restrict__ w, int N,
                                                          int ldw, int ntaps, int C, int Kp,
                                                          __bf16* __restrict__ out) {
  const int64_t total = (int64_t)N * Kp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / Kp);
    const int k = (int)(i - (int64_t)n * Kp);
    float v = 0.f;
    int part = 0;
    if (k < ntaps * 3 * C) {
      const int t = k / (3 * C);
      const int r = k - t * 3 * C;
      part = r / C;
      v = w[(int64_t)n * ldw + t * C + (r - part * C)];
    }
    const __bf16 hi = (__bf16)v;
    out[i] = part == 2 ? (__bf16)(v - (float)hi) : hi;
  }
}

}  // namespace clskd

extern "C" int clskd_split_planes(const float* src, int64_t rows, int32_t C, void* dst,
                                  void* stream) {
  CLSKD_CHECK_ARG(src && dst, "split_planes: null pointer");
  CLSKD_CHECK_SHAPE(rows >= 0 && C > 0 && C % 4 == 0, "split_planes: C=%d must be a multiple of 4", C);
  CLSKD_CHECK_ARG(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 7) == 0,
                  "split_planes: src 16-B / dst 8-B alignment");
  const int64_t nq = rows * (C / 4);
  if (nq == 0) return CLSKD_OK;
  hipLaunchKernelGGL(clskd::split_planes_kernel, dim3(clskd::grid_for(nq)), dim3(256), 0,
                     clskd::as_stream(stream), src, rows, C, reinterpret_cast<__bf16*>(dst));
  CLSKD_LAUNCH_CHECK("split_planes");
  return CLSKD_OK;
}

extern "C" int clskd_pack_split3(const float* w, int32_t N, int32_t ldw, int32_t ntaps, int32_t C,
                                 int32_t Kp, void* out, void* stream) {
  CLSKD_CHECK_ARG(w && out, "pack_split3: null pointer");
  CLSKD_CHECK_SHAPE(N > 0 && ntaps > 0 && C > 0 && ldw >= ntaps * C && Kp >= ntaps * 3 * C &&
                        Kp % 64 == 0,
                    "pack_split3: N=%d ldw=%d ntaps=%d C=%d Kp=%d", N, ldw, ntaps, C, Kp);
  const int64_t total = (int64_t)N * Kp;
  hipLaunchKernelGGL(clskd::pack_split3_kernel, dim3(clskd::grid_for(total)), dim3(256), 0,
                     clskd::as_stream(stream), w, N, ldw, ntaps, C, Kp,
                     reinterpret_cast<__bf16*>(out));
  CLSKD_LAUNCH_CHECK("pack_split3");
  return CLSKD_OK;
}
