// Backward of the elementwise / normalisation ops of the CLSKD step (student side):
// BatchNorm2d(train) + PReLU, ReviewKD ABF attention fusion and nearest upsampling, masking
// mode 'E', ConviSTFT overlap-add + clamp, framing pads, the STFT log-magnitude L1 loss and the
// complex-LSTM output combine.  HBM-bound passes; statistics reductions in fp64 with fixed
// orders (no float atomics), so every gradient is bitwise repeatable.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace clskd {

typedef __bf16 bf16x4b __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ f32x4 ld4(const T* p);
template <>
__device__ __forceinline__ f32x4 ld4<float>(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}
template <>
__device__ __forceinline__ f32x4 ld4<__bf16>(const __bf16* p) {
  const bf16x4b v = *reinterpret_cast<const bf16x4b*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

// 4 channels as their raw storage vector (loaded without conversion) and its fp32 widening
template <typename T> struct Raw4;
template <> struct Raw4<float> {
  typedef f32x4 V;
  static __device__ __forceinline__ V ld(const float* p) { return *reinterpret_cast<const V*>(p); }
  static __device__ __forceinline__ f32x4 cvt(V v) { return v; }
};
template <> struct Raw4<__bf16> {
  typedef bf16x4b V;
  static __device__ __forceinline__ V ld(const __bf16* p) { return *reinterpret_cast<const V*>(p); }
  static __device__ __forceinline__ f32x4 cvt(V v) {
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
};

// ------------------------------------------------------------------------------------------
// BatchNorm (train) + optional PReLU backward.  Forward: y_bn = x*scale + shift (scale = gamma *
// rstd, shift = beta - mean*scale), y = prelu(y_bn) when alpha != NULL.  Given dy = dL/dy:
//   dz = alpha ? (y_bn > 0 ? dy : alpha*dy) : dy      (torch prelu backward)
//   dbeta = sum dz, dgamma = sum dz*xhat, dalpha = sum_{y_bn<=0} y_bn*dy
//   dx = k1*dz + k2*x + k3   with k1 = gamma*rstd, k2 = -gamma*rstd^2*dgamma/n,
//                              k3 = -gamma*rstd*dbeta/n + gamma*rstd^2*mean*dgamma/n
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const T* __restrict__ x, const float* __restrict__ dy, int64_t rows, int C, int64_t rpb,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ mean, const float* __restrict__ var, float eps,
    const float* __restrict__ alpha, double* __restrict__ partial) {
  const int CG = C >> 2;
  const int RP = 256 / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG;
  const int rl = tid / CG;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(rows, r0 + rpb);
  const float al = alpha ? alpha[0] : 1.f;
  f32x4 sc, sh, mu, rs;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = (cg * 4 + j) % C;
    sc[j] = scale[c];
    sh[j] = shift[c];
    mu[j] = mean[c];
    rs[j] = (float)(1.0 / sqrt((double)var[c] + (double)eps));
  }
  double sb[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0}, sa[4] = {0, 0, 0, 0};
  if (rl < RP) {
    for (int64_t r = r0 + rl; r < r1; r += RP) {
      const f32x4 xv = ld4<T>(x + r * C + cg * 4);
      const f32x4 gv = *reinterpret_cast<const f32x4*>(dy + r * C + cg * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float yb = fmaf(xv[j], sc[j], sh[j]);
        float dz = gv[j];
        if (alpha) {
          if (!(yb > 0.f)) {
            sa[j] += (double)yb * (double)gv[j];
            dz = al * gv[j];
          }
        }
        const float xh = (xv[j] - mu[j]) * rs[j];
        sb[j] += (double)dz;
        sg[j] += (double)dz * (double)xh;
      }
    }
  }
  __shared__ double red[256][13];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[tid][j] = sb[j];
    red[tid][4 + j] = sg[j];
    red[tid][8 + j] = sa[j];
  }
  __syncthreads();
  if (tid < CG) {
    double B[4] = {0, 0, 0, 0}, G[4] = {0, 0, 0, 0}, A[4] = {0, 0, 0, 0};
    for (int l = 0; l < RP; ++l) {
      const int t = l * CG + tid;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        B[j] += red[t][j];
        G[j] += red[t][4 + j];
        A[j] += red[t][8 + j];
      }
    }
    double* p = partial + ((int64_t)blockIdx.x * C + tid * 4) * 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[3 * j] = B[j];
      p[3 * j + 1] = G[j];
      p[3 * j + 2] = A[j];
    }
  }
}

// one block per channel; writes dgamma/dbeta (accumulate optional), k[3][C], alpha_part[C]
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    const double* __restrict__ partial, int nblk, int64_t rows, int C, const float* gamma,
    const float* mean, const float* var, float eps, float* dgamma, float* dbeta, float* k,
    double* alpha_part, int accumulate) {
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  // eight independent accumulators: eight strided partial rows in flight per thread (the loop
  // was one L2 round trip per 256 rows — latency-bound at nblk ~ 16k); fixed combine order
  double sb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sg[8] = {0, 0, 0, 0, 0, 0, 0, 0},
         sa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int b = tid;
  for (; b + 7 * 256 < nblk; b += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double* p = partial + ((int64_t)(b + u * 256) * C + c) * 3;
      sb[u] += p[0];
      sg[u] += p[1];
      sa[u] += p[2];
    }
  }
  for (; b < nblk; b += 256) {
    const double* p = partial + ((int64_t)b * C + c) * 3;
    sb[0] += p[0];
    sg[0] += p[1];
    sa[0] += p[2];
  }
  double SB = ((sb[0] + sb[1]) + (sb[2] + sb[3])) + ((sb[4] + sb[5]) + (sb[6] + sb[7]));
  double SG = ((sg[0] + sg[1]) + (sg[2] + sg[3])) + ((sg[4] + sg[5]) + (sg[6] + sg[7]));
  const double SA = ((sa[0] + sa[1]) + (sa[2] + sa[3])) + ((sa[4] + sa[5]) + (sa[6] + sa[7]));
  __shared__ double r0[256], r1[256], r2[256];
  r0[tid] = SB;
  r1[tid] = SG;
  r2[tid] = SA;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      r0[tid] += r0[tid + o];
      r1[tid] += r1[tid + o];
      r2[tid] += r2[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    SB = r0[0];
    SG = r1[0];
    const double n = (double)rows;
    const double rs = 1.0 / sqrt((double)var[c] + (double)eps);
    const double g = gamma ? (double)gamma[c] : 1.0;
    k[c] = (float)(g * rs);
    k[C + c] = (float)(-g * rs * rs * SG / n);
    k[2 * C + c] = (float)(-g * rs * SB / n + g * rs * rs * (double)mean[c] * SG / n);
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)SG : (float)SG;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)SB : (float)SB;
    if (alpha_part) alpha_part[c] = r2[0];
  }
}

// dalpha (+)= sum over channels of alpha_part (fixed order)
__global__ void bn_bwd_alpha_kernel(const double* alpha_part, int C, float* dalpha, int accumulate) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0;
    for (int c = 0; c < C; ++c) s += alpha_part[c];
    dalpha[0] = accumulate ? dalpha[0] + (float)s : (float)s;
  }
}

template <typename T, typename GT = float>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const T* __restrict__ x, const GT* __restrict__ dy, int64_t rows, int C,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ alpha, const float* __restrict__ k, float* __restrict__ dx,
    int accumulate) {
  const int64_t nq = rows * C / 4;
  const float al = alpha ? alpha[0] : 1.f;
  // channel of the thread's first quad, then advanced by the grid stride (mod C): no 64-bit
  // modulo per quad; the per-channel vectors are 16-B loads (C % 4 == 0, 16-B aligned: host)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cstep = (int)((stride * 4) % C);
  int c0 = (int)((q0 * 4) % C);
  for (int64_t q = q0; q < nq; q += stride) {
    const f32x4 xv = ld4<T>(x + q * 4);
    const f32x4 gv = load4<GT>(dy + q * 4);
    const f32x4 k0 = *reinterpret_cast<const f32x4*>(k + c0);
    const f32x4 k1 = *reinterpret_cast<const f32x4*>(k + C + c0);
    const f32x4 k2 = *reinterpret_cast<const f32x4*>(k + 2 * C + c0);
    f32x4 dz = gv;
    if (alpha) {
      const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c0);
      const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (!(fmaf(xv[j], sc[j], sh[j]) > 0.f)) dz[j] = al * gv[j];
    }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf(k0[j], dz[j], fmaf(k1[j], xv[j], k2[j]));
    c0 += cstep;
    if (c0 >= C) c0 -= C;
    if (accumulate) o += *reinterpret_cast<const f32x4*>(dx + q * 4);
    *reinterpret_cast<f32x4*>(dx + q * 4) = o;
  }
}

// ------------------------------------------------------------------------------------------
// ABF fusion backward (framework.py:209-219), mid = 64.  Forward (abf_fuse_kernel): x = x1*xs +
// xh, y = res[nearest(f), nearest(t)], z_k = sigmoid(w_k . [x; y] + b_k), out = x*z0 + y*z1.
// Given dout: dx = dout*z0 + a0*w0x + a1*w1x, dy = dout*z1 + a0*w0y + a1*w1y with
// a_k = (sum_c dout_c * {x,y}_c) * z_k (1 - z_k).  dx is w.r.t. the BN1 output x; dy is w.r.t.
// the UPSAMPLED residual (reduce with clskd_nearest_down_sum).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int nearest_src_b(int dst, int in_size, int out_size) {
  if (out_size == in_size) return dst;
  if (out_size == 2 * in_size) return dst >> 1;
  const float scale = (float)in_size / (float)out_size;
  const int s = (int)floorf((float)dst * scale);
  return s < in_size - 1 ? s : in_size - 1;
}

// smallest dst with nearest_src(dst) >= s (nearest_src is non-decreasing in dst)
__device__ __forceinline__ int first_dst_b(int s, int in_size, int out_size) {
  if (out_size == in_size) return s;           // the nearest_src_b fast paths, inverted
  if (out_size == 2 * in_size) return 2 * s;
  int d0 = (int)((double)s * out_size / in_size) - 2;
  if (d0 < 0) d0 = 0;
  while (d0 < out_size && nearest_src_b(d0, in_size, out_size) < s) ++d0;
  return d0;
}

// Fused ReviewKD mid-channel backward: dout = d(conv2 input) of this level plus, when dnext is
// given, the NEXT level's gradient w.r.t. its upsampled residual folded back onto this grid
// (nearest upsampling (F, T) -> (F2, T2), framework.py:213-215) — so no separate down-sum pass;
// when bnpart is given, per-block fp64 partials {sum dx, sum dx*xhat1, 0} of the conv1 BatchNorm
// backward (xhat1 = (x1 - mean1) * rstd1) are emitted — so no separate BN reduce pass.
// GT: storage type of the four gradient maps (dout, dnext, dx, dyup): fp32, or bf16 in the
// mixed-precision step (halves the pass's dominant bytes; arithmetic stays fp32).
template <typename DT, typename GT>
__global__ __launch_bounds__(256) void abf_fuse_bwd_kernel(
    const DT* __restrict__ x1, const DT* __restrict__ res, int B, int F, int T, int Fr, int Tr,
    const float* __restrict__ w, const float* __restrict__ bias, const float* __restrict__ xs,
    const float* __restrict__ xh, const GT* __restrict__ dout, GT* __restrict__ dx,
    GT* __restrict__ dyup, const GT* __restrict__ dnext, int F2, int T2,
    const float* __restrict__ mean1, const float* __restrict__ var1, float eps,
    double* __restrict__ bnpart) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & 15;
  const int c = sub * 4;
  f32x4 mu = {0.f, 0.f, 0.f, 0.f}, rs = {0.f, 0.f, 0.f, 0.f};
  if (bnpart) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = mean1[c + j];
      rs[j] = (float)(1.0 / sqrt((double)var1[c + j] + (double)eps));
    }
  }
  double sb[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0};
  f32x4 sx = {1.f, 1.f, 1.f, 1.f}, hx = {0.f, 0.f, 0.f, 0.f};
  if (xs) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sx[j] = xs[c + j];
      hx[j] = xh[c + j];
    }
  }
  f32x4 w0x, w0y, w1x, w1y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w0x[j] = w[c + j];
    w0y[j] = w[64 + c + j];
    w1x[j] = w[128 + c + j];
    w1y[j] = w[192 + c + j];
  }
  const float b0 = bias[0], b1 = bias[1];
  // next grid an exact 1x / 2x upsampling in each axis (nearest_src_b's fast paths): the children
  // of (f, t) are {rf*f, rf*f + 1} x {rt*t, rt*t + 1}, no search loop (rf = 0: general grids)
  int rf = 0, rt = 0;
  if (dnext && (F2 == F || F2 == 2 * F) && (T2 == T || T2 == 2 * T)) {
    rf = F2 / F;
    rt = T2 / T;
  }
  const int64_t npix = (int64_t)B * F * T;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int64_t nslots = ((int64_t)gridDim.x * blockDim.x) >> 4;
  // a pixel's operands as loaded (raw vectors) and its grid coordinates
  struct Px {
    typename Raw4<DT>::V xr, yr;
    typename Raw4<GT>::V gr, c00, c01, c10, c11;
    int b, f, t;
  };
  auto load_px = [&](int64_t p, Px& o) {
    // 32-bit index split (npix < 2^31, checked by the host): no 64-bit division per pixel
    const uint32_t p32 = (uint32_t)p, bf = p32 / (uint32_t)T;
    o.t = (int)(p32 - bf * (uint32_t)T);
    o.b = (int)(bf / (uint32_t)F);
    o.f = (int)(bf - (uint32_t)o.b * (uint32_t)F);
    const int fr = nearest_src_b(o.f, Fr, F);
    const int tr = nearest_src_b(o.t, Tr, T);
    const GT* gp = dout + p * 64 + c;
    const GT* q = gp;  // children of a 1x / 2x next grid (rf = 0: dout again, unused)
    int64_t df = 0, dt = 0;
    if (rf) {
      q = dnext + ((((int64_t)o.b * F2 + o.f * rf) * T2 + o.t * rt) * 64) + c;
      df = rf == 2 ? (int64_t)T2 * 64 : 0;
      dt = rt == 2 ? 64 : 0;
    }
    o.xr = Raw4<DT>::ld(x1 + p * 64 + c);
    o.yr = Raw4<DT>::ld(res + (((int64_t)o.b * Fr + fr) * Tr + tr) * 64 + c);
    o.gr = Raw4<GT>::ld(gp);
    o.c00 = Raw4<GT>::ld(q);
    o.c01 = Raw4<GT>::ld(q + dt);
    o.c10 = Raw4<GT>::ld(q + df);
    o.c11 = Raw4<GT>::ld(q + df + dt);
  };
  auto compute_px = [&](int64_t p, const Px& o) {
    const f32x4 xraw = Raw4<DT>::cvt(o.xr);
    f32x4 xv;
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = fmaf(xraw[j], sx[j], hx[j]);
    const f32x4 yv = Raw4<DT>::cvt(o.yr);
    f32x4 g = Raw4<GT>::cvt(o.gr);
    if (rf) {  // summed in the general loop's order: (f2, t2), (f2, t2+1), (f2+1, t2), ...
      g += Raw4<GT>::cvt(o.c00);
      if (rt == 2) g += Raw4<GT>::cvt(o.c01);
      if (rf == 2) {
        g += Raw4<GT>::cvt(o.c10);
        if (rt == 2) g += Raw4<GT>::cvt(o.c11);
      }
    } else if (dnext) {  // children of (f, t) on the next level's grid
      const int fa = first_dst_b(o.f, F, F2), ta = first_dst_b(o.t, T, T2);
      for (int f2 = fa; f2 < F2 && nearest_src_b(f2, F, F2) == o.f; ++f2)
        for (int t2 = ta; t2 < T2 && nearest_src_b(t2, T, T2) == o.t; ++t2)
          g += load4<GT>(dnext + ((((int64_t)o.b * F2 + f2) * T2 + t2) * 64) + c);
    }
    float d0 = 0.f, d1 = 0.f, e0 = 0.f, e1 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d0 += w0x[j] * xv[j] + w0y[j] * yv[j];
      d1 += w1x[j] * xv[j] + w1y[j] * yv[j];
      e0 += g[j] * xv[j];
      e1 += g[j] * yv[j];
    }
#pragma unroll
    for (int sh = 8; sh > 0; sh >>= 1) {
      d0 += __shfl_xor(d0, sh, 16);
      d1 += __shfl_xor(d1, sh, 16);
      e0 += __shfl_xor(e0, sh, 16);
      e1 += __shfl_xor(e1, sh, 16);
    }
    const float z0 = sigmoidf_(d0 + b0);
    const float z1 = sigmoidf_(d1 + b1);
    const float a0 = e0 * z0 * (1.f - z0);
    const float a1 = e1 * z1 * (1.f - z1);
    f32x4 ox, oy;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ox[j] = g[j] * z0 + a0 * w0x[j] + a1 * w1x[j];
      oy[j] = g[j] * z1 + a0 * w0y[j] + a1 * w1y[j];
    }
    if constexpr (sizeof(GT) == 2) {
      // the BN partials sum the stored (rounded) dx, so the apply pass that reads it back sees
      // statistics consistent with its own input
#pragma unroll
      for (int j = 0; j < 4; ++j) ox[j] = (float)(GT)ox[j];
    }
    store4<GT>(dx + p * 64 + c, ox);
    if (dyup) store4<GT>(dyup + p * 64 + c, oy);
    if (bnpart) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sb[j] += (double)ox[j];
        sg[j] += (double)ox[j] * (double)((xraw[j] - mu[j]) * rs[j]);
      }
    }
  };
  // two pixels per iteration (p, p + nslots: the same per-thread order as one at a time, so the
  // partials are bitwise unchanged): their 14 loads issued together, pinned ahead of the uniform
  // branches (the compiler would sink each child load into its branch behind a vmcnt(0))
  for (int64_t p = gw; p < npix; p += 2 * nslots) {
    const int64_t p2 = p + nslots;
    const bool two = p2 < npix;
    Px A, Bq;
    load_px(p, A);
    load_px(two ? p2 : p, Bq);
    asm volatile("" : "+v"(A.xr), "+v"(A.yr), "+v"(A.gr), "+v"(A.c00), "+v"(A.c01), "+v"(A.c10),
                 "+v"(A.c11), "+v"(Bq.xr), "+v"(Bq.yr), "+v"(Bq.gr), "+v"(Bq.c00), "+v"(Bq.c01),
                 "+v"(Bq.c10), "+v"(Bq.c11));
    compute_px(p, A);
    if (two) compute_px(p2, Bq);
  }
  if (bnpart) {  // the block's 16 pixel slots share the channel mapping: fixed-order slot sum
    __shared__ double red[16][64][2];
    const int slot = threadIdx.x >> 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[slot][c + j][0] = sb[j];
      red[slot][c + j][1] = sg[j];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      double S = 0.0, G = 0.0;
      for (int s2 = 0; s2 < 16; ++s2) {
        S += red[s2][threadIdx.x][0];
        G += red[s2][threadIdx.x][1];
      }
      double* q = bnpart + ((int64_t)blockIdx.x * 64 + threadIdx.x) * 3;
      q[0] = S;
      q[1] = G;
      q[2] = 0.0;
    }
  }
}

// out[b][fr][tr][c] (+)= sum of g[b][f][t][c] over the (f, t) whose nearest source is (fr, tr)
__device__ __forceinline__ int first_dst(int s, int in_size, int out_size) {
  // smallest dst with nearest_src(dst) >= s (nearest_src is non-decreasing in dst)
  int d0 = (int)((double)s * out_size / in_size) - 2;
  if (d0 < 0) d0 = 0;
  while (d0 < out_size && nearest_src_b(d0, in_size, out_size) < s) ++d0;
  return d0;
}

template <typename GT>
__global__ __launch_bounds__(256) void nearest_down_sum_kernel(
    const GT* __restrict__ g, int B, int F, int T, int Fr, int Tr, int C,
    float* __restrict__ out, int accumulate) {
  const int CQ = C / 4;
  const int64_t total = (int64_t)B * Fr * Tr * CQ;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cq = (int)(i % CQ);
    const int64_t pix = i / CQ;
    const int tr = (int)(pix % Tr);
    const int64_t bf = pix / Tr;
    const int fr = (int)(bf % Fr);
    const int b = (int)(bf / Fr);
    const int fa = first_dst(fr, Fr, F), ta = first_dst(tr, Tr, T);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int f = fa; f < F && nearest_src_b(f, Fr, F) == fr; ++f)
      for (int t = ta; t < T && nearest_src_b(t, Tr, T) == tr; ++t)
        s += load4<GT>(g + ((((int64_t)b * F + f) * T + t) * C) + cq * 4);
    float* op = out + pix * C + cq * 4;
    if (accumulate) s += *reinterpret_cast<const f32x4*>(op);
    *reinterpret_cast<f32x4*>(op) = s;
  }
}

// ------------------------------------------------------------------------------------------
// masking mode 'E' backward (DCCRN.py:207-226): d est (real at 0.., imag at 257..) -> d mask,
// mask = last decoder output [B][256][Tm][2] read at time t+1 (time 0 gets no gradient).
// A = tanh|M| * |S|, psi = angle(S) + atan2(mi, mr):
//   dA = dre cos psi + dim sin psi,  dpsi = A (dim cos psi - dre sin psi)
//   dmr = dA |S| (1 - tanh^2|M|) mr/|M| - dpsi mi/|M|^2,  dmi = ... mi/|M| + dpsi mr/|M|^2
// (the atan2 of the 1/(|M|+1e-8)-scaled pair is scale invariant, so its derivative is atan2's).
// ------------------------------------------------------------------------------------------
// The block tiling of mask_e_kernel (norm.hip): MASK_TT frames per block, the mask columns staged
// in LDS and the mask gradient written back through the same tile in 128-B runs per bin; block 0
// of each utterance writes the zero columns (tm = 0 and tm > T).  Round 6: the thread-per-column
// form read the spectrum and its gradient with a 2-KB stride (PMC 380 MB read per launch at C3's
// shape against ~40 MB algorithmic).
__global__ __launch_bounds__(256) void mask_e_bwd_kernel(const float* __restrict__ spec, int ldspec,
                                                         const float* __restrict__ mask, int Tm,
                                                         int B, int T,
                                                         const float* __restrict__ dest, int ldest,
                                                         float* __restrict__ dmask) {
  __shared__ __attribute__((aligned(16))) float ml[256 * MASK_LD];
  const int b = blockIdx.y, t0 = blockIdx.x * MASK_TT;
  const int nt = min(MASK_TT, T - t0);
  const int64_t col0 = ((int64_t)b * 256 * Tm + t0 + 1) * 2;
  mask_tile_load(mask + col0, Tm, nt, ml);
  __syncthreads();
  for (int i = threadIdx.x; i < nt * 256; i += 256) {
    const int tt = i >> 8, fm = i & 255;
    const int f = fm + 1;
    const int64_t bt = (int64_t)b * T + t0 + tt;
    const float re = spec[bt * ldspec + f];
    const float im = spec[bt * ldspec + 257 + f];
    const float mags = sqrtf(re * re + im * im + 1e-8f);
    const float phase = atan2f(im, re);
    float* mp = ml + fm * MASK_LD + 2 * tt;  // read, then overwritten by this thread only
    const float mr = mp[0], mi = mp[1];
    const float m2 = mr * mr + mi * mi;
    const float mm = sqrtf(m2);
    const float rp = mr / (mm + 1e-8f);
    const float ip = mi / (mm + 1e-8f);
    const float th = tanhf(mm);
    const float A = th * mags;
    const float psi = phase + atan2f(ip, rp);
    const float cp = cosf(psi), sp = sinf(psi);
    const float dre = dest[bt * ldest + f], dim = dest[bt * ldest + 257 + f];
    const float dA = dre * cp + dim * sp;
    const float dpsi = A * (dim * cp - dre * sp);
    float gr = 0.f, gi = 0.f;
    if (mm > 0.f) {
      const float dmm = dA * mags * (1.f - th * th);
      gr = dmm * mr / mm - dpsi * mi / m2;
      gi = dmm * mi / mm + dpsi * mr / m2;
    }
    mp[0] = gr;
    mp[1] = gi;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256 * 2 * MASK_TT; i += 256) {
    const int fm = i / (2 * MASK_TT), r = i - fm * 2 * MASK_TT;
    if (r < 2 * nt) dmask[col0 + (int64_t)fm * Tm * 2 + r] = ml[fm * MASK_LD + r];
  }
  if (blockIdx.x == 0) {  // columns without a gradient: tm = 0 and T < tm < Tm
    const int nz = Tm - T;
    for (int i = threadIdx.x; i < 256 * nz; i += 256) {
      const int fm = i / nz, j = i - fm * nz;
      const int tm = j == 0 ? 0 : T + j;
      float* dp = dmask + (((int64_t)b * 256 + fm) * Tm + tm) * 2;
      dp[0] = 0.f;
      dp[1] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------
// ConviSTFT overlap-add backward (tools_for_model.py:95-107 + clamp DCCRN.py:237):
// dframes[b][t][o] = dwav[b][t*hop+o-trim] * [|pre| <= 1] / (sum window^2 + 1e-8), with the
// pre-clamp sample recomputed from the frames (clamp passes the gradient for -1 <= pre <= 1).
// ------------------------------------------------------------------------------------------
__global__ void ola_bwd_kernel(const float* __restrict__ frames, const float* __restrict__ window,
                               const float* __restrict__ dwav, int B, int T, int win, int hop,
                               int out_len, int trim, int clamp, float* __restrict__ dframes) {
  const int64_t total = (int64_t)B * T * win;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i % win);
    const int64_t bt = i / win;
    const int t = (int)(bt % T);
    const int b = (int)(bt / T);
    const int p = t * hop + o;
    const int n = p - trim;
    float g = 0.f;
    if (n >= 0 && n < out_len) {
      int t_hi = p / hop;
      if (t_hi > T - 1) t_hi = T - 1;
      const int t_lo = p - win + 1 <= 0 ? 0 : (p - win + 1 + hop - 1) / hop;
      float acc = 0.f, coff = 0.f;
      for (int u = t_lo; u <= t_hi; ++u) {
        const int q = p - u * hop;
        acc += frames[((int64_t)b * T + u) * win + q];
        const float w = window[q];
        coff += w * w;
      }
      const float den = coff + 1e-8f;
      const float v = acc / den;
      const bool pass = !clamp || (v >= -1.f && v <= 1.f);
      if (pass) g = dwav[(int64_t)b * out_len + n] / den;
    }
    dframes[i] = g;
  }
}

// framing pad backward: dx[b][j] (+)= sum of dxp[b][i] over the padded positions i reading x[j]
__global__ void frame_pad_bwd_kernel(const float* __restrict__ dxp, int B, int L, int pad, int Lp,
                                     int mode, float* __restrict__ dx, int64_t ldx, int accumulate) {
  const int64_t total = (int64_t)B * L;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / L);
    const int j = (int)(i - (int64_t)b * L);
    const float* row = dxp + (int64_t)b * Lp;
    float s = 0.f;
    if (j + pad < Lp) s = row[j + pad];
    if (mode == 1) {
      if (j >= 1 && j <= pad && pad - j < Lp) s += row[pad - j];  // src = -(j) reflected
      const int src = 2 * (L - 1) - j;                           // src >= L reflected onto j
      if (src >= L && src < L + pad && src + pad < Lp) s += row[src + pad];
    }
    float* o = dx + (int64_t)b * ldx + j;
    *o = accumulate ? *o + s : s;
  }
}

// ------------------------------------------------------------------------------------------
// STFT log-magnitude L1 backward (framework.py:58-68, 85-101): loss = scale_sum * sum|log Y -
// log X| with X = sqrt(max(re^2 + im^2, 1e-7)) of the estimate's spectrum.
// dre = -scale * sign(log Y - log X) * re / X^2 (clamp passes for re^2+im^2 >= 1e-7), same for im.
// ------------------------------------------------------------------------------------------
__global__ void stft_mag_loss_bwd_kernel(const float* __restrict__ X, const float* __restrict__ Y,
                                         int64_t rows, int ld, int nbins, float scale,
                                         float* __restrict__ dX, int ldd) {
  const int64_t total = rows * ldd;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int col = (int)(i % ldd);
    const int64_t r = i / ldd;
    float g = 0.f;
    if (col < 2 * nbins) {
      const int f = col < nbins ? col : col - nbins;
      const float* xr = X + r * ld;
      const float* yr = Y + r * ld;
      const float xre = xr[f], xim = xr[nbins + f];
      const float yre = yr[f], yim = yr[nbins + f];
      const float px = xre * xre + xim * xim;
      const float py = yre * yre + yim * yim;
      const float mx = sqrtf(fmaxf(px, 1e-7f));
      const float my = sqrtf(fmaxf(py, 1e-7f));
      const float dlog = logf(my) - logf(mx);
      const float sgn = dlog > 0.f ? 1.f : (dlog < 0.f ? -1.f : 0.f);
      if (px >= 1e-7f) {
        const float comp = col < nbins ? xre : xim;
        g = -scale * sgn * comp / (mx * mx);
      }
    }
    dX[i] = g;
  }
}

// complex-LSTM combine backward: real = h[0][:B] - h[1][B:], imag = h[0][B:] + h[1][:B]
// (tools_for_model.py:168-169) -> dh[ws][2B][n] from dreal/dimag [B][n]
__global__ void complex_combine_bwd_kernel(const float* __restrict__ dre, const float* __restrict__ dim,
                                           int B, int64_t n, float* __restrict__ dh) {
  const int64_t total = (int64_t)B * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float r = dre[i], m = dim[i];
    const int64_t half = (int64_t)B * n;
    dh[i] = r;                  // ws 0 (real_lstm), real input
    dh[half + i] = m;           // ws 0, imag input
    dh[2 * half + i] = m;       // ws 1 (imag_lstm), real input
    dh[3 * half + i] = -r;      // ws 1, imag input
  }
}

// ------------------------------------------------------------------------------------------
// SPKD gradient fused into the BatchNorm backward of a ReviewKD output (framework.py:150-172 +
// the ABF conv2 BatchNorm, framework.py:183-186).  The Gram read z_b = round(raw_b*scale + shift)
// (the deferred BN); its gradient dz_b = sum_j M[b][j] z_j is never stored: the reduce pass
// forms the BN statistics sums of dz from it and the apply pass recomputes it to write
// d raw = k1*dz + k2*raw + k3.  One thread = (position, 4 channels) over all B samples.
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ f32x4 z_from(f32x4 v, const f32x4& sc, const f32x4& sh) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float z = fmaf(v[i], sc[i], sh[i]);
    v[i] = sizeof(T) == 2 ? (float)(__bf16)z : z;  // the Gram's rounding to the storage type
  }
  return v;
}

// z of the B samples of one (position, 4 channels), the BM loads issued together before any
// use (sample index clamped to B - 1: the k >= B terms are never read) — a `b < B ? load : 0`
// form compiled to one load + vmcnt(0) per sample.  The per-sample pass then walks b as a loop
// (M's row b in SGPRs; unrolling it put all B x B coefficients in VGPRs and halved occupancy)
// and re-reads x_b one sample ahead (cache-resident: it was just loaded).
// The raw quads are also parked in LDS ([b][thread], conflict-free 8 / 16-B rows) when they fit
// (xs != nullptr), so the sample loop reads x_b back from LDS instead of re-reading global memory.
template <typename T, int BM>
__device__ __forceinline__ void load_z(const T* base, int64_t sB, int B, const f32x4& sc,
                                       const f32x4& sh, f32x4 (&z)[BM],
                                       typename Raw4<T>::V* xs) {
  typedef typename Raw4<T>::V V;
  V t[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) t[b] = Raw4<T>::ld(base + (b < B ? b : B - 1) * sB);
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    z[b] = z_from<T>(Raw4<T>::cvt(t[b]), sc, sh);
    if (xs) xs[b * 256] = t[b];
  }
}

// LDS parking space of load_z for a 256-thread block (0 when it does not fit 64 KiB)
template <typename T, int BM>
constexpr int park_elems() {
  return sizeof(typename Raw4<T>::V) * BM * 256 <= 64 * 1024 ? BM * 256 : 1;
}
template <typename T, int BM>
constexpr bool parks() { return park_elems<T, BM>() > 1; }

template <typename T, int BM, bool EX = false>
__global__ __launch_bounds__(256) void spkd_bn_bwd_reduce_kernel(
    const T* __restrict__ raw, int64_t sB, int64_t P, int C, int Bdyn, int64_t ppb,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ Mc, const float* __restrict__ mean, const float* __restrict__ var,
    float eps, double* __restrict__ partial) {
  const int B = EX ? BM : Bdyn;
  __shared__ typename Raw4<T>::V park[park_elems<T, BM>()];
  const int CG = C >> 2;
  const int RP = 256 / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG;
  const int rl = tid / CG;
  // M [B][B] is read with uniform addresses: scalar loads into SGPRs feed the FMAs directly
  f32x4 sc, sh, mu, rs;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = cg * 4 + j;
    sc[j] = scale[c];
    sh[j] = shift[c];
    mu[j] = mean[c];
    rs[j] = (float)(1.0 / sqrt((double)var[c] + (double)eps));
  }
  const int64_t p0 = (int64_t)blockIdx.x * ppb;
  const int64_t p1 = min(P, p0 + ppb);
  double sb[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0};
  if (rl < RP) {
    for (int64_t p = p0 + rl; p < p1; p += RP) {
      const T* base = raw + p * C + cg * 4;
      f32x4 z[BM];
      load_z<T, BM>(base, sB, B, sc, sh, z, parks<T, BM>() ? park + tid : nullptr);
      float fb[4] = {0, 0, 0, 0}, fg[4] = {0, 0, 0, 0};
#pragma unroll 1
      for (int b = 0; b < B; ++b) {
        const f32x4 x = parks<T, BM>() ? Raw4<T>::cvt(park[b * 256 + tid])
                                         : ld4<T>(base + b * sB);
        f32x4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < BM; ++k)
          if (k < B) dz += Mc[b * B + k] * z[k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          fb[j] += dz[j];
          fg[j] = fmaf(dz[j], (x[j] - mu[j]) * rs[j], fg[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sb[j] += (double)fb[j];
        sg[j] += (double)fg[j];
      }
    }
  }
  __shared__ double red[256][9];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[tid][j] = sb[j];
    red[tid][4 + j] = sg[j];
  }
  __syncthreads();
  if (tid < CG) {
    double Bv[4] = {0, 0, 0, 0}, G[4] = {0, 0, 0, 0};
    for (int l = 0; l < RP; ++l) {
      const int t = l * CG + tid;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Bv[j] += red[t][j];
        G[j] += red[t][4 + j];
      }
    }
    double* q = partial + ((int64_t)blockIdx.x * C + tid * 4) * 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q[3 * j] = Bv[j];
      q[3 * j + 1] = G[j];
      q[3 * j + 2] = 0.0;
    }
  }
}

template <typename T, typename OT, int BM, bool EX = false>
__global__ __launch_bounds__(256) void spkd_bn_bwd_apply_kernel(
    const T* __restrict__ raw, int64_t sB, int64_t P, int C, int Bdyn,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ Mc, const float* __restrict__ k, OT* __restrict__ draw) {
  const int B = EX ? BM : Bdyn;
  __shared__ typename Raw4<T>::V park[park_elems<T, BM>()];
  const int CQ = C / 4;
  const int64_t nq = P * CQ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = q / CQ;
    const int c0 = (int)(q - p * CQ) * 4;
    f32x4 sc, sh, k1, k2, k3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc[j] = scale[c0 + j];
      sh[j] = shift[c0 + j];
      k1[j] = k[c0 + j];
      k2[j] = k[C + c0 + j];
      k3[j] = k[2 * C + c0 + j];
    }
    const T* base = raw + p * C + c0;
    f32x4 z[BM];
    load_z<T, BM>(base, sB, B, sc, sh, z, parks<T, BM>() ? park + threadIdx.x : nullptr);
#pragma unroll 1
    for (int b = 0; b < B; ++b) {
      const f32x4 x = parks<T, BM>() ? Raw4<T>::cvt(park[b * 256 + threadIdx.x])
                                       : ld4<T>(base + b * sB);
      f32x4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < BM; ++kk)
        if (kk < B) dz += Mc[b * B + kk] * z[kk];
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf(k1[j], dz[j], fmaf(k2[j], x[j], k3[j]));
      OT* dst = draw + b * sB + p * C + c0;
      if constexpr (sizeof(OT) == 2) {
        bf16x4b ob;
#pragma unroll
        for (int j = 0; j < 4; ++j) ob[j] = (__bf16)o[j];
        *reinterpret_cast<bf16x4b*>(dst) = ob;
      } else {
        *reinterpret_cast<f32x4*>(dst) = o;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// ABF conv1 BatchNorm backward apply fused with conv1's data gradient (framework.py:179-182:
// conv1 = 1x1 Cin -> 64, no bias).  Per row: d[c] = k0[c]*dy[c] + k1[c]*x[c] + k2[c] (the
// bn_bwd_apply of a finalize's coefficients, no PReLU), then out[n] (+)= sum_c w[c][n] * d[c] —
// the 64-channel gradient d never reaches HBM (the two-pass form wrote and re-read it in fp32:
// 2 x rows x 256 B).  Eight lanes per row, lane q owning channels 8q..8q+7: one wave load
// instruction reads 8 whole rows (1 KB contiguous).  Round 6's first form (a thread per row,
// 16 B of its 128-B row per step) fetched every line from HBM several times (PMC 1,197 MB per
// launch at N = 8 against 263 MB algorithmic: the lines left L2 between the row's steps).  Each
// lane forms its 8 channels' partial sums of all N outputs (weights from LDS, a padded stride per
// 8-channel chunk: the 8 chunks of one instruction hit disjoint banks), then the 8 lanes
// reduce-scatter them over xor 4 / 2 / 1, lane q ending with outputs q*N/8 .. (q+1)*N/8 - 1.
// ------------------------------------------------------------------------------------------
template <typename XT, typename GT, int N>
__global__ __launch_bounds__(256) void bn_bwd_conv1x1_kernel(
    const XT* __restrict__ x, const GT* __restrict__ dy, int64_t rows, const float* __restrict__ k,
    const float* __restrict__ w, float* __restrict__ out, int accumulate) {
  constexpr int C = 64;
  constexpr int WS = 8 * N + 4;  // floats per 8-channel chunk of the weights in LDS (padded)
  constexpr int RPB = 32;        // rows per block pass
  constexpr int NO = N / 8;      // outputs per lane after the reduce-scatter
  __shared__ __attribute__((aligned(16))) float wl[8 * WS];
  const int tid = threadIdx.x;
  for (int i = tid; i < C * N; i += 256) {
    const int c = i / N;
    wl[(c >> 3) * WS + (c & 7) * N + (i - c * N)] = w[i];
  }
  const int q = tid & 7;
  float k0[8], k1[8], k2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k0[j] = k[q * 8 + j];
    k1[j] = k[C + q * 8 + j];
    k2[j] = k[2 * C + q * 8 + j];
  }
  __syncthreads();
  int woff = q * WS;
  for (int64_t m = (int64_t)blockIdx.x * RPB + (tid >> 3); m < rows;
       m += (int64_t)gridDim.x * RPB) {
    // an opaque per-row offset: the weight reads stay inside the loop (hoisted, N = 8 alone held
    // 64 weights per lane in VGPRs and the wide instances spilled)
    asm volatile("" : "+v"(woff));
    const float* wq = wl + woff;
    const f32x4 xa = Raw4<XT>::cvt(Raw4<XT>::ld(x + m * C + q * 8));
    const f32x4 xb = Raw4<XT>::cvt(Raw4<XT>::ld(x + m * C + q * 8 + 4));
    const f32x4 ga = Raw4<GT>::cvt(Raw4<GT>::ld(dy + m * C + q * 8));
    const f32x4 gb = Raw4<GT>::cvt(Raw4<GT>::ld(dy + m * C + q * 8 + 4));
    float o[N];
#pragma unroll
    for (int n = 0; n < N; ++n) o[n] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = j < 4 ? xa[j & 3] : xb[j & 3];
      const float gv = j < 4 ? ga[j & 3] : gb[j & 3];
      const float dv = fmaf(k0[j], gv, fmaf(k1[j], xv, k2[j]));
#pragma unroll
      for (int n4 = 0; n4 < N; n4 += 4) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(&wq[j * N + n4]);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[n4 + e] = fmaf(dv, w4[e], o[n4 + e]);
      }
    }
#pragma unroll
    for (int s = 0; s < 3; ++s) {  // reduce-scatter over the row's 8 lanes
      const int mask = 4 >> s;
      const int H = N >> (s + 1);
      const bool hi = (q & mask) != 0;
#pragma unroll
      for (int i = 0; i < H; ++i) {
        // both values loaded first: `hi ? o[H + i] : o[i]` selects an address, and the array
        // then lived as a dynamically indexed one (a compare / select chain per access)
        const float lo_v = o[i], hi_v = o[H + i];
        const float keep = hi ? hi_v : lo_v;
        const float send = hi ? lo_v : hi_v;
        o[i] = keep + __shfl_xor(send, mask);
      }
    }
    float* op = out + m * N + q * NO;
    if constexpr (NO == 1) {
      *op = accumulate ? *op + o[0] : o[0];
    } else if constexpr (NO == 2) {
      float2 v = make_float2(o[0], o[1]);
      if (accumulate) {
        const float2 p = *reinterpret_cast<const float2*>(op);
        v.x += p.x;
        v.y += p.y;
      }
      *reinterpret_cast<float2*>(op) = v;
    } else {
#pragma unroll
      for (int i = 0; i < NO; i += 4) {
        f32x4 v = {o[i], o[i + 1], o[i + 2], o[i + 3]};
        if (accumulate) v += *reinterpret_cast<const f32x4*>(op + i);
        *reinterpret_cast<f32x4*>(op + i) = v;
      }
    }
  }
}

inline unsigned grid_of(int64_t n, int64_t cap = 8192) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), cap));
}

}  // namespace clskd

using namespace clskd;

extern "C" int32_t clskd_bn_bwd_blocks(int64_t rows, int32_t C) {
  (void)C;
  return (int32_t)std::max<int64_t>(1, std::min<int64_t>(1024, cdiv(rows, 512)));
}

extern "C" int clskd_bn_bwd(const void* x, const float* dy, int64_t rows, int32_t C,
                            const float* scale, const float* shift, const float* mean,
                            const float* var, float eps, const float* gamma, const float* alpha,
                            double* work, int32_t nblk, float* dgamma, float* dbeta,
                            float* dalpha, float* dx, int32_t accumulate_dx,
                            int32_t accumulate_params, int32_t dtype, void* stream) {
  CLSKD_CHECK_ARG(x && dy && scale && shift && mean && var && work, "bn_bwd: null pointer");
  CLSKD_CHECK_SHAPE(rows > 0 && C >= 4 && C % 4 == 0 && C <= 1024 && nblk >= 1,
                    "bn_bwd: rows=%lld C=%d nblk=%d", (long long)rows, C, nblk);
  CLSKD_CHECK_ARG(dtype == CLSKD_F32 || dtype == CLSKD_BF16, "bn_bwd: dtype");
  CLSKD_CHECK_ARG(((uintptr_t)work & 15) == 0 &&
                      (!alpha || (((uintptr_t)scale & 15) == 0 && ((uintptr_t)shift & 15) == 0)),
                  "bn_bwd: work (and scale/shift with PReLU) must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  // work layout: partial[nblk][C][3] | k[3C] (as floats) | alpha_part[C]
  double* partial = work;
  float* k = reinterpret_cast<float*>(work + (int64_t)nblk * C * 3);
  double* apart = work + (int64_t)nblk * C * 3 + cdiv(3 * C, 2);
  const int64_t rpb = cdiv(rows, nblk);
  if (dtype == CLSKD_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<__bf16>, dim3(nblk), dim3(256), 0, st,
                       (const __bf16*)x, dy, rows, C, rpb, scale, shift, mean, var, eps, alpha, partial);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(nblk), dim3(256), 0, st, (const float*)x,
                       dy, rows, C, rpb, scale, shift, mean, var, eps, alpha, partial);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, partial, nblk, rows, C,
                     gamma, mean, var, eps, dgamma, dbeta, k, alpha ? apart : nullptr,
                     accumulate_params);
  if (alpha && dalpha)
    hipLaunchKernelGGL(bn_bwd_alpha_kernel, dim3(1), dim3(64), 0, st, apart, C, dalpha,
                       accumulate_params);
  if (!dx) {  // coefficients only (k at work + nblk*C*3 doubles): the apply runs in a consumer
    CLSKD_LAUNCH_CHECK("bn_bwd");
    return CLSKD_OK;
  }
  const int64_t nq = rows * C / 4;
  if (dtype == CLSKD_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<__bf16>, dim3(grid_of(nq)), dim3(256), 0, st,
                       (const __bf16*)x, dy, rows, C, scale, shift, alpha, k, dx, accumulate_dx);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(grid_of(nq)), dim3(256), 0, st,
                       (const float*)x, dy, rows, C, scale, shift, alpha, k, dx, accumulate_dx);
  CLSKD_LAUNCH_CHECK("bn_bwd");
  return CLSKD_OK;
}

extern "C" int64_t clskd_bn_bwd_workspace(int32_t nblk, int32_t C) {
  return (int64_t)nblk * C * 3 + cdiv(3 * C, 2) + C;  // doubles
}

extern "C" int32_t clskd_abf_fuse_bwd_blocks(int32_t B, int32_t F, int32_t T) {
  const int64_t npix = (int64_t)B * F * T;
  // CLSKD_ABF_BWD_BLOCKS (experiments build, A/B): the grid cap — every block writes one row of
  // BN partials and pays the slot-reduce tail, so fewer blocks trade per-thread pixels for less
  const int cap = std::max(64, knob(KNOB_ABF_BWD_BLOCKS));
  return (int32_t)std::min<int64_t>(cdiv(npix * 16, 256), cap);
}

extern "C" int clskd_abf_fuse_bwd(const void* x1, const void* res, int32_t B, int32_t F, int32_t T,
                                  int32_t Fr, int32_t Tr, const float* w, const float* b,
                                  const float* x_scale, const float* x_shift, const void* dout,
                                  void* dx, void* dyup, const void* dnext, int32_t F2,
                                  int32_t T2, const float* mean1, const float* var1, float eps,
                                  double* bn_partial, int32_t dtype, int32_t grad_dtype,
                                  void* stream) {
  CLSKD_CHECK_ARG(x1 && res && w && b && dout && dx, "abf_fuse_bwd: null pointer");
  CLSKD_CHECK_ARG((x_scale == nullptr) == (x_shift == nullptr), "abf_fuse_bwd: scale/shift pair");
  CLSKD_CHECK_ARG(!bn_partial || (mean1 && var1), "abf_fuse_bwd: BN partials need mean1/var1");
  CLSKD_CHECK_SHAPE(!dnext || (F2 >= F && T2 >= T), "abf_fuse_bwd: next grid smaller than this one");
  CLSKD_CHECK_SHAPE(B > 0 && F > 0 && T > 0 && (int64_t)B * F * T < ((int64_t)1 << 31),
                    "abf_fuse_bwd: B*F*T must be positive and below 2^31");
  CLSKD_CHECK_ARG(grad_dtype == CLSKD_F32 || grad_dtype == CLSKD_BF16,
                  "abf_fuse_bwd: grad_dtype must be CLSKD_F32 or CLSKD_BF16");
  const unsigned grid = (unsigned)clskd_abf_fuse_bwd_blocks(B, F, T);
  hipStream_t st = as_stream(stream);
#define ABF_BWD_LAUNCH(DT, GT)                                                                   \
  hipLaunchKernelGGL((abf_fuse_bwd_kernel<DT, GT>), dim3(grid), dim3(256), 0, st,             \
                     (const DT*)x1, (const DT*)res, B, F, T, Fr, Tr, w, b, x_scale, x_shift,  \
                     (const GT*)dout, (GT*)dx, (GT*)dyup, (const GT*)dnext, F2, T2, mean1,    \
                     var1, eps, bn_partial)
  if (dtype == CLSKD_BF16) {
    if (grad_dtype == CLSKD_BF16) ABF_BWD_LAUNCH(__bf16, __bf16);
    else ABF_BWD_LAUNCH(__bf16, float);
  } else {
    if (grad_dtype == CLSKD_BF16) ABF_BWD_LAUNCH(float, __bf16);
    else ABF_BWD_LAUNCH(float, float);
  }
#undef ABF_BWD_LAUNCH
  CLSKD_LAUNCH_CHECK("abf_fuse_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_bn_bwd_conv1x1(const void* x, int32_t dtype, const void* dy,
                                    int32_t dy_dtype, int64_t rows, int32_t C, const float* k,
                                    const float* w, int32_t N, float* out, int32_t accumulate,
                                    void* stream) {
  CLSKD_CHECK_ARG(x && dy && k && w && out, "bn_bwd_conv1x1: null pointer");
  CLSKD_CHECK_SHAPE(C == 64 && (N == 8 || N == 16 || N == 32 || N == 64) && rows > 0,
                    "bn_bwd_conv1x1: C=%d (64) N=%d (8/16/32/64)", C, N);
  CLSKD_CHECK_ARG((dtype == CLSKD_F32 || dtype == CLSKD_BF16) &&
                      (dy_dtype == CLSKD_F32 || dy_dtype == CLSKD_BF16),
                  "bn_bwd_conv1x1: dtype");
  CLSKD_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 &&
                      ((uintptr_t)out & 15) == 0 && ((uintptr_t)k & 15) == 0,
                  "bn_bwd_conv1x1: x, dy, k, out must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(rows, 32), 8192));
#define BC1_N(XT_, GT_)                                                                           \
  do {                                                                                            \
    if (N == 8)                                                                                   \
      hipLaunchKernelGGL((bn_bwd_conv1x1_kernel<XT_, GT_, 8>), dim3(grid), dim3(256), 0, st,     \
                         (const XT_*)x, (const GT_*)dy, rows, k, w, out, accumulate);             \
    else if (N == 16)                                                                             \
      hipLaunchKernelGGL((bn_bwd_conv1x1_kernel<XT_, GT_, 16>), dim3(grid), dim3(256), 0, st,    \
                         (const XT_*)x, (const GT_*)dy, rows, k, w, out, accumulate);             \
    else if (N == 32)                                                                             \
      hipLaunchKernelGGL((bn_bwd_conv1x1_kernel<XT_, GT_, 32>), dim3(grid), dim3(256), 0, st,    \
                         (const XT_*)x, (const GT_*)dy, rows, k, w, out, accumulate);             \
    else                                                                                          \
      hipLaunchKernelGGL((bn_bwd_conv1x1_kernel<XT_, GT_, 64>), dim3(grid), dim3(256), 0, st,    \
                         (const XT_*)x, (const GT_*)dy, rows, k, w, out, accumulate);             \
  } while (0)
  if (dtype == CLSKD_BF16) {
    if (dy_dtype == CLSKD_BF16) BC1_N(__bf16, __bf16); else BC1_N(__bf16, float);
  } else {
    if (dy_dtype == CLSKD_BF16) BC1_N(float, __bf16); else BC1_N(float, float);
  }
#undef BC1_N
  CLSKD_LAUNCH_CHECK("bn_bwd_conv1x1");
  return CLSKD_OK;
}

extern "C" int clskd_bn_bwd_from_partials(const void* x, const void* dy, int64_t rows, int32_t C,
                                          const float* scale, const float* shift,
                                          const float* mean, const float* var, float eps,
                                          const float* gamma, double* partial, int32_t nblk,
                                          float* kbuf, float* dgamma, float* dbeta, float* dx,
                                          int32_t accumulate_dx, int32_t dtype,
                                          int32_t dy_dtype, void* stream) {
  CLSKD_CHECK_ARG(x && dy && scale && shift && mean && var && partial && kbuf,
                  "bn_bwd_from_partials: null pointer");
  CLSKD_CHECK_ARG(dy_dtype == CLSKD_F32 || dy_dtype == CLSKD_BF16,
                  "bn_bwd_from_partials: dy_dtype must be CLSKD_F32 or CLSKD_BF16");
  CLSKD_CHECK_SHAPE(rows > 0 && C >= 4 && C % 4 == 0 && nblk >= 1, "bn_bwd_from_partials: shape");
  CLSKD_CHECK_ARG(((uintptr_t)kbuf & 15) == 0, "bn_bwd_from_partials: kbuf must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  nblk = fold_partials(partial, nblk, 3 * C, 1, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, partial, nblk, rows, C,
                     gamma, mean, var, eps, dgamma, dbeta, kbuf, nullptr, 0);
  if (!dx) {  // coefficients only (kbuf): the apply runs fused into its consumer
    CLSKD_LAUNCH_CHECK("bn_bwd_from_partials");
    return CLSKD_OK;
  }
  const int64_t nq = rows * C / 4;
#define BN_APPLY_LAUNCH(T, GT)                                                                  \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, GT>), dim3(grid_of(nq)), dim3(256), 0, st,        \
                     (const T*)x, (const GT*)dy, rows, C, scale, shift, nullptr, kbuf, dx,     \
                     accumulate_dx)
  if (dtype == CLSKD_BF16) {
    if (dy_dtype == CLSKD_BF16) BN_APPLY_LAUNCH(__bf16, __bf16);
    else BN_APPLY_LAUNCH(__bf16, float);
  } else {
    if (dy_dtype == CLSKD_BF16) BN_APPLY_LAUNCH(float, __bf16);
    else BN_APPLY_LAUNCH(float, float);
  }
#undef BN_APPLY_LAUNCH
  CLSKD_LAUNCH_CHECK("bn_bwd_from_partials");
  return CLSKD_OK;
}

extern "C" int clskd_nearest_down_sum(const void* g, int32_t B, int32_t F, int32_t T, int32_t Fr,
                                      int32_t Tr, int32_t C, float* out, int32_t accumulate,
                                      int32_t g_dtype, void* stream) {
  CLSKD_CHECK_ARG(g && out, "nearest_down_sum: null pointer");
  CLSKD_CHECK_ARG(g_dtype == CLSKD_F32 || g_dtype == CLSKD_BF16,
                  "nearest_down_sum: g_dtype must be CLSKD_F32 or CLSKD_BF16");
  CLSKD_CHECK_SHAPE(C % 4 == 0 && F >= Fr && T >= Tr, "nearest_down_sum: shape");
  const int64_t total = (int64_t)B * Fr * Tr * (C / 4);
  if (g_dtype == CLSKD_BF16)
    hipLaunchKernelGGL(nearest_down_sum_kernel<__bf16>, dim3(grid_of(total)), dim3(256), 0,
                       as_stream(stream), (const __bf16*)g, B, F, T, Fr, Tr, C, out, accumulate);
  else
    hipLaunchKernelGGL(nearest_down_sum_kernel<float>, dim3(grid_of(total)), dim3(256), 0,
                       as_stream(stream), (const float*)g, B, F, T, Fr, Tr, C, out, accumulate);
  CLSKD_LAUNCH_CHECK("nearest_down_sum");
  return CLSKD_OK;
}

extern "C" int clskd_mask_e_bwd(const float* spec, int32_t ldspec, const float* mask, int32_t Tm,
                                int32_t B, int32_t T, const float* dest, int32_t ldest,
                                float* dmask, void* stream) {
  CLSKD_CHECK_ARG(spec && mask && dest && dmask, "mask_e_bwd: null pointer");
  CLSKD_CHECK_SHAPE(Tm >= T + 1, "mask_e_bwd: Tm=%d < T+1", Tm);
  CLSKD_CHECK_SHAPE(B > 0 && B <= 65535 && T > 0, "mask_e_bwd: B=%d T=%d", B, T);
  hipLaunchKernelGGL(mask_e_bwd_kernel, dim3((unsigned)cdiv(T, MASK_TT), (unsigned)B), dim3(256), 0,
                     as_stream(stream), spec, ldspec, mask, Tm, B, T, dest, ldest, dmask);
  CLSKD_LAUNCH_CHECK("mask_e_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_spkd_bn_bwd(const void* raw, int32_t dtype, int64_t sB, int64_t P, int32_t C,
                                 int32_t B, const float* scale, const float* shift, const float* coef,
                                 const float* mean, const float* var, float eps, const float* gamma,
                                 double* work, int32_t nblk, float* dgamma, float* dbeta,
                                 void* draw, int32_t draw_dtype, void* stream) {
  CLSKD_CHECK_ARG(raw && scale && shift && coef && mean && var && work && draw,
                  "spkd_bn_bwd: null pointer");
  CLSKD_CHECK_SHAPE(B >= 1 && B <= 32 && C >= 4 && C % 4 == 0 && C <= 1024 && P >= 1 && nblk >= 1,
                    "spkd_bn_bwd: B=%d C=%d P=%lld nblk=%d", B, C, (long long)P, nblk);
  CLSKD_CHECK_ARG((dtype == CLSKD_F32 || dtype == CLSKD_BF16) &&
                      (draw_dtype == CLSKD_F32 || draw_dtype == CLSKD_BF16),
                  "spkd_bn_bwd: dtype");
  hipStream_t st = as_stream(stream);
  double* partial = work;
  float* k = reinterpret_cast<float*>(work + (int64_t)nblk * C * 3);
  const int64_t ppb = cdiv(P, nblk);
  const int64_t nq = P * (C / 4);
  const unsigned ga = grid_of(nq, 16384);
#define SBB_RED(T_, BM_)                                                                            \
  do {                                                                                              \
    if (B == BM_)                                                                                   \
      hipLaunchKernelGGL((spkd_bn_bwd_reduce_kernel<T_, BM_, true>), dim3(nblk), dim3(256), 0, st, \
                         (const T_*)raw, sB, P, C, B, ppb, scale, shift, coef, mean, var, eps,     \
                         partial);                                                                  \
    else                                                                                            \
      hipLaunchKernelGGL((spkd_bn_bwd_reduce_kernel<T_, BM_, false>), dim3(nblk), dim3(256), 0, st,\
                         (const T_*)raw, sB, P, C, B, ppb, scale, shift, coef, mean, var, eps,     \
                         partial);                                                                  \
  } while (0)
#define SBB_APP(T_, OT_, BM_)                                                                       \
  do {                                                                                              \
    if (B == BM_)                                                                                   \
      hipLaunchKernelGGL((spkd_bn_bwd_apply_kernel<T_, OT_, BM_, true>), dim3(ga), dim3(256), 0,   \
                         st, (const T_*)raw, sB, P, C, B, scale, shift, coef, k, (OT_*)draw);      \
    else                                                                                            \
      hipLaunchKernelGGL((spkd_bn_bwd_apply_kernel<T_, OT_, BM_, false>), dim3(ga), dim3(256), 0,  \
                         st, (const T_*)raw, sB, P, C, B, scale, shift, coef, k, (OT_*)draw);      \
  } while (0)
  const bool big = B > 16;
  if (dtype == CLSKD_BF16) {
    if (big) SBB_RED(__bf16, 32); else SBB_RED(__bf16, 16);
  } else {
    if (big) SBB_RED(float, 32); else SBB_RED(float, 16);
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, partial, nblk,
                     (int64_t)B * P, C, gamma, mean, var, eps, dgamma, dbeta, k, nullptr, 0);
  if (dtype == CLSKD_BF16) {
    if (draw_dtype == CLSKD_BF16) { if (big) SBB_APP(__bf16, __bf16, 32); else SBB_APP(__bf16, __bf16, 16); }
    else { if (big) SBB_APP(__bf16, float, 32); else SBB_APP(__bf16, float, 16); }
  } else {
    if (draw_dtype == CLSKD_BF16) { if (big) SBB_APP(float, __bf16, 32); else SBB_APP(float, __bf16, 16); }
    else { if (big) SBB_APP(float, float, 32); else SBB_APP(float, float, 16); }
  }
#undef SBB_RED
#undef SBB_APP
  CLSKD_LAUNCH_CHECK("spkd_bn_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_ola_bwd(const float* frames, const float* window, const float* dwav, int32_t B,
                             int32_t T, int32_t win, int32_t hop, int32_t out_len, int32_t trim,
                             int32_t clamp, float* dframes, void* stream) {
  CLSKD_CHECK_ARG(frames && window && dwav && dframes, "ola_bwd: null pointer");
  const int64_t total = (int64_t)B * T * win;
  hipLaunchKernelGGL(ola_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream), frames,
                     window, dwav, B, T, win, hop, out_len, trim, clamp, dframes);
  CLSKD_LAUNCH_CHECK("ola_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_frame_pad_bwd(const float* dxp, int32_t B, int32_t L, int32_t pad, int32_t Lp,
                                   int32_t mode, float* dx, int64_t ldx, int32_t accumulate,
                                   void* stream) {
  CLSKD_CHECK_ARG(dxp && dx, "frame_pad_bwd: null pointer");
  CLSKD_CHECK_SHAPE(mode == 0 || (mode == 1 && pad < L), "frame_pad_bwd: reflect pad %d >= L %d", pad, L);
  const int64_t total = (int64_t)B * L;
  hipLaunchKernelGGL(frame_pad_bwd_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream), dxp,
                     B, L, pad, Lp, mode, dx, ldx, accumulate);
  CLSKD_LAUNCH_CHECK("frame_pad_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_stft_mag_loss_bwd(const float* X, const float* Y, int64_t rows, int32_t ld,
                                       int32_t nbins, float scale, float* dX, int32_t ldd,
                                       void* stream) {
  CLSKD_CHECK_ARG(X && Y && dX, "stft_mag_loss_bwd: null pointer");
  CLSKD_CHECK_SHAPE(ld >= 2 * nbins && ldd >= 2 * nbins, "stft_mag_loss_bwd: ld");
  hipLaunchKernelGGL(stft_mag_loss_bwd_kernel, dim3(grid_of(rows * ldd)), dim3(256), 0,
                     as_stream(stream), X, Y, rows, ld, nbins, scale, dX, ldd);
  CLSKD_LAUNCH_CHECK("stft_mag_loss_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_complex_combine_bwd(const float* dreal, const float* dimag, int32_t B,
                                         int64_t n, float* dh, void* stream) {
  CLSKD_CHECK_ARG(dreal && dimag && dh, "complex_combine_bwd: null pointer");
  hipLaunchKernelGGL(complex_combine_bwd_kernel, dim3(grid_of((int64_t)B * n)), dim3(256), 0,
                     as_stream(stream), dreal, dimag, B, n, dh);
  CLSKD_LAUNCH_CHECK("complex_combine_bwd");
  return CLSKD_OK;
}
