// BatchNorm (train/eval) + PReLU, masking mode 'E', ConviSTFT overlap-add, framing pads,
// complex-LSTM combine and the ReviewKD ABF attention fusion.  All HBM-bound elementwise /
// reduction work: float4 (16 B/lane) loads, fp64 accumulation for statistics, deterministic
// two-level reductions (no float atomics).
#include "common.h"

namespace clskd {

// ------------------------------------------------------------------------------------------
// BatchNorm statistics: block `blk` reduces rows [blk*rpb, (blk+1)*rpb) of x[rows][C] into
// partial[blk][C][2] = {sum, sumsq} (fp64).  Threads map to (row-lane, channel quad).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const T* __restrict__ x,
                                                               int64_t rows, int C, int64_t rpb,
                                                               double* __restrict__ partial) {
  const int CG = C >> 2;                 // channel quads
  const int RP = 256 / CG;               // rows in flight per pass
  const int tid = threadIdx.x;
  const int cg = tid % CG;
  const int rl = tid / CG;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = min(rows, r0 + rpb);
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  if (rl < RP) {
    for (int64_t r = r0 + rl; r < r1; r += RP) {
      const f32x4 v = load4<T>(x + r * C + cg * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] += (double)v[j];
        q[j] += (double)v[j] * (double)v[j];
      }
    }
  }
  __shared__ double red[256][9];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[tid][j] = s[j];
    red[tid][4 + j] = q[j];
  }
  __syncthreads();
  if (tid < CG) {
    double S[4] = {0, 0, 0, 0}, Q[4] = {0, 0, 0, 0};
    for (int l = 0; l < RP; ++l) {
      const int t = l * CG + tid;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        S[j] += red[t][j];
        Q[j] += red[t][4 + j];
      }
    }
    double* p = partial + ((int64_t)blockIdx.x * C + tid * 4) * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[2 * j] = S[j];
      p[2 * j + 1] = Q[j];
    }
  }
}

// one block per channel: sum partials in a fixed order (16-B {sum, sumsq} loads, eight in flight
// per lane), then a fixed LDS tree, then scale / shift & running stats.  Reads any number of
// partials directly (a 1.3 M-row activation's conv epilogue emits ~10 k): no level-2 compaction
// launch.  (1024-thread blocks measured slower inside the concurrent step: 20.9 vs 14.2 us mean.)
constexpr int BNF_T = 256;
__global__ __launch_bounds__(BNF_T) void bn_finalize_kernel(
    const double* __restrict__ partial, int nblk, int64_t rows, int C, const float* gamma,
    const float* beta, float eps, float* running_mean, float* running_var, float momentum,
    int n_updates, float* scale, float* shift, float* mean_out, float* var_out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  d2 acc = {0.0, 0.0};
#pragma unroll 8
  for (int b = tid; b < nblk; b += BNF_T) acc += *reinterpret_cast<const d2*>(partial + ((int64_t)b * C + c) * 2);
  __shared__ d2 rsq[BNF_T];
  rsq[tid] = acc;
  __syncthreads();
  for (int o = BNF_T / 2; o > 0; o >>= 1) {
    if (tid < o) rsq[tid] += rsq[tid + o];
    __syncthreads();
  }
  if (tid == 0)
    bn_channel_coeffs(c, rsq[0].x, rsq[0].y, rows, gamma, beta, eps, running_mean, running_var,
                      momentum, n_updates, scale, shift, mean_out, var_out);
}

__global__ void bn_eval_coeffs_kernel(const float* rm, const float* rv, const float* gamma,
                                      const float* beta, float eps, int C, float* scale,
                                      float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / sqrtf(rv[c] + eps);
  const float sc = invstd * (gamma ? gamma[c] : 1.f);
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - rm[c] * sc;
}

template <typename T>
struct Vec8;
template <>
struct Vec8<float> {
  __device__ static void load(const float* p, float (&v)[8]) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = a[j];
      v[4 + j] = b[j];
    }
  }
  __device__ static void store(float* p, const float (&v)[8]) {
    reinterpret_cast<f32x4*>(p)[0] = f32x4{v[0], v[1], v[2], v[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
};
template <>
struct Vec8<__bf16> {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  __device__ static void load(const __bf16* p, float (&v)[8]) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
  }
  __device__ static void store(__bf16* p, const float (&v)[8]) {
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (__bf16)v[j];
    *reinterpret_cast<bf16x8*>(p) = a;
  }
};

template <>
struct Vec8<_Float16> {
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  __device__ static void load(const _Float16* p, float (&v)[8]) {
    const f16x8 a = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
  }
  __device__ static void store(_Float16* p, const float (&v)[8]) {
    f16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (_Float16)v[j];
    *reinterpret_cast<f16x8*>(p) = a;
  }
};

// y = x*scale[c] + shift[c] (+ PReLU).  8 channels per thread; with C/8 dividing the grid
// stride each thread keeps one channel group, so scale/shift stay in registers.
template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x,
                                                       T* __restrict__ y, int64_t items, int CG,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ alpha,
                                                       int split) {
  // PReLU slope: alpha[0], or alpha[0] below channel `split` and alpha[1] from it (split > 0:
  // asteroid's OnReIm(PReLU), one slope for the real and one for the imaginary channels)
  const float a = alpha ? alpha[0] : 0.f;
  const float a1 = (alpha && split > 0) ? alpha[1] : a;
  const bool act = alpha != nullptr;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int cg = (int)(i % CG);
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[cg * 8 + j];
    sh[j] = shift[cg * 8 + j];
  }
  const bool fixed = (stride % CG) == 0;
  for (; i < items; i += stride) {
    if (!fixed) {
      const int c2 = (int)(i % CG);
      if (c2 != cg) {
        cg = c2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sc[j] = scale[cg * 8 + j];
          sh[j] = shift[cg * 8 + j];
        }
      }
    }
    float v[8];
    Vec8<T>::load(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(v[j], sc[j], sh[j]);
      if (act) t = t >= 0.f ? t : (split > 0 && cg * 8 + j >= split ? a1 : a) * t;
      v[j] = t;
    }
    Vec8<T>::store(y + i * 8, v);
  }
}

// ------------------------------------------------------------------------------------------
// framing pad: zero (mode 0) or reflect (mode 1, torch.stft center=True pad_mode='reflect')
// ------------------------------------------------------------------------------------------
__global__ void frame_pad_kernel(const float* __restrict__ x, int64_t ldx, int B, int L, int pad,
                                 int Lp, int mode, float* __restrict__ xp) {
  const int64_t total = (int64_t)B * Lp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / Lp);
    const int j = (int)(i - (int64_t)b * Lp);
    int src = j - pad;
    float v = 0.f;
    if (mode == 0) {
      if (src >= 0 && src < L) v = x[(int64_t)b * ldx + src];
    } else {
      if (src >= -pad && src < L + pad) {
        if (src < 0) src = -src;
        if (src >= L) src = 2 * (L - 1) - src;
        v = x[(int64_t)b * ldx + src];
      }
    }
    xp[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// masking mode 'E' (DCCRN.py:150-159, 207-226)
// ------------------------------------------------------------------------------------------
// The mask is time-minor ([B][256][Tm][2]) and the spectrum / estimate frequency-minor
// ([B][T][ld]): a block owns MASK_TT frames of one utterance and stages their mask columns in LDS
// (one 128-B run per bin), so both sides are read and written in contiguous runs.  Round 6: the
// one-thread-per-bin form gathered the mask with a 3.2-KB stride (PMC 195 MB read per launch at
// C2's shape against ~40 MB algorithmic).
__global__ __launch_bounds__(256) void mask_e_kernel(const float* __restrict__ spec, int ldspec,
                                                     const float* __restrict__ mask, int Tm, int B,
                                                     int T, float* __restrict__ est, int ldest,
                                                     float* __restrict__ mask_r,
                                                     float* __restrict__ mask_i) {
  __shared__ __attribute__((aligned(16))) float ml[256 * MASK_LD];
  const int b = blockIdx.y, t0 = blockIdx.x * MASK_TT;
  const int nt = min(MASK_TT, T - t0);
  mask_tile_load(mask + ((int64_t)b * 256 * Tm + t0 + 1) * 2, Tm, nt, ml);
  __syncthreads();
  for (int i = threadIdx.x; i < nt * 257; i += 256) {
    const int tt = i / 257, f = i - tt * 257;
    const int64_t bt = (int64_t)b * T + t0 + tt;
    const float re = spec[bt * ldspec + f];
    const float im = spec[bt * ldspec + 257 + f];
    const float mags = sqrtf(re * re + im * im + 1e-8f);
    const float phase = atan2f(im, re);
    float mr = 0.f, mi = 0.f;
    if (f > 0) {
      mr = ml[(f - 1) * MASK_LD + 2 * tt];
      mi = ml[(f - 1) * MASK_LD + 2 * tt + 1];
    }
    const float mm = sqrtf(mr * mr + mi * mi);
    const float rp = mr / (mm + 1e-8f);
    const float ip = mi / (mm + 1e-8f);
    const float mphase = atan2f(ip, rp);
    const float em = tanhf(mm) * mags;
    const float ep = phase + mphase;
    est[bt * ldest + f] = em * cosf(ep);
    est[bt * ldest + 257 + f] = em * sinf(ep);
    if (f < ldest - 514) est[bt * ldest + 514 + f] = 0.f;
    if (mask_r) {
      mask_r[bt * 257 + f] = mr;
      mask_i[bt * 257 + f] = mi;
    }
  }
}

// asteroid DCCRNet: mask = tanh(|M|) e^{i angle(M)} (complex_nn.BoundComplexMask('tanh')), est =
// mask * X on bins 0..255 (the Nyquist bin was dropped before the masker and is padded back as
// zero); mask BFTC [B][256][Tm][2] read at t, spectrum / est rows [B][T][ld] (re 0.., im 257..)
__global__ void mask_bdt_kernel(const float* __restrict__ spec, int ldspec,
                                const float* __restrict__ mask, int Tm, int B, int T,
                                float* __restrict__ est, int ldest) {
  const int64_t total = (int64_t)B * T * 257;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i % 257);
    const int64_t bt = i / 257;
    const int t = (int)(bt % T);
    const int b = (int)(bt / T);
    float er = 0.f, ei = 0.f;
    if (f < 256) {
      const float* mp = mask + (((int64_t)b * 256 + f) * Tm + t) * 2;
      const float mr = mp[0], mi = mp[1];
      const float mag = tanhf(hypotf(mr, mi));
      const float ph = atan2f(mi, mr);
      const float br = mag * cosf(ph), bi = mag * sinf(ph);
      const float xr = spec[bt * ldspec + f], xi = spec[bt * ldspec + 257 + f];
      er = br * xr - bi * xi;
      ei = br * xi + bi * xr;
    }
    est[bt * ldest + f] = er;
    est[bt * ldest + 257 + f] = ei;
    if (f < ldest - 514) est[bt * ldest + 514 + f] = 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// ConviSTFT overlap-add + window-energy normalisation + trim (+ clamp)
// ------------------------------------------------------------------------------------------
__global__ void ola_kernel(const float* __restrict__ frames, const float* __restrict__ window,
                           int B, int T, int win, int hop, int out_len, int trim, int clamp,
                           float* __restrict__ wav) {
  const int64_t total = (int64_t)B * out_len;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / out_len);
    const int n = (int)(i - (int64_t)b * out_len);
    const int p = n + trim;
    int t_hi = p / hop;
    if (t_hi > T - 1) t_hi = T - 1;
    int t_lo = p - win + 1 <= 0 ? 0 : (p - win + 1 + hop - 1) / hop;
    float acc = 0.f, coff = 0.f;
    for (int t = t_lo; t <= t_hi; ++t) {
      const int o = p - t * hop;
      acc += frames[((int64_t)b * T + t) * win + o];
      if (window) {
        const float w = window[o];
        coff += w * w;
      }
    }
    float v = window ? acc / (coff + 1e-8f) : acc;
    if (clamp) v = fminf(fmaxf(v, -1.f), 1.f);
    wav[i] = v;
  }
}

// real = rr - ii ; imag = ir + ri   (tools_for_model.py:168-169)
template <typename OutT>
__global__ void complex_combine_kernel(const float* rr, const float* ii, const float* ir,
                                       const float* ri, OutT* ro, OutT* io, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    ro[i] = (OutT)(rr[i] - ii[i]);
    io[i] = (OutT)(ir[i] + ri[i]);
  }
}

// ------------------------------------------------------------------------------------------
// ABF attention fusion, mid = 64 channels: 16 lanes per pixel, 4 channels per lane.
// ------------------------------------------------------------------------------------------
template <typename DT>
__global__ __launch_bounds__(256) void abf_fuse_kernel(const DT* __restrict__ x,
                                                       const DT* __restrict__ res, int B,
                                                       int F, int T, int Fr, int Tr,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       const float* __restrict__ xs,
                                                       const float* __restrict__ xh,
                                                       DT* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & 15;  // channel quad
  const int c = sub * 4;
  // optional per-channel affine on x (the ABF conv1 BatchNorm, applied on load)
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
  const int64_t npix = (int64_t)B * F * T;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;  // pixel slot
  const int64_t nslots = ((int64_t)gridDim.x * blockDim.x) >> 4;
  for (int64_t p = gw; p < npix; p += nslots) {
    const int t = (int)(p % T);
    const int64_t bf = p / T;
    const int f = (int)(bf % F);
    const int b = (int)(bf / F);
    const int fr = nearest_src(f, Fr, F);
    const int tr = nearest_src(t, Tr, T);
    f32x4 xv = load4<DT>(x + p * 64 + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = fmaf(xv[j], sx[j], hx[j]);
    const f32x4 yv = load4<DT>(res + (((int64_t)b * Fr + fr) * Tr + tr) * 64 + c);
    float d0 = 0.f, d1 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      d0 += w0x[j] * xv[j] + w0y[j] * yv[j];
      d1 += w1x[j] * xv[j] + w1y[j] * yv[j];
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      d0 += __shfl_xor(d0, o, 16);
      d1 += __shfl_xor(d1, o, 16);
    }
    const float z0 = sigmoidf_(d0 + b0);
    const float z1 = sigmoidf_(d1 + b1);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = xv[j] * z0 + yv[j] * z1;
    store4<DT>(out + p * 64 + c, o);
  }
}

__global__ void zero_f64_kernel(double* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0.0;
}

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 8192) {
  int64_t g = cdiv(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}


// Frame-major spectrum -> BFTC encoder input: out[b][f][t][0|1] = spec[b][t][re0|im0 + f].
// 64 frames x 32 bins per block through LDS: reads are 128-B bin runs of a frame, writes are
// 512-B (64 frames x re/im) runs of a bin, both coalesced.
__global__ __launch_bounds__(256) void spec_bftc_kernel(const float* __restrict__ spec, int T,
                                                        int ld, int re0, int im0, int F,
                                                        float* __restrict__ out) {
  __shared__ float tile[2][64][33];
  const int b = blockIdx.z, f0 = blockIdx.y * 32, t0 = blockIdx.x * 64;
  const float* sp = spec + (int64_t)b * T * ld;
  for (int i = threadIdx.x; i < 64 * 32; i += 256) {
    const int tt = i >> 5, ff = i & 31;
    const int t = t0 + tt, f = f0 + ff;
    const bool ok = t < T && f < F;
    tile[0][tt][ff] = ok ? sp[(int64_t)t * ld + re0 + f] : 0.f;
    tile[1][tt][ff] = ok ? sp[(int64_t)t * ld + im0 + f] : 0.f;
  }
  __syncthreads();
  float* op = out + (int64_t)b * F * T * 2;
  for (int i = threadIdx.x; i < 32 * 128; i += 256) {
    const int ff = i >> 7, r = i & 127, tt = r >> 1, c = r & 1;
    const int t = t0 + tt, f = f0 + ff;
    if (t < T && f < F) op[((int64_t)f * T + t) * 2 + c] = tile[c][tt][ff];
  }
}


// Level-2 reduction of BatchNorm partials: out[g][c] = sum_{r in [g*group, (g+1)*group)} in[r][c]
// (fixed order).  Block = 64 channels x 4 row lanes; each lane sums group/4 rows with coalesced
// 16-B {sum, sumsq} loads (consecutive lanes = consecutive channels).
__global__ __launch_bounds__(256) void bn_compact_kernel(const double* __restrict__ in, int nblk,
                                                         int C, int group,
                                                         double* __restrict__ out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int g = blockIdx.x;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int lane_r = threadIdx.x >> 6;
  const int r0 = g * group, r1 = min(nblk, r0 + group);
  d2 acc = {0.0, 0.0};
  if (c < C) {
#pragma unroll 4
    for (int r = r0 + lane_r; r < r1; r += 4)
      acc += *reinterpret_cast<const d2*>(in + ((int64_t)r * C + c) * 2);
  }
  __shared__ d2 red[4][64];
  red[lane_r][threadIdx.x & 63] = acc;
  __syncthreads();
  if (lane_r == 0 && c < C) {
    const int l = threadIdx.x & 63;
    const d2 v = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
    *reinterpret_cast<d2*>(out + ((int64_t)g * C + c) * 2) = v;
  }
}

// In-place level-2 fold of a [nblk][E] fp64 partial table (E = 2C forward {sum, sumsq}, 3C
// backward {dbeta, dgamma, dalpha}): workgroup g of G sums rows g, g+G, g+2G, ... in that order and
// overwrites row g.  Only workgroup g reads the rows = g (mod G), so the overwrite races nothing.
// Lanes = (row lane, element): consecutive lanes read consecutive elements of a row (coalesced),
// eight rows in flight per lane, then a fixed-order LDS combine over the row lanes.
constexpr int PFOLD_G = 512;
__global__ __launch_bounds__(256) void partial_fold_kernel(double* part, int nblk, int E, int G) {
  const int g = blockIdx.x;
  const int Ec = E < 256 ? E : 256;
  const int RL = 256 / Ec;
  const int tid = threadIdx.x;
  const int rl = tid / Ec;
  const int el = tid - rl * Ec;
  const int nr = (nblk - g + G - 1) / G;  // rows g + k*G, k < nr
  __shared__ double red[256];
  for (int e0 = 0; e0 < E; e0 += Ec) {
    const int e = e0 + el;
    double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rl < RL && e < E) {
      int k = rl;
      for (; k + 7 * RL < nr; k += 8 * RL) {
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += part[(int64_t)(g + (k + u * RL) * G) * E + e];
      }
      for (; k < nr; k += RL) s[0] += part[(int64_t)(g + k * G) * E + e];
    }
    red[tid] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    __syncthreads();
    if (rl == 0 && e < E) {
      double v = red[el];
      for (int l = 1; l < RL; ++l) v += red[l * Ec + el];
      part[(int64_t)g * E + e] = v;
    }
    __syncthreads();
  }
}

int fold_partials(double* part, int nblk, int E, int bit, hipStream_t st) {
  if (!(knob(KNOB_BN_PFOLD) & bit) || nblk <= 2 * PFOLD_G) return nblk;
  hipLaunchKernelGGL(partial_fold_kernel, dim3(PFOLD_G), dim3(256), 0, st, part, nblk, E, PFOLD_G);
  return PFOLD_G;
}

}  // namespace clskd

using namespace clskd;

extern "C" int32_t clskd_bn_partial_blocks(int64_t rows, int32_t C) {
  int64_t work = rows * (int64_t)C / (256 * 64);
  if (work < 1) work = 1;
  if (work > 2048) work = 2048;
  if (work > rows) work = rows;
  return (int32_t)work;
}

extern "C" int clskd_bn_stats_partial(const void* x, int64_t rows, int32_t C, double* partial,
                                      int32_t nblk, int32_t dtype, void* stream) {
  CLSKD_CHECK_ARG(x && partial, "bn_stats: null pointer");
  CLSKD_CHECK_SHAPE(rows > 0 && C >= 4 && C % 4 == 0 && C <= 1024, "bn_stats: bad C=%d", C);
  CLSKD_CHECK_SHAPE(nblk >= 1, "bn_stats: nblk");
  CLSKD_CHECK_ARG(((uintptr_t)x & 15) == 0, "bn_stats: x must be 16-byte aligned");
  CLSKD_CHECK_ARG(dtype == CLSKD_F32 || dtype == CLSKD_BF16 || dtype == CLSKD_F16, "bn_stats: dtype");
  const int64_t rpb = cdiv(rows, nblk);
  if (dtype == CLSKD_BF16)
    hipLaunchKernelGGL(bn_stats_partial_kernel<__bf16>, dim3(nblk), dim3(256), 0, as_stream(stream),
                       (const __bf16*)x, rows, C, rpb, partial);
  else if (dtype == CLSKD_F16)
    hipLaunchKernelGGL(bn_stats_partial_kernel<_Float16>, dim3(nblk), dim3(256), 0, as_stream(stream),
                       (const _Float16*)x, rows, C, rpb, partial);
  else
    hipLaunchKernelGGL(bn_stats_partial_kernel<float>, dim3(nblk), dim3(256), 0, as_stream(stream),
                       (const float*)x, rows, C, rpb, partial);
  CLSKD_LAUNCH_CHECK("bn_stats_partial");
  return CLSKD_OK;
}

extern "C" int clskd_bn_compact(const double* partial, int32_t nblk, int32_t C, int32_t group,
                                double* out, void* stream) {
  CLSKD_CHECK_ARG(partial && out, "bn_compact: null pointer");
  CLSKD_CHECK_SHAPE(nblk > 0 && C > 0 && group >= 4, "bn_compact: shape");
  CLSKD_CHECK_ARG(((uintptr_t)partial & 15) == 0 && ((uintptr_t)out & 15) == 0,
                  "bn_compact: partials must be 16-byte aligned");
  hipLaunchKernelGGL(bn_compact_kernel, dim3((unsigned)cdiv(nblk, group), (unsigned)cdiv(C, 64)),
                     dim3(256), 0, as_stream(stream), partial, nblk, C, group, out);
  CLSKD_LAUNCH_CHECK("bn_compact");
  return CLSKD_OK;
}

extern "C" int clskd_bn_finalize(double* partial, int32_t nblk, int64_t rows, int32_t C,
                                 const float* gamma, const float* beta, float eps,
                                 float* running_mean, float* running_var, float momentum,
                                 int32_t n_updates, float* scale, float* shift, float* mean_out,
                                 float* var_out, void* stream) {
  CLSKD_CHECK_ARG(partial && scale && shift, "bn_finalize: null pointer");
  CLSKD_CHECK_SHAPE(C > 0 && nblk > 0 && rows > 0, "bn_finalize: shape");
  CLSKD_CHECK_ARG(((uintptr_t)partial & 15) == 0, "bn_finalize: partials must be 16-byte aligned");
  if (skip_kernel(SKIP_BN_FINALIZE)) return CLSKD_OK;
  nblk = fold_partials(partial, nblk, 2 * C, 2, as_stream(stream));
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(BNF_T), 0, as_stream(stream), partial, nblk,
                     rows, C, gamma, beta, eps, running_mean, running_var, momentum, n_updates,
                     scale, shift, mean_out, var_out);
  CLSKD_LAUNCH_CHECK("bn_finalize");
  return CLSKD_OK;
}

extern "C" int clskd_bn_eval_coeffs(const float* running_mean, const float* running_var,
                                    const float* gamma, const float* beta, float eps, int32_t C,
                                    float* scale, float* shift, void* stream) {
  CLSKD_CHECK_ARG(running_mean && running_var && scale && shift, "bn_eval: null pointer");
  hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3((unsigned)cdiv(C, 256)), dim3(256), 0,
                     as_stream(stream), running_mean, running_var, gamma, beta, eps, C, scale,
                     shift);
  CLSKD_LAUNCH_CHECK("bn_eval_coeffs");
  return CLSKD_OK;
}

static int bn_apply_impl(const void* x, void* y, int64_t rows, int32_t C, const float* scale,
                         const float* shift, const float* alpha, int split, int32_t dtype,
                         void* stream) {
  CLSKD_CHECK_ARG(x && y && scale && shift, "bn_apply: null pointer");
  CLSKD_CHECK_SHAPE(C % 8 == 0 && rows > 0, "bn_apply: C=%d must be a multiple of 8", C);
  CLSKD_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "bn_apply: alignment");
  CLSKD_CHECK_ARG(dtype == CLSKD_F32 || dtype == CLSKD_BF16 || dtype == CLSKD_F16, "bn_apply: dtype");
  if (skip_kernel(SKIP_BN_APPLY)) return CLSKD_OK;
  const int64_t items = rows * C / 8;
  const int CG = C / 8;
  // grid a multiple of CG-friendly size: 256 threads/block, stride = 256*grid
  int64_t g = cdiv(items, 256);
  if (g > 4096) g = 4096;
  if (dtype == CLSKD_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<__bf16>, dim3((unsigned)g), dim3(256), 0, as_stream(stream),
                       (const __bf16*)x, (__bf16*)y, items, CG, scale, shift, alpha, split);
  else if (dtype == CLSKD_F16)
    hipLaunchKernelGGL(bn_apply_kernel<_Float16>, dim3((unsigned)g), dim3(256), 0, as_stream(stream),
                       (const _Float16*)x, (_Float16*)y, items, CG, scale, shift, alpha, split);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3((unsigned)g), dim3(256), 0, as_stream(stream),
                       (const float*)x, (float*)y, items, CG, scale, shift, alpha, split);
  CLSKD_LAUNCH_CHECK("bn_apply");
  return CLSKD_OK;
}

extern "C" int clskd_bn_apply(const void* x, void* y, int64_t rows, int32_t C,
                              const float* scale, const float* shift, const float* alpha,
                              int32_t dtype, void* stream) {
  return bn_apply_impl(x, y, rows, C, scale, shift, alpha, 0, dtype, stream);
}

extern "C" int clskd_bn_apply_reim(const void* x, void* y, int64_t rows, int32_t C,
                                   const float* scale, const float* shift,
                                   const float* alpha_re_im, int32_t dtype, void* stream) {
  CLSKD_CHECK_ARG(alpha_re_im, "bn_apply_reim: null alpha");
  CLSKD_CHECK_SHAPE(C % 2 == 0, "bn_apply_reim: C=%d must be even", C);
  return bn_apply_impl(x, y, rows, C, scale, shift, alpha_re_im, C / 2, dtype, stream);
}

extern "C" int clskd_frame_pad(const float* x, int64_t ldx, int32_t B, int32_t L, int32_t pad,
                               int32_t Lp, int32_t mode, float* xp, void* stream) {
  CLSKD_CHECK_ARG(x && xp, "frame_pad: null pointer");
  CLSKD_CHECK_SHAPE(B > 0 && L > 0 && Lp > 0 && pad >= 0, "frame_pad: shape");
  CLSKD_CHECK_SHAPE(mode == 0 || pad < L, "frame_pad: reflect pad %d needs L > pad", pad);
  hipLaunchKernelGGL(frame_pad_kernel, dim3(grid_for((int64_t)B * Lp)), dim3(256), 0,
                     as_stream(stream), x, ldx, B, L, pad, Lp, mode, xp);
  CLSKD_LAUNCH_CHECK("frame_pad");
  return CLSKD_OK;
}

extern "C" int clskd_spec_bftc(const float* spec, int32_t B, int32_t T, int32_t ld, int32_t re0,
                               int32_t im0, int32_t F, float* out, void* stream) {
  CLSKD_CHECK_ARG(spec && out, "spec_bftc: null pointer");
  CLSKD_CHECK_SHAPE(B > 0 && T > 0 && F > 0 && re0 >= 0 && im0 >= 0 && re0 + F <= ld &&
                        im0 + F <= ld,
                    "spec_bftc: bins [%d,+%d) / [%d,+%d) outside a row of %d", re0, F, im0, F, ld);
  hipLaunchKernelGGL(spec_bftc_kernel, dim3((unsigned)cdiv(T, 64), (unsigned)cdiv(F, 32), B),
                     dim3(256), 0, as_stream(stream), spec, T, ld, re0, im0, F, out);
  CLSKD_LAUNCH_CHECK("spec_bftc");
  return CLSKD_OK;
}

extern "C" int clskd_mask_e(const float* spec, int32_t ldspec, const float* mask, int32_t Tm,
                            int32_t B, int32_t T, float* est, int32_t ldest, float* mask_r,
                            float* mask_i, void* stream) {
  CLSKD_CHECK_ARG(spec && mask && est, "mask_e: null pointer");
  CLSKD_CHECK_SHAPE(ldspec >= 514 && ldest >= 514 && ldest - 514 <= 257 && Tm >= T + 1,
                    "mask_e: bad strides");
  CLSKD_CHECK_SHAPE(B > 0 && B <= 65535 && T > 0, "mask_e: B=%d T=%d", B, T);
  hipLaunchKernelGGL(mask_e_kernel, dim3((unsigned)cdiv(T, MASK_TT), (unsigned)B), dim3(256), 0,
                     as_stream(stream), spec, ldspec, mask, Tm, B, T, est, ldest, mask_r, mask_i);
  CLSKD_LAUNCH_CHECK("mask_e");
  return CLSKD_OK;
}

extern "C" int clskd_mask_bdt(const float* spec, int32_t ldspec, const float* mask, int32_t Tm,
                              int32_t B, int32_t T, float* est, int32_t ldest, void* stream) {
  CLSKD_CHECK_ARG(spec && mask && est, "mask_bdt: null pointer");
  CLSKD_CHECK_SHAPE(ldspec >= 514 && ldest >= 514 && ldest - 514 <= 257 && Tm >= T,
                    "mask_bdt: bad strides");
  hipLaunchKernelGGL(mask_bdt_kernel, dim3(grid_for((int64_t)B * T * 257)), dim3(256), 0,
                     as_stream(stream), spec, ldspec, mask, Tm, B, T, est, ldest);
  CLSKD_LAUNCH_CHECK("mask_bdt");
  return CLSKD_OK;
}

extern "C" int clskd_ola(const float* frames, const float* window, int32_t B, int32_t T,
                         int32_t win, int32_t hop, int32_t out_len, int32_t trim, int32_t clamp,
                         float* wav, void* stream) {
  CLSKD_CHECK_ARG(frames && wav, "ola: null pointer");
  CLSKD_CHECK_SHAPE(out_len > 0 && T > 0 && hop > 0 && win >= hop, "ola: shape");
  hipLaunchKernelGGL(ola_kernel, dim3(grid_for((int64_t)B * out_len)), dim3(256), 0,
                     as_stream(stream), frames, window, B, T, win, hop, out_len, trim, clamp, wav);
  CLSKD_LAUNCH_CHECK("ola");
  return CLSKD_OK;
}

extern "C" int clskd_complex_combine(const float* rr, const float* ii, const float* ir,
                                     const float* ri, float* real_out, float* imag_out,
                                     int64_t n, void* stream) {
  CLSKD_CHECK_ARG(rr && ii && ir && ri && real_out && imag_out, "complex_combine: null pointer");
  hipLaunchKernelGGL(complex_combine_kernel<float>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                     rr, ii, ir, ri, real_out, imag_out, n);
  CLSKD_LAUNCH_CHECK("complex_combine");
  return CLSKD_OK;
}

extern "C" int clskd_complex_combine_dt(const float* rr, const float* ii, const float* ir,
                                        const float* ri, void* real_out, void* imag_out, int64_t n,
                                        int32_t out_dtype, void* stream) {
  CLSKD_CHECK_ARG(rr && ii && ir && ri && real_out && imag_out, "complex_combine_dt: null pointer");
  CLSKD_CHECK_ARG(out_dtype == CLSKD_F32 || out_dtype == CLSKD_BF16 || out_dtype == CLSKD_F16,
                  "complex_combine_dt: dtype");
  const dim3 g(grid_for(n)), b(256);
  if (out_dtype == CLSKD_BF16)
    hipLaunchKernelGGL(complex_combine_kernel<__bf16>, g, b, 0, as_stream(stream), rr, ii, ir, ri,
                       (__bf16*)real_out, (__bf16*)imag_out, n);
  else if (out_dtype == CLSKD_F16)
    hipLaunchKernelGGL(complex_combine_kernel<_Float16>, g, b, 0, as_stream(stream), rr, ii, ir, ri,
                       (_Float16*)real_out, (_Float16*)imag_out, n);
  else
    hipLaunchKernelGGL(complex_combine_kernel<float>, g, b, 0, as_stream(stream), rr, ii, ir, ri,
                       (float*)real_out, (float*)imag_out, n);
  CLSKD_LAUNCH_CHECK("complex_combine_dt");
  return CLSKD_OK;
}

extern "C" int clskd_abf_fuse(const void* x, const void* res, int32_t B, int32_t F, int32_t T,
                              int32_t Fr, int32_t Tr, const float* w, const float* b,
                              const float* x_scale, const float* x_shift, void* out,
                              int32_t dtype, void* stream) {
  CLSKD_CHECK_ARG(x && res && w && b && out, "abf_fuse: null pointer");
  CLSKD_CHECK_ARG((x_scale == nullptr) == (x_shift == nullptr),
                  "abf_fuse: x_scale and x_shift go together");
  CLSKD_CHECK_SHAPE(B > 0 && F > 0 && T > 0 && Fr > 0 && Tr > 0, "abf_fuse: shape");
  CLSKD_CHECK_ARG(dtype == CLSKD_F32 || dtype == CLSKD_BF16, "abf_fuse: dtype");
  const int64_t npix = (int64_t)B * F * T;
  if (dtype == CLSKD_BF16)
    hipLaunchKernelGGL(abf_fuse_kernel<__bf16>, dim3(grid_for(npix * 16)), dim3(256), 0,
                       as_stream(stream), (const __bf16*)x, (const __bf16*)res, B, F, T, Fr, Tr, w, b,
                       x_scale, x_shift, (__bf16*)out);
  else
    hipLaunchKernelGGL(abf_fuse_kernel<float>, dim3(grid_for(npix * 16)), dim3(256), 0,
                       as_stream(stream), (const float*)x, (const float*)res, B, F, T, Fr, Tr, w, b,
                       x_scale, x_shift, (float*)out);
  CLSKD_LAUNCH_CHECK("abf_fuse");
  return CLSKD_OK;
}

extern "C" int clskd_zero_f64(double* p, int64_t n, void* stream) {
  CLSKD_CHECK_ARG(p, "zero_f64: null pointer");
  hipLaunchKernelGGL(zero_f64_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, n);
  CLSKD_LAUNCH_CHECK("zero_f64");
  return CLSKD_OK;
}
