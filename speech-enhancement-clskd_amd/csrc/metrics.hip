// Validation metrics of distill.py:149-199 (asteroid get_metrics with COMPUTE_METRICS =
// ["si_sdr", "stoi"], distill.py:35): scale-invariant SDR and short-time objective
// intelligibility, per utterance, on the device.
//
// SI-SDR is pb_bss_eval's (= tools_for_loss.py:50-92 without eps): float64, no mean removal,
// two passes per row (the residual is formed explicitly, not by expanding the square).
//
// STOI is pystoi 0.3.3's classic measure (tools_for_model.py:595-600 calls it), restated as six
// small fp64 kernels, all per utterance and deterministic (fixed reduction orders):
//   1. stoi_filter_kernel     Octave resample() anti-aliasing filter (Kaiser-windowed sinc,
//                             normalised, x up), with scipy resample_poly's pre-padding;
//   2. stoi_resample_kernel   polyphase resampling to 10 kHz (upfirdn, output samples centred);
//   3. stoi_mask_kernel       frame energies of the clean signal (256-sample MATLAB-Hanning
//                             frames, hop 128), frames more than 40 dB below the loudest one
//                             dropped, kept-frame list by a block scan;
//   4. stoi_ola_kernel        overlap-add of the kept windowed frames (both signals);
//   5. stoi_band_kernel       per 256-sample frame of those: 512-point DFT power summed into the
//                             15 one-third-octave bands (150 Hz ... 4.3 kHz) -> band envelopes;
//   6. stoi_corr_kernel       30-frame segments: normalise and clip the processed envelope
//                             (-15 dB SDR bound), correlate with the clean one, mean over
//                             segments and bands.
// The kept-frame count is data-dependent: it stays in device memory and every later kernel
// reads it (no host round trip); grids are sized for the all-kept case.
#include <math.h>

#include "common.h"

namespace clskd {

namespace stoi {
constexpr int FS = 10000;
constexpr int NFRAME = 256;
constexpr int HOP = 128;
constexpr int NFFT = 512;
constexpr int NBAND = 15;
constexpr int NSEG = 30;
constexpr double BETA = -15.0;
constexpr double DYN_RANGE = 40.0;
constexpr double EPS = 2.220446049250313e-16;  // np.finfo(float).eps
}  // namespace stoi

struct StoiPlan {
  int up, down;         // reduced resampling ratio (1, 1: none)
  int half_len;         // filter half length L (filter = 2L + 1 taps)
  int pre_pad;          // scipy resample_poly zero pre-padding of the filter
  int pre_remove;       // output samples dropped at the front
  int n_in, n_out;      // samples per utterance before / after resampling
  int nfr;              // energy frames of the 10 kHz signal (range(0, n_out - 256, 128))
  int ls_max;           // longest silence-removed signal ((nfr - 1) * 128 + 256)
  int nst_max;          // most STFT frames of it (nfr - 1)
  int band_lo[stoi::NBAND], band_hi[stoi::NBAND];
  double beta;          // Kaiser beta
  double stop;          // stopband cut-off (fraction of the up-sampled rate)
  int64_t off_h, off_x, off_kept, off_nkept, off_sil, off_tob, bytes;  // workspace layout
};

static int64_t gcd64(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

static StoiPlan stoi_plan(int B, int L, int fs) {
  using namespace stoi;
  StoiPlan p{};
  p.n_in = L;
  if (fs == FS) {
    p.up = p.down = 1;
    p.n_out = L;
  } else {
    const int64_t g = gcd64(FS, fs);
    p.up = (int)(FS / g);
    p.down = (int)(fs / g);
    // pystoi _resample_window_oct: 60 dB rejection, roll-off = stopband / 10
    const double stop = 1.0 / (2.0 * (p.up > p.down ? p.up : p.down));
    const double roll = stop / 10.0;
    const double rej = 60.0;
    p.half_len = (int)ceil((rej - 8.0) / (28.714 * roll));
    p.beta = 0.1102 * (rej - 8.7);
    p.stop = stop;
    p.pre_pad = p.down - p.half_len % p.down;  // scipy.signal.resample_poly
    p.pre_remove = (p.half_len + p.pre_pad) / p.down;
    const int64_t n = (int64_t)L * p.up;
    p.n_out = (int)(n / p.down + (n % p.down ? 1 : 0));
  }
  p.nfr = p.n_out > NFRAME ? (p.n_out - NFRAME + HOP - 1) / HOP : 0;
  p.ls_max = p.nfr > 0 ? (p.nfr - 1) * HOP + NFRAME : NFRAME;
  p.nst_max = p.nfr > 1 ? p.nfr - 1 : 1;
  // pystoi thirdoct: band edges matched to the nearest DFT bin of the 10 kHz / 512 grid
  for (int k = 0; k < NBAND; ++k) {
    const double lo = 150.0 * pow(2.0, (2.0 * k - 1.0) / 6.0);
    const double hi = 150.0 * pow(2.0, (2.0 * k + 1.0) / 6.0);
    int bl = 0, bh = 0;
    double dl = 1e300, dh = 1e300;
    for (int i = 0; i <= NFFT / 2; ++i) {
      const double f = (double)FS * i / NFFT;
      const double el = (f - lo) * (f - lo), eh = (f - hi) * (f - hi);
      if (el < dl) { dl = el; bl = i; }
      if (eh < dh) { dh = eh; bh = i; }
    }
    p.band_lo[k] = bl;
    p.band_hi[k] = bh;
  }
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  int64_t o = 0;
  p.off_h = o;     o += al(8LL * (2 * p.half_len + 1 + p.pre_pad + 8));
  p.off_x = o;     o += al(8LL * 2 * B * p.n_out);
  p.off_kept = o;  o += al(4LL * B * (p.nfr > 0 ? p.nfr : 1));
  p.off_nkept = o; o += al(4LL * B);
  p.off_sil = o;   o += al(8LL * 2 * B * p.ls_max);
  p.off_tob = o;   o += al(8LL * 2 * B * NBAND * p.nst_max);
  p.bytes = o;
  return p;
}

// MATLAB hanning(256) = numpy hanning(258)[1:-1]
__device__ __forceinline__ double hann256(int n) {
  return 0.5 - 0.5 * cospi(2.0 * (n + 1) / 257.0);
}

// I0 by its power series (converges to fp64 precision in < 40 terms for x <= 10)
__device__ double bessel_i0(double x) {
  double term = 1.0, sum = 1.0;
  const double q = 0.25 * x * x;
  for (int k = 1; k < 60; ++k) {
    term *= q / ((double)k * k);
    sum += term;
    if (term < 1e-17 * sum) break;
  }
  return sum;
}

// hp[j] = 0 for j < pre_pad, else up * h[j - pre_pad] / sum(h): the filter resample_poly runs
__global__ __launch_bounds__(1024) void stoi_filter_kernel(int L, int up, int pre_pad, double stop,
                                                           double beta, double* __restrict__ hp) {
  const int M = 2 * L + 1;
  __shared__ double red[1024];
  const double i0b = bessel_i0(beta);
  double part = 0.0;
  for (int t = threadIdx.x; t < M; t += 1024) {
    const double r = (double)(t - L) / (double)L;
    const double kais = bessel_i0(beta * sqrt(fmax(0.0, 1.0 - r * r))) / i0b;
    const double xx = 2.0 * stop * (double)(t - L);
    const double sinc = xx == 0.0 ? 1.0 : sinpi(xx) / (M_PI * xx);
    const double h = kais * 2.0 * up * stop * sinc;
    hp[pre_pad + t] = h;
    part += h;
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double scale = (double)up / red[0];
  for (int t = threadIdx.x; t < M; t += 1024) hp[pre_pad + t] *= scale;
  for (int t = threadIdx.x; t < pre_pad; t += 1024) hp[t] = 0.0;
}

// y[k] = sum_s hp[(k + pre_remove) * down - s * up] x[s]   (upfirdn, zero padding)
__global__ __launch_bounds__(256) void stoi_resample_kernel(
    const float* __restrict__ clean, const float* __restrict__ est, int64_t ldc, int64_t lde,
    int n_in, int n_out, int up, int down, int pre_remove, int lenhp,
    const double* __restrict__ hp, double* __restrict__ xr) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int u = blockIdx.y, sig = blockIdx.z;
  if (k >= n_out) return;
  const float* x = sig == 0 ? clean + u * ldc : est + u * lde;
  double acc = 0.0;
  if (up == 1 && down == 1) {
    acc = (double)x[k];
  } else {
    const int64_t i = (int64_t)(k + pre_remove) * down;
    // s with 0 <= i - s*up < lenhp, 0 <= s < n_in; ascending s
    int64_t s0 = (i - (lenhp - 1) + up - 1) / up;
    if (i - (lenhp - 1) < 0) s0 = 0;
    int64_t s1 = i / up;
    if (s1 > n_in - 1) s1 = n_in - 1;
    for (int64_t s = s0; s <= s1; ++s) acc += hp[i - s * up] * (double)x[s];
  }
  xr[((int64_t)sig * gridDim.y + u) * n_out + k] = acc;
}

// kept-frame list of utterance u: clean-frame energies (dB), loudest frame - 40 dB threshold,
// block scan over frames in order
__global__ __launch_bounds__(1024) void stoi_mask_kernel(const double* __restrict__ xr, int n_out,
                                                         int nfr, int* __restrict__ kept,
                                                         int* __restrict__ n_kept) {
  using namespace stoi;
  const int u = blockIdx.x, tid = threadIdx.x;
  const double* x = xr + (int64_t)u * n_out;  // signal 0 = clean
  extern __shared__ double e_s[];             // [nfr] frame energies (dB)
  __shared__ double red[1024];
  __shared__ int cnt[1024];
  double mx = -1e300;
  for (int f = tid; f < nfr; f += 1024) {
    double s = 0.0;
    for (int n = 0; n < NFRAME; ++n) {
      const double v = hann256(n) * x[f * HOP + n];
      s += v * v;
    }
    const double e = 20.0 * log10(sqrt(s) + EPS);
    e_s[f] = e;
    mx = fmax(mx, e);
  }
  red[tid] = mx;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  const double thr = red[0] - DYN_RANGE;
  // contiguous frame range per thread, counts, exclusive scan, ordered writes
  const int per = (nfr + 1023) / 1024;
  const int f0 = tid * per, f1 = min(nfr, f0 + per);
  int c = 0;
  for (int f = f0; f < f1; ++f) c += (thr - e_s[f]) < 0.0 ? 1 : 0;
  cnt[tid] = c;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = tid >= o ? cnt[tid - o] : 0;
    __syncthreads();
    cnt[tid] += v;
    __syncthreads();
  }
  int pos = cnt[tid] - c;
  int* kl = kept + (int64_t)u * nfr;
  for (int f = f0; f < f1; ++f)
    if ((thr - e_s[f]) < 0.0) kl[pos++] = f;
  if (tid == 1023) n_kept[u] = cnt[1023];
}

// silence-removed signals: sum of the kept windowed frames, placed at hop spacing
__global__ __launch_bounds__(256) void stoi_ola_kernel(const double* __restrict__ xr, int n_out,
                                                       const int* __restrict__ kept, int nfr,
                                                       const int* __restrict__ n_kept, int ls_max,
                                                       double* __restrict__ sil) {
  using namespace stoi;
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int u = blockIdx.y, sig = blockIdx.z, B = gridDim.y;
  const int nk = n_kept[u];
  const int ls = (nk - 1) * HOP + NFRAME;
  if (n >= ls) return;
  const double* x = xr + ((int64_t)sig * B + u) * n_out;
  const int* kl = kept + (int64_t)u * nfr;
  double acc = 0.0;
  const int ih = n / HOP;
  for (int i = ih - 1; i <= ih; ++i) {  // frames in pystoi's accumulation order
    if (i < 0 || i >= nk) continue;
    const int r = n - i * HOP;
    if (r < 0 || r >= NFRAME) continue;
    acc += hann256(r) * x[kl[i] * HOP + r];
  }
  sil[((int64_t)sig * B + u) * ls_max + n] = acc;
}

struct BandArgs {
  int lo[stoi::NBAND], hi[stoi::NBAND];
};

// band envelope of STFT frame j (one workgroup): tob[sig][u][band][j] = sqrt(sum |X_k|^2)
__global__ __launch_bounds__(256) void stoi_band_kernel(const double* __restrict__ sil, int ls_max,
                                                        const int* __restrict__ n_kept, int nst_max,
                                                        BandArgs bands, int kmax,
                                                        double* __restrict__ tob) {
  using namespace stoi;
  const int j = blockIdx.x, u = blockIdx.y, sig = blockIdx.z, B = gridDim.y;
  const int nst = n_kept[u] - 1;
  if (j >= nst) return;
  __shared__ double v[NFRAME];
  __shared__ double cs[NFFT], sn[NFFT];
  __shared__ double pw[NFFT / 2 + 1];
  const int tid = threadIdx.x;
  const double* x = sil + ((int64_t)sig * B + u) * ls_max + (int64_t)j * HOP;
  v[tid] = hann256(tid) * x[tid];
  for (int m = tid; m < NFFT; m += 256) {
    double s, c;
    sincospi((double)m / (NFFT / 2), &s, &c);
    cs[m] = c;
    sn[m] = s;
  }
  __syncthreads();
  for (int k = tid; k < kmax; k += 256) {
    double re = 0.0, im = 0.0;
    for (int n = 0; n < NFRAME; ++n) {
      const int m = (k * n) & (NFFT - 1);
      re += v[n] * cs[m];
      im -= v[n] * sn[m];
    }
    pw[k] = re * re + im * im;
  }
  __syncthreads();
  if (tid < NBAND) {
    double s = 0.0;
    for (int k = bands.lo[tid]; k < bands.hi[tid]; ++k) s += pw[k];
    tob[(((int64_t)sig * B + u) * NBAND + tid) * nst_max + j] = sqrt(s);
  }
}

// d[u] = mean over 30-frame segments and bands of the clipped, normalised envelope correlation
__global__ __launch_bounds__(256) void stoi_corr_kernel(const double* __restrict__ tob,
                                                        const int* __restrict__ n_kept, int nst_max,
                                                        double* __restrict__ d) {
  using namespace stoi;
  const int u = blockIdx.x, B = gridDim.x, tid = threadIdx.x;
  const int nst = n_kept[u] - 1;
  if (nst < NSEG) {  // pystoi: "Not enough STFT frames", returns 1e-5
    if (tid == 0) d[u] = 1e-5;
    return;
  }
  const int J = nst - NSEG + 1;
  const double clip = 1.0 + pow(10.0, -BETA / 20.0);
  const double* tx = tob + ((int64_t)0 * B + u) * NBAND * nst_max;
  const double* ty = tob + ((int64_t)1 * B + u) * NBAND * nst_max;
  double acc = 0.0;
  for (int q = tid; q < J * NBAND; q += 256) {
    const int s = q / NBAND, b = q - (q / NBAND) * NBAND;
    const double* xs = tx + b * nst_max + s;
    const double* ys = ty + b * nst_max + s;
    double nx = 0.0, ny = 0.0;
    for (int i = 0; i < NSEG; ++i) {
      nx += xs[i] * xs[i];
      ny += ys[i] * ys[i];
    }
    const double alpha = sqrt(nx) / (sqrt(ny) + EPS);
    double yp[NSEG];
    double my = 0.0, mxv = 0.0;
    for (int i = 0; i < NSEG; ++i) {
      yp[i] = fmin(ys[i] * alpha, xs[i] * clip);
      my += yp[i];
      mxv += xs[i];
    }
    my /= NSEG;
    mxv /= NSEG;
    double nyp = 0.0, nxc = 0.0;
    for (int i = 0; i < NSEG; ++i) {
      yp[i] -= my;
      const double xc = xs[i] - mxv;
      nyp += yp[i] * yp[i];
      nxc += xc * xc;
    }
    const double iy = 1.0 / (sqrt(nyp) + EPS), ix = 1.0 / (sqrt(nxc) + EPS);
    double c = 0.0;
    for (int i = 0; i < NSEG; ++i) c += (yp[i] * iy) * ((xs[i] - mxv) * ix);
    acc += c;
  }
  __shared__ double red[256];
  red[tid] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) d[u] = red[0] / ((double)J * NBAND);
}

// pb_bss SI-SDR per row (float64, no eps): alpha = <r,e>/<r,r>; 10 log10(|a r|^2 / |e - a r|^2)
__global__ __launch_bounds__(256) void sisdr_rows_f64_kernel(const float* __restrict__ ref,
                                                             const float* __restrict__ est, int L,
                                                             int64_t ldr, int64_t lde,
                                                             double* __restrict__ out) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* r = ref + row * ldr;
  const float* e = est + row * lde;
  __shared__ double red[2][256];
  double re = 0.0, rr = 0.0;
  for (int i = tid; i < L; i += 256) {
    re += (double)r[i] * (double)e[i];
    rr += (double)r[i] * (double)r[i];
  }
  red[0][tid] = re;
  red[1][tid] = rr;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
    }
    __syncthreads();
  }
  const double energy = red[1][0];
  const double alpha = red[0][0] / energy;
  __syncthreads();
  double nn = 0.0;
  for (int i = tid; i < L; i += 256) {
    const double n = (double)e[i] - alpha * (double)r[i];
    nn += n * n;
  }
  red[0][tid] = nn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[0][tid] += red[0][tid + o];
    __syncthreads();
  }
  if (tid == 0) out[row] = 10.0 * log10(alpha * alpha * energy / red[0][0]);
}

}  // namespace clskd

using namespace clskd;

extern "C" int64_t clskd_stoi_workspace(int32_t B, int32_t L, int32_t fs) {
  if (B < 1 || L < 1 || fs < 1) return -1;
  return stoi_plan(B, L, fs).bytes;
}

extern "C" int clskd_stoi(const float* clean, const float* est, int32_t B, int32_t L,
                          int64_t ld_clean, int64_t ld_est, int32_t fs, void* workspace,
                          int64_t ws_bytes, double* out, void* stream) {
  using namespace stoi;
  CLSKD_CHECK_ARG(clean && est && workspace && out, "stoi: null pointer");
  CLSKD_CHECK_SHAPE(B >= 1 && L >= 1 && fs >= 1, "stoi: shape");
  const StoiPlan p = stoi_plan(B, L, fs);
  CLSKD_CHECK_ARG(ws_bytes >= p.bytes, "stoi: workspace of %lld bytes, need %lld",
                  (long long)ws_bytes, (long long)p.bytes);
  CLSKD_CHECK_SHAPE(p.nfr >= 1 && p.nfr <= 6144,
                    "stoi: %d energy frames at 10 kHz (need 1 .. 6144, i.e. <= 78 s)", p.nfr);
  const hipStream_t st = as_stream(stream);
  unsigned char* ws = reinterpret_cast<unsigned char*>(workspace);
  double* hp = reinterpret_cast<double*>(ws + p.off_h);
  double* xr = reinterpret_cast<double*>(ws + p.off_x);
  int* kept = reinterpret_cast<int*>(ws + p.off_kept);
  int* nk = reinterpret_cast<int*>(ws + p.off_nkept);
  double* sil = reinterpret_cast<double*>(ws + p.off_sil);
  double* tob = reinterpret_cast<double*>(ws + p.off_tob);
  const int lenhp = p.pre_pad + 2 * p.half_len + 1;
  if (!(p.up == 1 && p.down == 1))
    hipLaunchKernelGGL(stoi_filter_kernel, dim3(1), dim3(1024), 0, st, p.half_len, p.up, p.pre_pad,
                       p.stop, p.beta, hp);
  hipLaunchKernelGGL(stoi_resample_kernel, dim3((unsigned)cdiv(p.n_out, 256), B, 2), dim3(256), 0,
                     st, clean, est, ld_clean, ld_est, L, p.n_out, p.up, p.down, p.pre_remove,
                     lenhp, (const double*)hp, xr);
  hipLaunchKernelGGL(stoi_mask_kernel, dim3(B), dim3(1024), (size_t)p.nfr * 8, st,
                     (const double*)xr, p.n_out, p.nfr, kept, nk);
  hipLaunchKernelGGL(stoi_ola_kernel, dim3((unsigned)cdiv(p.ls_max, 256), B, 2), dim3(256), 0, st,
                     (const double*)xr, p.n_out, (const int*)kept, p.nfr, (const int*)nk,
                     p.ls_max, sil);
  BandArgs ba;
  int kmax = 0;
  for (int b = 0; b < NBAND; ++b) {
    ba.lo[b] = p.band_lo[b];
    ba.hi[b] = p.band_hi[b];
    kmax = p.band_hi[b] > kmax ? p.band_hi[b] : kmax;
  }
  hipLaunchKernelGGL(stoi_band_kernel, dim3(p.nst_max, B, 2), dim3(256), 0, st,
                     (const double*)sil, p.ls_max, (const int*)nk, p.nst_max, ba, kmax, tob);
  hipLaunchKernelGGL(stoi_corr_kernel, dim3(B), dim3(256), 0, st, (const double*)tob,
                     (const int*)nk, p.nst_max, out);
  CLSKD_LAUNCH_CHECK("stoi");
  return CLSKD_OK;
}

extern "C" int clskd_sisdr_f64(const float* ref, const float* est, int32_t rows, int32_t L,
                               int64_t ld_ref, int64_t ld_est, double* out, void* stream) {
  CLSKD_CHECK_ARG(ref && est && out, "sisdr_f64: null pointer");
  CLSKD_CHECK_SHAPE(rows >= 1 && L >= 1, "sisdr_f64: shape");
  hipLaunchKernelGGL(sisdr_rows_f64_kernel, dim3(rows), dim3(256), 0, as_stream(stream), ref, est, L,
                     ld_ref, ld_est, out);
  CLSKD_LAUNCH_CHECK("sisdr_f64");
  return CLSKD_OK;
}
