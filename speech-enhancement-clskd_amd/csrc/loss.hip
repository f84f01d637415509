// CLSKD losses: batched Gram (SPKD, framework.py:150-172), MRSTFT log-magnitude / spectral
// convergence reductions (framework.py:16-101) and SI-SNR (tools_for_loss.py:22-47).
//
// Gram: memory-bound (arithmetic intensity = B FLOP/byte).  One launch serves every tap of the
// step: the host flattens all taps into "slabs" (chunk positions of one tap); each workgroup
// streams 16 (or 32) batch rows of its slab with 16-B loads straight into the
// v_mfma_f32_16x16x4_f32 operand layout (lane l: row l&15, 4 consecutive elements at 4*(l>>4));
// A and B operands are the same register, so one load feeds both.  Partial 32x32 slabs are
// summed in a fixed order by the finalize kernel: bitwise reproducible, no atomics.
#include <vector>

#include "common.h"

namespace clskd {

typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));

// Kernel-argument job tables: no device-side descriptor upload, so a step is graph-capturable
// and the host never waits on a copy.
struct GramJobsArg {
  clskd_gram_job j[CLSKD_GRAM_MAX_JOBS];
  int32_t n;      // jobs in this launch
  int32_t slab0;  // absolute slab index of blockIdx.x == 0
};

// Per pair: the student / teacher job's first slab (any slab buffer: gram launches of one step
// may run on different streams into different buffers) and slab count.
struct SpkdPairsArg {
  const float* s_ptr[CLSKD_SPKD_MAX_PAIRS];
  const float* t_ptr[CLSKD_SPKD_MAX_PAIRS];
  int32_t s_n[CLSKD_SPKD_MAX_PAIRS], t_n[CLSKD_SPKD_MAX_PAIRS];
  int32_t pair0;  // absolute pair index of blockIdx.x == 0
};

// Optional folded BatchNorm (job.scale/shift): the job's per-channel affine, staged in LDS by
// the workgroup (aff[0][ch] = scale, aff[1][ch] = shift, ch in [0, Ctot)).
constexpr int GRAM_AFF_MAX = 1024;

// Slab-relative element e -> row-relative offset (p - p0) * Ctot + c0 + c with p - p0 = e / Cs
// and c = e % Cs by a 32-bit multiply-high (exact for e * Cs < 2^32: the kernel only asks for
// e < nel = (p1 - p0) * Cs <= max(16384, Cs) elements per row per slab, and a slab of one
// position needs no split at all); no 64-bit division per load.
struct ESplit {
  uint32_t cs, magic, ctot, c0;
  bool one;  // the slab holds one position: e < Cs
};
__device__ __forceinline__ ESplit make_split(const clskd_gram_job& j, int64_t p0, int64_t p1) {
  ESplit s;
  s.cs = (uint32_t)j.Cs;
  s.magic = 0xFFFFFFFFu / s.cs + 1u;
  s.ctot = (uint32_t)j.Ctot;
  s.c0 = (uint32_t)j.c0;
  s.one = p1 - p0 <= 1;
  return s;
}
__device__ __forceinline__ void split_e(uint32_t e, const ESplit& s, uint32_t& pr, uint32_t& c) {
  if (s.one) {
    pr = 0;
    c = e;
  } else {
    pr = __umulhi(e, s.magic);
    c = e - pr * s.cs;
  }
}

// Element transform of a job (MODE): 0 = as stored; 1 = folded BatchNorm affine; 2 = affine +
// PReLU(alpha) — both with the fmaf + compare + storage rounding of clskd_bn_apply, so a Gram
// over the transformed elements is bitwise a Gram over the applied tensor.  OUT: the transformed
// elements are also written back to job.out at the same offset (the fused apply pass).
struct GramXf {
  const float (*aff)[GRAM_AFF_MAX];
  float alpha;
};

template <int MODE>
__device__ __forceinline__ float gram_xf(float x, float sc, float sh, float a) {
  if constexpr (MODE == 0) {
    return x;
  } else {
    const float t = fmaf(x, sc, sh);
    if constexpr (MODE == 2) return t >= 0.f ? t : a * t;
    return t;
  }
}

// Slab-relative element e -> element offset of the job's row (rowbase) and the channel c of
// its first element.
__device__ __forceinline__ int64_t elem_off(const ESplit& sp, int64_t rowbase, uint32_t e,
                                            uint32_t& c) {
  uint32_t pr;
  split_e(e, sp, pr, c);
  return rowbase + (int64_t)((uint64_t)pr * sp.ctot + c);
}

// Loads of a batch are all issued before any transform or store: a store issued between two
// loads would be waited for with the later load (vmcnt counts both), and the output may alias
// the input (in-place apply).
template <int MODE>
__device__ __forceinline__ f32x4 xf4_f32(f32x4 v, uint32_t c, const ESplit& sp, const GramXf& xf) {
  if constexpr (MODE != 0) {
    const f32x4 sc = *reinterpret_cast<const f32x4*>(&xf.aff[0][sp.c0 + c]);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(&xf.aff[1][sp.c0 + c]);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = gram_xf<MODE>(v[i], sc[i], sh[i], xf.alpha);
  }
  return v;
}

template <int MODE>
__device__ __forceinline__ bf16x8g xf8_bf16(bf16x8g v, uint32_t c, const ESplit& sp,
                                            const GramXf& xf) {
  if constexpr (MODE != 0) {  // the same fmaf (+ PReLU) + RNE rounding as clskd_bn_apply
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(&xf.aff[0][sp.c0 + c]);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(&xf.aff[0][sp.c0 + c + 4]);
    const f32x4 h0 = *reinterpret_cast<const f32x4*>(&xf.aff[1][sp.c0 + c]);
    const f32x4 h1 = *reinterpret_cast<const f32x4*>(&xf.aff[1][sp.c0 + c + 4]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = (__bf16)gram_xf<MODE>((float)v[i], s0[i], h0[i], xf.alpha);
      v[i + 4] = (__bf16)gram_xf<MODE>((float)v[i + 4], s1[i], h1[i], xf.alpha);
    }
  }
  return v;
}

// Fixed-order reduction of the 4 waves' 16x16 accumulators into the 32x32 slab.
// C layout (16x16 MFMA): col = l&15, row = 4*(l>>4)+i.
__device__ __forceinline__ void gram_store_slab(float (*red)[3][256], const f32x4& acc00,
                                                const f32x4& acc01, const f32x4& acc11,
                                                float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[wave][0][lane * 4 + i] = acc00[i];
    red[wave][1][lane * 4 + i] = acc01[i];
    red[wave][2][lane * 4 + i] = acc11[i];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 1024; idx += 256) {
    const int row = idx >> 5, col = idx & 31;
    const int I = row >> 4, J = col >> 4;
    // the lower-left block is the transpose of the upper-right one
    const bool lower = (I == 1 && J == 0);
    const int t = lower ? 1 : ((I == 0 && J == 0) ? 0 : (I == 0 ? 1 : 2));
    const int rr = lower ? (col & 15) : (row & 15), cc = lower ? (row & 15) : (col & 15);
    const int l = cc + 16 * (rr >> 2), i = rr & 3;
    out[idx] = red[0][t][l * 4 + i] + red[1][t][l * 4 + i] + red[2][t][l * 4 + i] +
               red[3][t][l * 4 + i];
  }
}

// store target of lanes without an element (16 B per lane)
__device__ __attribute__((aligned(256))) unsigned char g_gram_sink[64 * 16];

template <int NB, int MODE, bool OUT>
__device__ __forceinline__ void gram_accumulate(const clskd_gram_job& j, int B, int64_t nel,
                                                int64_t p0, int64_t p1, const GramXf& xf,
                                                f32x4& acc00, f32x4& acc01, f32x4& acc11) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const ESplit sp = make_split(j, p0, p1);
  // rows past B read row 0 (valid memory) and are zeroed: the MFMA sees zeros for them
  const bool in0 = r < B, in1 = r + 16 < B;
  const int64_t rb0 = (int64_t)(in0 ? r : 0) * j.sB + p0 * j.Ctot + j.c0;
  const int64_t rb1 = (int64_t)(in1 ? r + 16 : 0) * j.sB + p0 * j.Ctot + j.c0;
  const uint32_t n32 = (uint32_t)nel;
  if (j.dtype == CLSKD_BF16) {
    // 16x16x32 bf16 MFMA: lane (r, g) holds row r, 8 consecutive k; A and B are the same
    // register (G = Z Z^T), so one 16-B load feeds both operands.  64 B per row per load.
    constexpr int U = 8;
    const __bf16* src = reinterpret_cast<const __bf16*>(j.ptr);
    __bf16* dst = reinterpret_cast<__bf16*>(j.out);
    for (uint32_t base = (uint32_t)wave * 32; base < n32; base += 128 * U) {
      bf16x8g v0[U], v1[U];
      int64_t o0[U], o1[U];
      uint32_t c0[U], c1[U];
      bool k0[U], k1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = base + (uint32_t)u * 128 + 8 * g;
        const bool ok = e < n32;
        k0[u] = ok && in0;
        o0[u] = elem_off(sp, rb0, e, c0[u]);
        v0[u] = k0[u] ? *reinterpret_cast<const bf16x8g*>(src + o0[u]) : bf16x8g{};
        if constexpr (NB == 2) {
          k1[u] = ok && in1;
          o1[u] = elem_off(sp, rb1, e, c1[u]);
          v1[u] = k1[u] ? *reinterpret_cast<const bf16x8g*>(src + o1[u]) : bf16x8g{};
        }
      }
      // transforms, then the stores back to back: a store followed by the next transform let the
      // compiler reuse the store's address registers behind a vmcnt(0) (one store round trip
      // per 16-B row piece); rows / elements that were not loaded stay zero for the MFMA
      if constexpr (MODE != 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (k0[u]) v0[u] = xf8_bf16<MODE>(v0[u], c0[u], sp, xf);
          if constexpr (NB == 2)
            if (k1[u]) v1[u] = xf8_bf16<MODE>(v1[u], c1[u], sp, xf);
        }
        if constexpr (OUT) {
          // straight-line stores: lanes without an element write their lane's slot of a sink
          // page (an exec-masked store per piece compiled to a branch + vmcnt(0) each)
          __bf16* sink = reinterpret_cast<__bf16*>(g_gram_sink) + lane * 8;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            *reinterpret_cast<bf16x8g*>(k0[u] ? dst + o0[u] : sink) = v0[u];
            if constexpr (NB == 2) *reinterpret_cast<bf16x8g*>(k1[u] ? dst + o1[u] : sink) = v1[u];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v0[u], v0[u], acc00, 0, 0, 0);
        if constexpr (NB == 2) {
          acc01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v0[u], v1[u], acc01, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v1[u], v1[u], acc11, 0, 0, 0);
        }
      }
    }
  } else {
    // fp32: 16x16x4 f32 MFMA, lane (r, g) holds row r, 4 consecutive elements per load
    constexpr int U = 4;
    const float* src = reinterpret_cast<const float*>(j.ptr);
    float* dst = reinterpret_cast<float*>(j.out);
    for (uint32_t base = (uint32_t)wave * 16; base < n32; base += 64 * U) {
      f32x4 v0[U], v1[U];
      int64_t o0[U], o1[U];
      uint32_t c0[U], c1[U];
      bool k0[U], k1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = base + (uint32_t)u * 64 + 4 * g;
        const bool ok = e < n32;
        k0[u] = ok && in0;
        o0[u] = elem_off(sp, rb0, e, c0[u]);
        v0[u] = k0[u] ? *reinterpret_cast<const f32x4*>(src + o0[u]) : f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (NB == 2) {
          k1[u] = ok && in1;
          o1[u] = elem_off(sp, rb1, e, c1[u]);
          v1[u] = k1[u] ? *reinterpret_cast<const f32x4*>(src + o1[u]) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if constexpr (MODE != 0) {  // transforms, then the stores back to back (as above)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (k0[u]) v0[u] = xf4_f32<MODE>(v0[u], c0[u], sp, xf);
          if constexpr (NB == 2)
            if (k1[u]) v1[u] = xf4_f32<MODE>(v1[u], c1[u], sp, xf);
        }
        if constexpr (OUT) {
          float* sink = reinterpret_cast<float*>(g_gram_sink) + lane * 4;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            *reinterpret_cast<f32x4*>(k0[u] ? dst + o0[u] : sink) = v0[u];
            if constexpr (NB == 2) *reinterpret_cast<f32x4*>(k1[u] ? dst + o1[u] : sink) = v1[u];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          acc00 = __builtin_amdgcn_mfma_f32_16x16x4f32(v0[u][qq], v0[u][qq], acc00, 0, 0, 0);
          if constexpr (NB == 2) {
            acc01 = __builtin_amdgcn_mfma_f32_16x16x4f32(v0[u][qq], v1[u][qq], acc01, 0, 0, 0);
            acc11 = __builtin_amdgcn_mfma_f32_16x16x4f32(v1[u][qq], v1[u][qq], acc11, 0, 0, 0);
          }
        }
      }
    }
  }
}

template <int NB>  // row blocks of 16: B <= 16*NB
__global__ __launch_bounds__(256) void gram_partial_kernel(const GramJobsArg jobs, int B,
                                                           float* __restrict__ slabs) {
  const int slab = jobs.slab0 + blockIdx.x;
  // uniform scan of the (<= 32) kernel-argument jobs for the one owning this slab
  int q = 0;
  for (int k = 1; k < jobs.n; ++k)
    if (slab >= jobs.j[k].first_slab) q = k;
  const clskd_gram_job j = jobs.j[q];
  const int si = slab - j.first_slab;
  const int64_t p0 = (int64_t)si * j.chunk;
  const int64_t p1 = min(j.P, p0 + j.chunk);
  const int64_t nel = (p1 - p0) * j.Cs;  // elements per row in this slab
  f32x4 acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  __shared__ __attribute__((aligned(16))) float aff[2][GRAM_AFF_MAX];
  GramXf xf{aff, j.alpha ? j.alpha[0] : 0.f};
  if (j.scale) {  // uniform per workgroup
    for (int c = threadIdx.x; c < j.Ctot; c += 256) {
      aff[0][c] = j.scale[c];
      aff[1][c] = j.shift[c];
    }
    __syncthreads();
    if (j.out) {
      if (j.alpha) gram_accumulate<NB, 2, true>(j, B, nel, p0, p1, xf, acc00, acc01, acc11);
      else gram_accumulate<NB, 1, true>(j, B, nel, p0, p1, xf, acc00, acc01, acc11);
    } else {
      gram_accumulate<NB, 1, false>(j, B, nel, p0, p1, xf, acc00, acc01, acc11);
    }
  } else {
    gram_accumulate<NB, 0, false>(j, B, nel, p0, p1, xf, acc00, acc01, acc11);
  }
  __shared__ float red[4][3][256];
  gram_store_slab(red, acc00, acc01, acc11, slabs + (int64_t)slab * 1024);
}

// One block per pair: Gs = sum of the student job's slabs, Gt likewise, L1-normalise rows,
// loss = ||Gt - Gs||_F^2 (/ B^2).  1024 threads: the B*B Gram entries x NPH slab phases, each
// thread summing every NPH-th slab with four independent fp64 accumulators (many loads in
// flight), then the phases combined in a fixed order: bitwise reproducible.  B <= 32.
constexpr int FIN_THREADS = 1024;

__device__ __forceinline__ double sum_slabs(const float* __restrict__ base, int n, int e, int ph,
                                            int nph) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int q = ph;
  for (; q + 3 * nph < n; q += 4 * nph) {
    a0 += (double)base[(int64_t)q * 1024 + e];
    a1 += (double)base[(int64_t)(q + nph) * 1024 + e];
    a2 += (double)base[(int64_t)(q + 2 * nph) * 1024 + e];
    a3 += (double)base[(int64_t)(q + 3 * nph) * 1024 + e];
  }
  for (; q < n; q += nph) a0 += (double)base[(int64_t)q * 1024 + e];
  return (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(FIN_THREADS) void spkd_finalize_kernel(const SpkdPairsArg pa, int B,
                                                                    int batchmean,
                                                                    float* grams_s, float* grams_t,
                                                                    float* losses) {
  const int lp = blockIdx.x;
  const int pr = pa.pair0 + lp;
  __shared__ double Ps[FIN_THREADS], Pt[FIN_THREADS];
  __shared__ double Gs[32 * 32], Gt[32 * 32];
  __shared__ double rs[32], rt[32];
  __shared__ double red[FIN_THREADS / 64];
  const int tid = threadIdx.x;
  const int E = B * B;
  const int nph = FIN_THREADS / E;  // >= 1 for B <= 32
  const int e = tid % E, ph = tid / E;
  double s = 0.0, t = 0.0;
  if (ph < nph) {
    const int slot = (e / B) * 32 + (e % B);  // slab layout [32][32]
    s = sum_slabs(pa.s_ptr[lp], pa.s_n[lp], slot, ph, nph);
    t = sum_slabs(pa.t_ptr[lp], pa.t_n[lp], slot, ph, nph);
  }
  Ps[tid] = s;
  Pt[tid] = t;
  __syncthreads();
  if (tid < E) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < nph; ++k) {
      a += Ps[k * E + tid];
      b += Pt[k * E + tid];
    }
    Gs[tid] = a;
    Gt[tid] = b;
  }
  __syncthreads();
  if (tid < B) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < B; ++k) {
      a += fabs(Gs[tid * B + k]);
      b += fabs(Gt[tid * B + k]);
    }
    rs[tid] = a > 1e-12 ? a : 1e-12;
    rt[tid] = b > 1e-12 ? b : 1e-12;
  }
  __syncthreads();
  double acc = 0.0;
  if (tid < E) {
    const int i = tid / B;
    const float gs = (float)(Gs[tid] / rs[i]);
    const float gt = (float)(Gt[tid] / rt[i]);
    if (grams_s) grams_s[(int64_t)pr * E + tid] = gs;
    if (grams_t) grams_t[(int64_t)pr * E + tid] = gt;
    const double dlt = (double)gt - (double)gs;
    acc = dlt * dlt;
  }
  // fixed-order block reduction: wave sums by DPP-free shuffles, then the 16 wave partials
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    double tot = 0.0;
    for (int w = 0; w < FIN_THREADS / 64; ++w) tot += red[w];
    losses[pr] = (float)(batchmean ? tot / ((double)B * B) : tot);
  }
}

// MRSTFT partials: per block {sum (Y-X)^2, sum Y^2, sum |log Y - log X|} over its elements.
__global__ __launch_bounds__(256) void stft_mag_loss_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ Y,
                                                            int64_t rows, int ld, int nb,
                                                            double* __restrict__ partial) {
  const int64_t total = rows * nb;
  double a = 0, b = 0, c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / nb;
    const int f = (int)(i - r * nb);
    const float xr = X[r * ld + f], xi = X[r * ld + nb + f];
    const float yr = Y[r * ld + f], yi = Y[r * ld + nb + f];
    const float xm = sqrtf(fmaxf(xr * xr + xi * xi, 1e-7f));
    const float ym = sqrtf(fmaxf(yr * yr + yi * yi, 1e-7f));
    const float d = ym - xm;
    a += (double)d * d;
    b += (double)ym * ym;
    c += fabs((double)logf(ym) - (double)logf(xm));
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  c = wave_sum_d(c);
  __shared__ double red[4][3];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = a;
    red[w][1] = b;
    red[w][2] = c;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    partial[blockIdx.x * 3 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// out[0] = factor_sc * sqrt(sum (Y-X)^2) / sqrt(sum Y^2) ; out[1] = factor_mag * sum|..| / count
// 64 threads: lane l sums partials l, l+64, ... (fixed order), then a fixed xor-tree.
__global__ __launch_bounds__(64) void stft_loss_finalize_kernel(const double* partial, int nblk,
                                                               int64_t count, float factor_sc,
                                                               float factor_mag, int accumulate,
                                                               float* out) {
  double a = 0, b = 0, c = 0;
  for (int i = threadIdx.x; i < nblk; i += 64) {
    a += partial[i * 3];
    b += partial[i * 3 + 1];
    c += partial[i * 3 + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if (threadIdx.x != 0) return;
  const float sc = (float)(factor_sc * (sqrt(a) / sqrt(b)));
  const float mag = (float)(factor_mag * (c / (double)count));
  out[0] = accumulate ? out[0] + sc : sc;
  out[1] = accumulate ? out[1] + mag : mag;
}

// SI-SNR per row, two passes over the row (tools_for_loss.py:37-47, eps as given).
__global__ __launch_bounds__(256) void sisnr_rows_kernel(const float* __restrict__ s1,
                                                         const float* __restrict__ s2, int L,
                                                         int64_t ld1, int64_t ld2, float eps,
                                                         float* __restrict__ out) {
  const int row = blockIdx.x;
  const float* a = s1 + row * ld1;
  const float* b = s2 + row * ld2;
  __shared__ double red[4][2];
  __shared__ float alpha_s;
  double d12 = 0, d22 = 0;
  for (int i = threadIdx.x; i < L; i += 256) {
    d12 += (double)a[i] * b[i];
    d22 += (double)b[i] * b[i];
  }
  d12 = wave_sum_d(d12);
  d22 = wave_sum_d(d22);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = d12;
    red[w][1] = d22;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double s12 = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    const double s22 = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    alpha_s = (float)s12 / ((float)s22 + eps);
  }
  __syncthreads();
  const float alpha = alpha_s;
  double tt = 0, ee = 0;
  for (int i = threadIdx.x; i < L; i += 256) {
    const float st = alpha * b[i];
    const float e = a[i] - st;
    tt += (double)st * st;
    ee += (double)e * e;
  }
  tt = wave_sum_d(tt);
  ee = wave_sum_d(ee);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = tt;
    red[w][1] = ee;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float T2 = (float)(red[0][0] + red[1][0] + red[2][0] + red[3][0]);
    const float E2 = (float)(red[0][1] + red[1][1] + red[2][1] + red[3][1]);
    out[row] = 10.f * log10f(T2 / (E2 + eps) + eps);
  }
}

__global__ void sum_f32_kernel(const float* a, int n, float scale, float* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0;
  for (int i = 0; i < n; ++i) s += a[i];
  out[0] = (float)(s * scale);
}


// ------------------------------------------------------------------------------------------
// SPKD backward (framework.py:150-172).  Per pair: recompute Gs / Gt from the slabs (same
// fixed-order sums as the finalize), then with n = G / max(||G_i||_1, 1e-12) row-wise,
//   dn = -2 * scale * inv * (n_t - n_s)         (inv = 1/B^2 for batchmean)
//   dG_ij = dn_ij / s_i - sign(G_ij) * (sum_k dn_ik G_ik) / s_i^2   (s_i > 1e-12)
// and M = dG + dG^T, so that dz = M z for G = z z^T.  M [pair][B][B] fp32.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(FIN_THREADS) void spkd_grad_kernel(const SpkdPairsArg pa, int B,
                                                                int batchmean, float scale,
                                                                float* __restrict__ mout) {
  const int lp = blockIdx.x;
  const int pr = pa.pair0 + lp;
  __shared__ double Ps[FIN_THREADS], Pt[FIN_THREADS];
  __shared__ double Gs[32 * 32], Gt[32 * 32], dG[32 * 32];
  __shared__ double rs[32], rt[32], dot[32];
  const int tid = threadIdx.x;
  const int E = B * B;
  const int nph = FIN_THREADS / E;
  const int e = tid % E, ph = tid / E;
  double sv = 0.0, tv = 0.0;
  if (ph < nph) {
    const int slot = (e / B) * 32 + (e % B);
    sv = sum_slabs(pa.s_ptr[lp], pa.s_n[lp], slot, ph, nph);
    tv = sum_slabs(pa.t_ptr[lp], pa.t_n[lp], slot, ph, nph);
  }
  Ps[tid] = sv;
  Pt[tid] = tv;
  __syncthreads();
  if (tid < E) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < nph; ++k) {
      a += Ps[k * E + tid];
      b += Pt[k * E + tid];
    }
    Gs[tid] = a;
    Gt[tid] = b;
  }
  __syncthreads();
  if (tid < B) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < B; ++k) {
      a += fabs(Gs[tid * B + k]);
      b += fabs(Gt[tid * B + k]);
    }
    rs[tid] = a;
    rt[tid] = b > 1e-12 ? b : 1e-12;
  }
  __syncthreads();
  const double inv = batchmean ? 1.0 / ((double)B * B) : 1.0;
  if (tid < E) {  // dn (kept in dG for now)
    const int i = tid / B;
    const double si = rs[i] > 1e-12 ? rs[i] : 1e-12;
    const double ns = Gs[tid] / si, nt = Gt[tid] / rt[i];
    dG[tid] = -2.0 * (double)scale * inv * (nt - ns);
  }
  __syncthreads();
  if (tid < B) {
    double a = 0.0;
    for (int k = 0; k < B; ++k) a += dG[tid * B + k] * Gs[tid * B + k];
    dot[tid] = a;
  }
  __syncthreads();
  double g = 0.0;
  if (tid < E) {
    const int i = tid / B;
    const double si = rs[i];
    if (si > 1e-12) {
      const double sg = Gs[tid] > 0 ? 1.0 : (Gs[tid] < 0 ? -1.0 : 0.0);
      g = dG[tid] / si - sg * dot[i] / (si * si);
    } else {
      g = dG[tid] / 1e-12;
    }
  }
  __syncthreads();
  if (tid < E) dG[tid] = g;
  __syncthreads();
  if (tid < E) {
    const int i = tid / B, j = tid % B;
    mout[(int64_t)pr * E + tid] = (float)(dG[i * B + j] + dG[j * B + i]);
  }
}

// dz[b] (+)= sum_j M[b][j] z_j over a job's elements; z read like the Gram (optional folded
// affine), dz written fp32 at out + b*o_sB + p*o_Ctot + o_c0 + c.  One thread per (p, 4 ch).
struct GramBwdJobsArg {
  clskd_gram_bwd_job j[CLSKD_GRAM_MAX_JOBS];
  int32_t blk0[CLSKD_GRAM_MAX_JOBS + 1];  // first block of each job
  int32_t n;
};

template <int BMAX>
__global__ __launch_bounds__(256) void gram_bwd_kernel(const GramBwdJobsArg a, int B) {
  int q = 0;
  for (int k = 1; k < a.n; ++k)
    if ((int)blockIdx.x >= a.blk0[k]) q = k;
  const clskd_gram_bwd_job& j = a.j[q];
  const float* __restrict__ Ms = j.coef;  // uniform reads: scalar loads, no LDS staging
  const int CQ = j.Cs / 4;
  const int64_t nq = j.P * CQ;
  const int64_t qi = (int64_t)(blockIdx.x - a.blk0[q]) * 256 + threadIdx.x;
  if (qi >= nq) return;
  const int64_t p = qi / CQ;
  const int c = (int)(qi - p * CQ) * 4;
  f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
  if (j.scale) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sc[i] = j.scale[j.c0 + c + i];
      sh[i] = j.shift[j.c0 + c + i];
    }
  }
  f32x4 z[BMAX];
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    z[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (b < B) {
      const int64_t off = (int64_t)b * j.sB + p * j.Ctot + j.c0 + c;
      f32x4 v;
      if (j.dtype == CLSKD_BF16) {
        typedef __bf16 bf16x4g __attribute__((ext_vector_type(4)));
        const bf16x4g w = *reinterpret_cast<const bf16x4g*>(reinterpret_cast<const __bf16*>(j.ptr) + off);
        v = f32x4{(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
        if (j.scale) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (float)(__bf16)fmaf(v[i], sc[i], sh[i]);
        }
      } else {
        v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(j.ptr) + off);
        if (j.scale) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = fmaf(v[i], sc[i], sh[i]);
        }
      }
      z[b] = v;
    }
  }
  for (int b = 0; b < B; ++b) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < BMAX; ++k) {
      if (k < B) {
        const float m = Ms[b * B + k];
        acc += m * z[k];
      }
    }
    float* o = j.out + (int64_t)b * j.o_sB + p * j.o_Ctot + j.o_c0 + c;
    if (j.accumulate) acc += *reinterpret_cast<const f32x4*>(o);
    *reinterpret_cast<f32x4*>(o) = acc;
  }
}
}  // namespace clskd

using namespace clskd;

static int validate_gram_jobs(const clskd_gram_job* jobs, int32_t njobs, int32_t B,
                              int32_t* total) {
  CLSKD_CHECK_ARG(jobs, "gram: null job array");
  CLSKD_CHECK_SHAPE(B >= 1 && B <= 32, "gram: batch %d must be in [1, 32]", B);
  CLSKD_CHECK_SHAPE(njobs >= 1, "gram: empty job list");
  int32_t next = 0;
  for (int k = 0; k < njobs; ++k) {
    const clskd_gram_job& j = jobs[k];
    CLSKD_CHECK_ARG(j.ptr, "gram: job %d has a null tensor", k);
    CLSKD_CHECK_SHAPE(j.dtype == CLSKD_F32 || j.dtype == CLSKD_BF16, "gram: job %d dtype", k);
    const int g = j.dtype == CLSKD_BF16 ? 8 : 4;
    CLSKD_CHECK_SHAPE(j.Cs > 0 && j.Cs % g == 0 && j.c0 % g == 0 && j.Ctot % g == 0 &&
                          j.sB % g == 0 && j.P > 0 && j.chunk > 0,
                      "gram: job %d geometry (Cs %d, c0 %d, Ctot %d) needs multiples of %d", k,
                      j.Cs, j.c0, j.Ctot, g);
    CLSKD_CHECK_SHAPE(j.chunk == 1 || (uint64_t)j.chunk * (uint64_t)j.Cs * (uint64_t)j.Cs < (1ull << 32),
                      "gram: job %d chunk %lld x Cs %d^2 must stay below 2^32", k, (long long)j.chunk, j.Cs);
    CLSKD_CHECK_ARG((j.scale == nullptr) == (j.shift == nullptr),
                    "gram: job %d scale and shift go together", k);
    CLSKD_CHECK_SHAPE(!j.scale || j.Ctot <= GRAM_AFF_MAX, "gram: job %d folded affine needs Ctot <= %d",
                      k, GRAM_AFF_MAX);
    CLSKD_CHECK_ARG(!j.alpha || j.scale, "gram: job %d PReLU alpha needs the folded affine", k);
    CLSKD_CHECK_ARG(!j.out || (j.scale && ((uintptr_t)j.out & 15) == 0),
                    "gram: job %d output needs the folded affine and 16-byte alignment", k);
    CLSKD_CHECK_SHAPE(j.first_slab == next && j.nslab == (int32_t)((j.P + j.chunk - 1) / j.chunk),
                      "gram: job %d slab range [%d, +%d) is not contiguous", k, j.first_slab,
                      j.nslab);
    next += j.nslab;
  }
  *total = next;
  return CLSKD_OK;
}

extern "C" int clskd_gram_partial(const clskd_gram_job* jobs, int32_t njobs, int32_t B,
                                  float* slabs, void* stream) {
  int32_t total = 0;
  const int rc = validate_gram_jobs(jobs, njobs, B, &total);
  if (rc != CLSKD_OK) return rc;
  CLSKD_CHECK_ARG(slabs, "gram_partial: null slab buffer");
  if (skip_kernel(SKIP_GRAM)) return CLSKD_OK;
  hipStream_t st = as_stream(stream);
  for (int k0 = 0; k0 < njobs; k0 += CLSKD_GRAM_MAX_JOBS) {
    GramJobsArg a;
    a.n = njobs - k0 < CLSKD_GRAM_MAX_JOBS ? njobs - k0 : CLSKD_GRAM_MAX_JOBS;
    for (int k = 0; k < a.n; ++k) a.j[k] = jobs[k0 + k];
    for (int k = a.n; k < CLSKD_GRAM_MAX_JOBS; ++k) a.j[k] = jobs[k0];
    a.slab0 = a.j[0].first_slab;
    const int nb = a.j[a.n - 1].first_slab + a.j[a.n - 1].nslab - a.slab0;
    if (B <= 16)
      hipLaunchKernelGGL(gram_partial_kernel<1>, dim3(nb), dim3(256), 0, st, a, B, slabs);
    else
      hipLaunchKernelGGL(gram_partial_kernel<2>, dim3(nb), dim3(256), 0, st, a, B, slabs);
    CLSKD_LAUNCH_CHECK("gram_partial");
  }
  return CLSKD_OK;
}

static int launch_spkd_finalize(const float* const* s_ptr, const int32_t* s_n,
                                const float* const* t_ptr, const int32_t* t_n, int32_t npairs,
                                int32_t B, int32_t batchmean, float* grams_s, float* grams_t,
                                float* losses, hipStream_t st) {
  for (int p0 = 0; p0 < npairs; p0 += CLSKD_SPKD_MAX_PAIRS) {
    SpkdPairsArg a;
    const int n = npairs - p0 < CLSKD_SPKD_MAX_PAIRS ? npairs - p0 : CLSKD_SPKD_MAX_PAIRS;
    for (int k = 0; k < CLSKD_SPKD_MAX_PAIRS; ++k) {
      const int q = k < n ? p0 + k : p0;
      a.s_ptr[k] = s_ptr[q];
      a.t_ptr[k] = t_ptr[q];
      a.s_n[k] = s_n[q];
      a.t_n[k] = t_n[q];
    }
    a.pair0 = p0;
    hipLaunchKernelGGL(spkd_finalize_kernel, dim3(n), dim3(FIN_THREADS), 0, st, a, B, batchmean,
                       grams_s, grams_t, losses);
    CLSKD_LAUNCH_CHECK("spkd_finalize");
  }
  return CLSKD_OK;
}

extern "C" int clskd_spkd_finalize(const clskd_gram_job* jobs, int32_t njobs, const int32_t* pairs,
                                   int32_t npairs, int32_t B, int32_t batchmean, const float* slabs,
                                   float* grams_s, float* grams_t, float* losses, void* stream) {
  int32_t total = 0;
  const int rc = validate_gram_jobs(jobs, njobs, B, &total);
  if (rc != CLSKD_OK) return rc;
  CLSKD_CHECK_ARG(pairs && slabs && losses, "spkd_finalize: null pointer");
  CLSKD_CHECK_SHAPE(npairs >= 1, "spkd_finalize: no pairs");
  std::vector<const float*> sp(npairs), tp(npairs);
  std::vector<int32_t> sn(npairs), tn(npairs);
  for (int i = 0; i < npairs; ++i) {
    const int s = pairs[2 * i], t = pairs[2 * i + 1];
    CLSKD_CHECK_SHAPE(s >= 0 && s < njobs && t >= 0 && t < njobs,
                      "spkd_finalize: pair %d names a job outside [0, %d)", i, njobs);
    sp[i] = slabs + (int64_t)jobs[s].first_slab * 1024;
    tp[i] = slabs + (int64_t)jobs[t].first_slab * 1024;
    sn[i] = jobs[s].nslab;
    tn[i] = jobs[t].nslab;
  }
  return launch_spkd_finalize(sp.data(), sn.data(), tp.data(), tn.data(), npairs, B, batchmean,
                              grams_s, grams_t, losses, as_stream(stream));
}

extern "C" int clskd_spkd_finalize_ranges(const float* const* s_slabs, const int32_t* s_nslab,
                                          const float* const* t_slabs, const int32_t* t_nslab,
                                          int32_t npairs, int32_t B, int32_t batchmean,
                                          float* grams_s, float* grams_t, float* losses,
                                          void* stream) {
  CLSKD_CHECK_ARG(s_slabs && s_nslab && t_slabs && t_nslab && losses,
                  "spkd_finalize_ranges: null pointer");
  CLSKD_CHECK_SHAPE(B >= 1 && B <= 32, "spkd_finalize_ranges: batch %d must be in [1, 32]", B);
  CLSKD_CHECK_SHAPE(npairs >= 1, "spkd_finalize_ranges: no pairs");
  for (int i = 0; i < npairs; ++i)
    CLSKD_CHECK_ARG(s_slabs[i] && t_slabs[i] && s_nslab[i] >= 1 && t_nslab[i] >= 1,
                    "spkd_finalize_ranges: pair %d has an empty slab range", i);
  return launch_spkd_finalize(s_slabs, s_nslab, t_slabs, t_nslab, npairs, B, batchmean, grams_s,
                              grams_t, losses, as_stream(stream));
}

extern "C" int clskd_stft_mag_loss(const float* X, const float* Y, int64_t rows, int32_t ld,
                                   int32_t nbins, double* acc, void* stream) {
  // acc: [256][3] partials (caller-owned); finalize with clskd_stft_loss_finalize
  CLSKD_CHECK_ARG(X && Y && acc, "stft_mag_loss: null pointer");
  CLSKD_CHECK_SHAPE(rows > 0 && ld >= 2 * nbins, "stft_mag_loss: shape");
  hipLaunchKernelGGL(stft_mag_loss_kernel, dim3(256), dim3(256), 0, as_stream(stream), X, Y, rows,
                     ld, nbins, acc);
  CLSKD_LAUNCH_CHECK("stft_mag_loss");
  return CLSKD_OK;
}

extern "C" int clskd_stft_loss_finalize(const double* acc, int64_t count, float factor_sc,
                                        float factor_mag, int32_t accumulate, float* out2,
                                        void* stream) {
  CLSKD_CHECK_ARG(acc && out2, "stft_loss_finalize: null pointer");
  hipLaunchKernelGGL(stft_loss_finalize_kernel, dim3(1), dim3(64), 0, as_stream(stream), acc, 256,
                     count, factor_sc, factor_mag, accumulate, out2);
  CLSKD_LAUNCH_CHECK("stft_loss_finalize");
  return CLSKD_OK;
}

extern "C" int clskd_sisnr_rows(const float* s1, const float* s2, int32_t rows, int32_t L,
                                int64_t ld1, int64_t ld2, float eps, float* out, void* stream) {
  CLSKD_CHECK_ARG(s1 && s2 && out, "sisnr: null pointer");
  CLSKD_CHECK_SHAPE(rows >= 1 && L >= 1, "sisnr: shape");
  hipLaunchKernelGGL(sisnr_rows_kernel, dim3(rows), dim3(256), 0, as_stream(stream), s1, s2, L, ld1,
                     ld2, eps, out);
  CLSKD_LAUNCH_CHECK("sisnr_rows");
  return CLSKD_OK;
}

extern "C" int clskd_sum_f32(const float* a, int32_t n, float scale, float* out, void* stream) {
  CLSKD_CHECK_ARG(a && out && n >= 1, "sum_f32: bad args");
  hipLaunchKernelGGL(sum_f32_kernel, dim3(1), dim3(64), 0, as_stream(stream), a, n, scale, out);
  CLSKD_LAUNCH_CHECK("sum_f32");
  return CLSKD_OK;
}

extern "C" int clskd_spkd_grad_ranges(const float* const* s_slabs, const int32_t* s_nslab,
                                      const float* const* t_slabs, const int32_t* t_nslab,
                                      int32_t npairs, int32_t B, int32_t batchmean, float scale,
                                      float* coef, void* stream) {
  CLSKD_CHECK_ARG(s_slabs && s_nslab && t_slabs && t_nslab && coef, "spkd_grad: null pointer");
  CLSKD_CHECK_SHAPE(B >= 1 && B <= 32 && npairs >= 1, "spkd_grad: B=%d npairs=%d", B, npairs);
  hipStream_t st = as_stream(stream);
  for (int p0 = 0; p0 < npairs; p0 += CLSKD_SPKD_MAX_PAIRS) {
    SpkdPairsArg a;
    const int n = npairs - p0 < CLSKD_SPKD_MAX_PAIRS ? npairs - p0 : CLSKD_SPKD_MAX_PAIRS;
    for (int k = 0; k < CLSKD_SPKD_MAX_PAIRS; ++k) {
      const int q = k < n ? p0 + k : p0;
      CLSKD_CHECK_ARG(s_slabs[q] && t_slabs[q] && s_nslab[q] >= 1 && t_nslab[q] >= 1,
                      "spkd_grad: pair %d has an empty slab range", q);
      a.s_ptr[k] = s_slabs[q];
      a.t_ptr[k] = t_slabs[q];
      a.s_n[k] = s_nslab[q];
      a.t_n[k] = t_nslab[q];
    }
    a.pair0 = p0;
    hipLaunchKernelGGL(spkd_grad_kernel, dim3(n), dim3(FIN_THREADS), 0, st, a, B, batchmean, scale,
                       coef);
    CLSKD_LAUNCH_CHECK("spkd_grad");
  }
  return CLSKD_OK;
}

extern "C" int clskd_gram_bwd(const clskd_gram_bwd_job* jobs, int32_t njobs, int32_t B,
                              void* stream) {
  CLSKD_CHECK_ARG(jobs && njobs >= 1, "gram_bwd: no jobs");
  CLSKD_CHECK_SHAPE(B >= 1 && B <= 32, "gram_bwd: batch %d must be in [1, 32]", B);
  hipStream_t st = as_stream(stream);
  for (int k0 = 0; k0 < njobs; k0 += CLSKD_GRAM_MAX_JOBS) {
    GramBwdJobsArg a;
    a.n = njobs - k0 < CLSKD_GRAM_MAX_JOBS ? njobs - k0 : CLSKD_GRAM_MAX_JOBS;
    int32_t blk = 0;
    for (int k = 0; k < a.n; ++k) {
      const clskd_gram_bwd_job& j = jobs[k0 + k];
      CLSKD_CHECK_ARG(j.ptr && j.out && j.coef && j.P >= 1 && j.Cs % 4 == 0 && j.o_c0 % 4 == 0 &&
                          j.o_Ctot % 4 == 0 && j.o_sB % 4 == 0 &&
                          (j.dtype == CLSKD_F32 || j.dtype == CLSKD_BF16),
                      "gram_bwd: job %d malformed", k0 + k);
      a.j[k] = j;
      a.blk0[k] = blk;
      blk += (int32_t)cdiv(j.P * (j.Cs / 4), 256);
    }
    for (int k = a.n; k < CLSKD_GRAM_MAX_JOBS; ++k) {
      a.j[k] = jobs[k0];
      a.blk0[k] = blk;
    }
    a.blk0[CLSKD_GRAM_MAX_JOBS] = blk;
    if (B <= 16)
      hipLaunchKernelGGL(gram_bwd_kernel<16>, dim3(blk), dim3(256), 0, st, a, B);
    else
      hipLaunchKernelGGL(gram_bwd_kernel<32>, dim3(blk), dim3(256), 0, st, a, B);
    CLSKD_LAUNCH_CHECK("gram_bwd");
  }
  return CLSKD_OK;
}
