// ReviewKD ABF level with conv1 folded into its consumers (framework.py:176-222, mid = 64).
//
// The reference runs, per level, conv1 = Conv2d(Cin -> 64, 1x1) + train-mode BatchNorm2d, then
// (levels with att_conv) the attention fusion with the nearest-upsampled residual, then conv2.
// Materialising conv1's 64-channel output costs a write + read of 64 channels at the student
// tap's full resolution (up to B x 128 x T rows) for an op that computes only Cin <= 64 MACs
// per output.  Here conv1 never reaches HBM:
//
//  * BatchNorm statistics of x1 = W1 s come from the input's moments: for output channel n,
//      sum_n   = w_n . S1            (S1 = sum over rows of s,     Cin)
//      sumsq_n = w_n^T S2 w_n        (S2 = sum over rows of s s^T, Cin x Cin)
//    abf_moments_kernel: S1/S2 of its rows on fp32 MFMA (exact products, fp64 across chunks),
//    projected onto the 64 output channels in fp64 inside the block (the projection is linear,
//    so per-block projections sum exactly to the total's) -> {sum, sumsq} partials in the
//    layout of the conv engines' fused statistics, finalised by clskd_bn_compact/_finalize.
//  * abf_conv1_fuse_kernel recomputes x1 = W1 s per row in registers (fp32 FMAs in ascending k,
//    as conv_pointwise_kernel did), applies the BN affine, the attention fusion and writes only
//    the fused 64-channel map (and, for the training tape, optionally the raw x1).
// Deterministic: fixed reduction orders, no atomics.
#include <stdlib.h>

#include <algorithm>

#include "bnfold.h"
#include "common.h"

namespace clskd {

// Row geometry of a tap [B][F][T][C] at element strides (sB, sF, sT): the offset of row
// m = (b*F + f)*T + t.  Contiguous taps (the common case) are m*C; otherwise the (b, f, t) of
// a run's first row is found once (uniform: scalar unit) and the lanes step from it.
struct TapRows {
  int F, T, sB, sF, sT;
  bool contig;
  __device__ __forceinline__ void split(int m, int& b, int& f, int& t) const {
    const int bf = m / T;
    t = m - bf * T;
    b = bf / F;
    f = bf - b * F;
  }
  // (b, f, t) of row m0 + r from those of m0 (r >= 0)
  __device__ __forceinline__ static void step(int F, int T, int r, int& b, int& f, int& t) {
    t += r;
    while (t >= T) {
      t -= T;
      if (++f == F) {
        f = 0;
        ++b;
      }
    }
  }
  __device__ __forceinline__ int off(int b, int f, int t) const { return b * sB + f * sF + t * sT; }
};

// ------------------------------------------------------------------------------------------
// moments: slab[blk] = { S1[C], S2[C][C] } (fp64) over rows [blk*rpb, (blk+1)*rpb)
// S2 = X^T X on v_mfma_f32_16x16x4_f32 (exact fp32 products): lane l holds X[row][16t + (l&15)]
// for channel tile t, at once the A operand (A[i][k] = X[k][i]) of the tile row and the B
// operand (B[k][j] = X[k][j]) of the tile column — no LDS, no shuffles.  C = 8 packs two rows
// per lane column group (lanes 0-7 row 2k, lanes 8-15 row 2k+1: the two diagonal 8x8 blocks of
// the 16x16 product are summed, the cross blocks ignored), 8 rows per MFMA.  Upper tile
// triangle only; four accumulator sets rotate (the 40-cycle dependent MFMA latency);
// accumulators flushed to fp64 per chunk.
// ------------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void abf_moments_kernel(const float* __restrict__ s,
                                                          TapRows g, int rows, int rpb,
                                                          const float* __restrict__ w1,
                                                          double* __restrict__ partial,
                                                          const BnFoldArgs fold) {
  constexpr int NT = C >= 16 ? C / 16 : 1;        // 16-channel tiles
  constexpr int NP = NT * (NT + 1) / 2;           // tiles with ti <= tj
  constexpr int RPG = C == 8 ? 8 : 4;             // rows per MFMA k-group
  constexpr int G = C == 64 ? 8 : 16;             // k-groups per chunk
  constexpr int NA = NP >= 4 ? 1 : 4;             // rotating accumulator sets
  constexpr int CH = RPG * G;                     // rows per chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15;
  // this lane's row within a k-group and its channel within a tile
  const int lrow = C == 8 ? 2 * (lane >> 4) + (col >> 3) : lane >> 4;
  const int lch = C == 8 ? (col & 7) : col;
  const int r0 = blockIdx.x * rpb;
  const int r1 = min(rows, r0 + rpb);
  double d2[NP][4], d1[NT];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int j = 0; j < 4; ++j) d2[p][j] = 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) d1[t] = 0.0;
  for (int c0 = r0 + wave * CH; c0 < r1; c0 += 4 * CH) {  // chunks dealt over the waves
    float x[G][NT];
    int b, f, t;
    if (!g.contig) {
      g.split(c0, b, f, t);  // uniform
      TapRows::step(g.F, g.T, lrow, b, f, t);
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int m = c0 + RPG * gi + lrow;
      const bool ok = m < r1;
      const float* row;
      if (g.contig) {
        row = s + (ok ? m : r0) * C;
      } else {
        row = s + (ok ? g.off(b, f, t) : g.off(0, 0, 0));
        TapRows::step(g.F, g.T, RPG, b, f, t);
      }
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) x[gi][ti] = ok ? row[16 * ti + lch] : 0.f;
    }
    f32x4 acc[NA][NP];
    float a1[NT];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int p = 0; p < NP; ++p) acc[a][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) a1[ti] = 0.f;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      int p = 0;
#pragma unroll
      for (int ti = 0; ti < NT; ++ti) {
        a1[ti] += x[gi][ti];
#pragma unroll
        for (int tj = ti; tj < NT; ++tj, ++p)
          acc[gi % NA][p] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(x[gi][ti], x[gi][tj], acc[gi % NA][p], 0, 0, 0);
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[0][p][j];
#pragma unroll
        for (int a = 1; a < NA; ++a) v += acc[a][p][j];
        d2[p][j] += (double)v;
      }
#pragma unroll
    for (int ti = 0; ti < NT; ++ti) d1[ti] += (double)a1[ti];
  }
  // S1: the lanes holding one channel (4 row lanes; C = 8: 8 row lanes), fixed order
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) {
    if (C == 8) d1[ti] += __shfl_xor(d1[ti], 8, 64);
    d1[ti] += __shfl_xor(d1[ti], 16, 64);
    d1[ti] += __shfl_xor(d1[ti], 32, 64);
  }
  // dense S2 [C][C + 2] + S1 (fp64) and W1 [64][C + 1] in LDS (padded rows: conflict-free);
  // the waves' partials are combined in a fixed order (wave 0 writes, waves 1..3 add in turn)
  constexpr int SP = C + 2;  // S2 row pitch (16-B aligned rows)
  __shared__ __attribute__((aligned(16))) double S[C * SP + C];
  __shared__ float wl[64 * (C + 1)];
  for (int e = tid; e < 64 * C; e += 256) wl[(e / C) * (C + 1) + e % C] = w1[e];
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
      int p = 0;
#pragma unroll
      for (int ti = 0; ti < NT; ++ti)
#pragma unroll
        for (int tj = ti; tj < NT; ++tj, ++p)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 16 * ti + 4 * (lane >> 4) + j, jj = 16 * tj + (lane & 15);  // C/D map
            if (C == 8) {  // two diagonal 8x8 blocks of the 16x16 tile, summed; cross blocks dropped
#pragma unroll
              for (int half = 0; half < 2; ++half) {
                if ((i >> 3) == half && (jj >> 3) == half) {
                  double& d = S[(i & 7) * SP + (jj & 7)];
                  d = (w == 0 && half == 0) ? d2[p][j] : d + d2[p][j];
                }
              }
            } else {
              double& d = S[i * SP + jj];
              d = w == 0 ? d2[p][j] : d + d2[p][j];
              if (ti != tj) {
                double& e = S[jj * SP + i];
                e = w == 0 ? d2[p][j] : e + d2[p][j];
              }
            }
          }
      if (lane < (C == 8 ? 8 : 16))
#pragma unroll
        for (int ti = 0; ti < NT; ++ti) {
          double& d = S[C * SP + 16 * ti + lane];
          d = w == 0 ? d1[ti] : d + d1[ti];
        }
    }
    __syncthreads();
  }
  // this block's statistics of x1 = W1 s: sum_n = w_n . S1, sumsq_n = w_n^T S2 w_n (an exact
  // split of the totals over blocks).  4 lanes per output channel, lane `part` owning the
  // column chunk j in [part*C/4, (part+1)*C/4) with its weights in registers; the lanes of a
  // wave read 4 distinct S2 row chunks (the 16 channels broadcast).
  constexpr int JC = C / 4;
  const int n = tid >> 2, part = tid & 3;
  const float* w = wl + n * (C + 1);
  float wj[JC];
#pragma unroll
  for (int jj = 0; jj < JC; ++jj) wj[jj] = w[part * JC + jj];
  double q = 0.0, sm = 0.0;
  for (int i = 0; i < C; ++i) {
    const double* Si = S + i * SP + part * JC;
    double row = 0.0;
#pragma unroll
    for (int jj = 0; jj < JC; ++jj) row += (double)wj[jj] * Si[jj];
    q += (double)w[i] * row;
  }
#pragma unroll
  for (int jj = 0; jj < JC; ++jj) sm += (double)wj[jj] * S[C * SP + part * JC + jj];
  q += __shfl_xor(q, 1, 4);
  q += __shfl_xor(q, 2, 4);
  sm += __shfl_xor(sm, 1, 4);
  sm += __shfl_xor(sm, 2, 4);
  if (fold.acc) {  // folded finalize (clskd_abf_bn1_fold): the block's 64 sums, then the ticket
    __shared__ double fin[64 * 2];
    __shared__ int flag;
    if (part == 0) {
      fin[n * 2] = sm;
      fin[n * 2 + 1] = q;
    }
    __syncthreads();
    bnfold_commit(fold, 64, [&](int c, double& S1, double& Q1) {
      S1 = fin[c * 2];
      Q1 = fin[c * 2 + 1];
    }, &flag, blockIdx.x, gridDim.x);
    return;
  }
  if (part == 0) {
    partial[((int64_t)blockIdx.x * 64 + n) * 2] = sm;
    partial[((int64_t)blockIdx.x * 64 + n) * 2 + 1] = q;
  }
}

// ------------------------------------------------------------------------------------------
// fused level: x1 = W1 s (fp32, ascending k), x = x1*scale + shift, [attention fusion with the
// nearest-upsampled residual], out = x (DT).  A wave pass covers 32 rows, 8 lanes per row
// (8 output channels = one 16-B bf16 chunk each), 4 rows per lane.  The pass's s rows are
// staged in a wave-private LDS slice by coalesced 16-B loads and its residual chunks loaded,
// both one pass ahead (register double buffer, residual kept packed); the FMAs run on
// broadcast LDS reads of s and W1^T.  Row indices step from the pass's first row (no per-lane
// divisions); BN and attention constants sit in LDS.
// ------------------------------------------------------------------------------------------
template <typename DT>
struct Chunk8;  // 8 channels of storage DT, packed as loaded
template <>
struct Chunk8<__bf16> {
  uint4 v;
  __device__ __forceinline__ void load(const __bf16* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { v = uint4{0u, 0u, 0u, 0u}; }
  __device__ __forceinline__ float get(int j) const {
    const unsigned u = (j >> 1) == 0 ? v.x : (j >> 1) == 1 ? v.y : (j >> 1) == 2 ? v.z : v.w;
    return __uint_as_float((j & 1) ? (u & 0xFFFF0000u) : (u << 16));
  }
};
template <>
struct Chunk8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = f32x4{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ float get(int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

template <typename DT>
__device__ __forceinline__ void store8(DT* p, const float (&v)[8]);
template <>
__device__ __forceinline__ void store8<float>(float* p, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
template <>
__device__ __forceinline__ void store8<__bf16>(__bf16* p, const float (&v)[8]) {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  b8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
  *reinterpret_cast<b8*>(p) = o;
}

template <int C, typename DT, bool FUSE>
__global__ __launch_bounds__(256) void abf_conv1_fuse_kernel(
    const float* __restrict__ s, TapRows g, int rows, const float* __restrict__ w1,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const DT* __restrict__ res, int Fr, int Tr, const float* __restrict__ aw,
    const float* __restrict__ ab, DT* __restrict__ out, DT* __restrict__ raw_out) {
  constexpr int C4 = C / 4;
  constexpr int RP = 32;                     // rows per wave pass
  constexpr int NQ = (RP * C4 + 63) / 64;    // staged float4 per lane
  __shared__ f32x4 wl[C][16];     // wl[k][q] = {w1[4q][k], w1[4q+1][k], w1[4q+2][k], w1[4q+3][k]}
  __shared__ f32x4 sl[4][RP][C4];  // per wave: the pass's rows of s
  __shared__ float cst[6][64];    // scale, shift, attention weights w0x, w0y, w1x, w1y
  const int tid = threadIdx.x;
  for (int e = tid; e < C * 16; e += 256) {
    const int k = e >> 4, q = e & 15;
    wl[k][q] = f32x4{w1[(4 * q) * C + k], w1[(4 * q + 1) * C + k], w1[(4 * q + 2) * C + k],
                     w1[(4 * q + 3) * C + k]};
  }
  if (tid < 64) {
    cst[0][tid] = scale[tid];
    cst[1][tid] = shift[tid];
  } else if (FUSE) {
    const int e = tid - 64;  // 192 threads: w0y, w1x, w1y; w0x below
    cst[3 + e / 64][e % 64] = aw[64 + e];
  }
  if (FUSE && tid < 64) cst[2][tid] = aw[tid];
  const int lane = tid & 63, wave = tid >> 6;
  const int sub = lane & 7, grp = lane >> 3;  // channels 8*sub..+7; rows grp + 8h
  const int c = sub * 8;
  float b0 = 0.f, b1 = 0.f;
  if constexpr (FUSE) {
    b0 = ab[0];
    b1 = ab[1];
  }
  __syncthreads();
  const int nunits = (rows + RP - 1) / RP;
  const int ustep = gridDim.x * 4;
  auto load_pass = [&](int u, f32x4 (&sv)[NQ], Chunk8<DT> (&yv)[4]) {
    const int mb = u * RP;
    int b0_ = 0, f0 = 0, t0 = 0;
    if (!g.contig || FUSE) g.split(mb, b0_, f0, t0);  // uniform
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = lane + 64 * i;
      const int r = q / C4, k4 = q % C4;
      sv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < RP * C4 && mb + r < rows) {
        int off;
        if (g.contig) {
          off = (mb + r) * C;
        } else {
          int b = b0_, f = f0, t = t0;
          TapRows::step(g.F, g.T, r, b, f, t);
          off = g.off(b, f, t);
        }
        sv[i] = *reinterpret_cast<const f32x4*>(s + off + 4 * k4);
      }
    }
    if constexpr (FUSE) {
      int b = b0_, f = f0, t = t0;
      TapRows::step(g.F, g.T, grp, b, f, t);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        yv[h].zero();
        if (mb + grp + 8 * h < rows) {
          const int fr = nearest_src(f, Fr, g.F), tr = nearest_src(t, Tr, g.T);
          yv[h].load(res + ((b * Fr + fr) * Tr + tr) * 64 + c);
        }
        TapRows::step(g.F, g.T, 8, b, f, t);
      }
    }
  };
  f32x4 sv[NQ];
  Chunk8<DT> yv[4];
  int u = blockIdx.x * 4 + wave;
  if (u < nunits) load_pass(u, sv, yv);
  for (; u < nunits; u += ustep) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = lane + 64 * i;
      if (q < RP * C4) sl[wave][q / C4][q % C4] = sv[i];
    }
    Chunk8<DT> ycur[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) ycur[h] = yv[h];
    if (u + ustep < nunits) load_pass(u + ustep, sv, yv);  // next pass's loads in flight
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float acc[4][8];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
#pragma unroll 2
    for (int k4 = 0; k4 < C4; ++k4) {
      f32x4 sr[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) sr[h] = sl[wave][grp + 8 * h][k4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const f32x4 wa = wl[4 * k4 + kk][2 * sub], wb = wl[4 * k4 + kk][2 * sub + 1];
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[h][j] = fmaf(sr[h][kk], wa[j], acc[h][j]);
            acc[h][4 + j] = fmaf(sr[h][kk], wb[j], acc[h][4 + j]);
          }
      }
    }
    const int mb = u * RP;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(acc[h][j], cst[0][c + j], cst[1][c + j]);
      if constexpr (FUSE) {
        float d0 = 0.f, d1 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float y = ycur[h].get(j);
          d0 += cst[2][c + j] * o[j] + cst[3][c + j] * y;
          d1 += cst[4][c + j] * o[j] + cst[5][c + j] * y;
        }
#pragma unroll
        for (int o2 = 4; o2 > 0; o2 >>= 1) {
          d0 += __shfl_xor(d0, o2, 8);
          d1 += __shfl_xor(d1, o2, 8);
        }
        const float z0 = sigmoidf_(d0 + b0);
        const float z1 = sigmoidf_(d1 + b1);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = o[j] * z0 + ycur[h].get(j) * z1;
      }
      const int m = mb + grp + 8 * h;
      if (m < rows) {
        store8<DT>(out + (int64_t)m * 64 + c, o);
        if (raw_out) store8<DT>(raw_out + (int64_t)m * 64 + c, acc[h]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // every lane's reads of the slice precede the next staging
  }
}

static TapRows tap_rows(int F, int T, int64_t sB, int64_t sF, int64_t sT, int C) {
  TapRows g;
  g.F = F;
  g.T = T;
  g.sB = (int)sB;
  g.sF = (int)sF;
  g.sT = (int)sT;
  g.contig = sT == C && sF == (int64_t)T * C && sB == (int64_t)F * T * C;
  return g;
}

template <int C>
static void launch_moments(const float* s, const TapRows& g, int rows, int nblk, const float* w1,
                           double* partial, hipStream_t st, const BnFoldArgs& fold = BnFoldArgs{}) {
  const int rpb = (int)cdiv(rows, nblk);
  hipLaunchKernelGGL(abf_moments_kernel<C>, dim3(nblk), dim3(256), 0, st, s, g, rows, rpb, w1,
                     partial, fold);
}

template <int C, typename DT>
static void launch_fuse(const float* s, const TapRows& g, int rows, const float* w1,
                        const float* scale, const float* shift, const void* res, int Fr, int Tr,
                        const float* aw, const float* ab, void* out, void* raw, hipStream_t st) {
  const int64_t nunits = cdiv(rows, 32);
  const int64_t nb = cdiv(nunits, 4 * 4);  // about four passes per wave
  const unsigned grid = (unsigned)(nb < 2048 ? (nb > 0 ? nb : 1) : 2048);
  if (res)
    hipLaunchKernelGGL((abf_conv1_fuse_kernel<C, DT, true>), dim3(grid), dim3(256), 0, st, s, g,
                       rows, w1, scale, shift, (const DT*)res, Fr, Tr, aw, ab, (DT*)out, (DT*)raw);
  else
    hipLaunchKernelGGL((abf_conv1_fuse_kernel<C, DT, false>), dim3(grid), dim3(256), 0, st, s, g,
                       rows, w1, scale, shift, (const DT*)nullptr, 1, 1, aw, ab, (DT*)out, (DT*)raw);
}

static bool cin_ok(int c) { return c == 8 || c == 16 || c == 32 || c == 64; }

static bool tap_ok(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB, int64_t sF,
                   int64_t sT, int32_t cin) {
  if (((uintptr_t)s & 15) || sB % 4 || sF % 4 || sT % 4 || sB < 0 || sF < 0 || sT < 0) return false;
  const int64_t last = (int64_t)(B - 1) * sB + (int64_t)(F - 1) * sF + (int64_t)(T - 1) * sT + cin;
  return (int64_t)B * F * T < INT32_MAX && last < INT32_MAX;
}

}  // namespace clskd

using namespace clskd;

extern "C" int32_t clskd_abf_moment_blocks(int64_t rows, int32_t cin) {
  // rows per block: the S2 MFMA work grows with cin^2 (10 tile MFMAs per 4 rows at cin = 64)
  int64_t per = cin >= 64 ? 768 : cin >= 32 ? 1024 : 2048;
  // A/B knob: CLSKD_ABF_MOMENT_DIV = d divides the rows per block (more blocks in flight)
  const int div = [] {
    const int v = knob(KNOB_ABF_MOMENT_DIV);
    return v >= 1 && v <= 16 ? v : 1;
  }();
  per = std::max<int64_t>(64, per / div);
  int64_t n = cdiv(rows, per);
  if (n < 1) n = 1;
  if (n > 1024) n = 1024;
  return (int32_t)n;
}

extern "C" int clskd_abf_bn1_partials(const float* s, int32_t B, int32_t F, int32_t T,
                                      int64_t sB, int64_t sF, int64_t sT, int32_t cin,
                                      const float* w1, double* partial, int32_t nblk,
                                      void* stream) {
  CLSKD_CHECK_ARG(s && w1 && partial, "abf_bn1_partials: null pointer");
  CLSKD_CHECK_SHAPE(B > 0 && F > 0 && T > 0 && nblk > 0 && cin_ok(cin),
                    "abf_bn1_partials: shape (cin=%d must be 8/16/32/64)", cin);
  CLSKD_CHECK_ARG(tap_ok(s, B, F, T, sB, sF, sT, cin),
                  "abf_bn1_partials: tap rows must be 16-B aligned channel runs with 32-bit offsets");
  const int rows = B * F * T;
  const TapRows g = tap_rows(F, T, sB, sF, sT, cin);
  const hipStream_t st = as_stream(stream);
  if (skip_kernel(SKIP_ABF)) return CLSKD_OK;
  switch (cin) {
    case 8: launch_moments<8>(s, g, rows, nblk, w1, partial, st); break;
    case 16: launch_moments<16>(s, g, rows, nblk, w1, partial, st); break;
    case 32: launch_moments<32>(s, g, rows, nblk, w1, partial, st); break;
    default: launch_moments<64>(s, g, rows, nblk, w1, partial, st); break;
  }
  CLSKD_LAUNCH_CHECK("abf_bn1_partials");
  return CLSKD_OK;
}

extern "C" int clskd_abf_bn1_fold(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB,
                                  int64_t sF, int64_t sT, int32_t cin, const float* w1,
                                  const clskd_bn_fold* fold, int32_t nblk, void* stream) {
  CLSKD_CHECK_ARG(s && w1 && fold && fold->acc && fold->ticket && fold->scale && fold->shift,
                  "abf_bn1_fold: null pointer");
  CLSKD_CHECK_SHAPE(B > 0 && F > 0 && T > 0 && nblk > 0 && nblk <= 1024 && cin_ok(cin),
                    "abf_bn1_fold: shape (cin=%d must be 8/16/32/64, nblk <= 1024)", cin);
  CLSKD_CHECK_SHAPE(fold->C == 64 && fold->c_off == 0 && fold->finalize == 1 &&
                        fold->count == (int64_t)B * F * T,
                    "abf_bn1_fold: the fold describes the 64 conv1 channels of these rows");
  CLSKD_CHECK_ARG(tap_ok(s, B, F, T, sB, sF, sT, cin),
                  "abf_bn1_fold: tap rows must be 16-B aligned channel runs with 32-bit offsets");
  const int rows = B * F * T;
  const TapRows g = tap_rows(F, T, sB, sF, sT, cin);
  const hipStream_t st = as_stream(stream);
  if (skip_kernel(SKIP_ABF)) return CLSKD_OK;
  clskd_conv_desc d{};
  d.bn_fold = fold;
  const BnFoldArgs f = make_bnfold(d);
  switch (cin) {
    case 8: launch_moments<8>(s, g, rows, nblk, w1, nullptr, st, f); break;
    case 16: launch_moments<16>(s, g, rows, nblk, w1, nullptr, st, f); break;
    case 32: launch_moments<32>(s, g, rows, nblk, w1, nullptr, st, f); break;
    default: launch_moments<64>(s, g, rows, nblk, w1, nullptr, st, f); break;
  }
  CLSKD_LAUNCH_CHECK("abf_bn1_fold");
  return CLSKD_OK;
}

extern "C" int clskd_abf_conv1_fuse(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB,
                                    int64_t sF, int64_t sT, int32_t cin, const float* w1,
                                    const float* scale, const float* shift, const void* res,
                                    int32_t Fr, int32_t Tr, const float* w, const float* b,
                                    void* out, void* x1_raw, int32_t dtype, void* stream) {
  CLSKD_CHECK_ARG(s && w1 && scale && shift && out, "abf_conv1_fuse: null pointer");
  CLSKD_CHECK_ARG(!res || (w && b), "abf_conv1_fuse: a residual needs the attention weights");
  CLSKD_CHECK_SHAPE(B > 0 && F > 0 && T > 0 && cin_ok(cin), "abf_conv1_fuse: shape");
  CLSKD_CHECK_SHAPE(!res || (Fr > 0 && Tr > 0 && (int64_t)B * Fr * Tr * 64 < INT32_MAX),
                    "abf_conv1_fuse: residual shape");
  CLSKD_CHECK_ARG(tap_ok(s, B, F, T, sB, sF, sT, cin),
                  "abf_conv1_fuse: tap rows must be 16-B aligned channel runs with 32-bit offsets");
  CLSKD_CHECK_ARG(dtype == CLSKD_F32 || dtype == CLSKD_BF16, "abf_conv1_fuse: dtype");
  const int rows = B * F * T;
  const TapRows g = tap_rows(F, T, sB, sF, sT, cin);
  const hipStream_t st = as_stream(stream);
  if (skip_kernel(SKIP_ABF)) return CLSKD_OK;
#define CLSKD_ABF_FUSE(CC)                                                                        \
  if (dtype == CLSKD_BF16)                                                                        \
    launch_fuse<CC, __bf16>(s, g, rows, w1, scale, shift, res, Fr, Tr, w, b, out, \
                            x1_raw, st);                                                          \
  else                                                                                            \
    launch_fuse<CC, float>(s, g, rows, w1, scale, shift, res, Fr, Tr, w, b, out,  \
                           x1_raw, st);
  switch (cin) {
    case 8: CLSKD_ABF_FUSE(8) break;
    case 16: CLSKD_ABF_FUSE(16) break;
    case 32: CLSKD_ABF_FUSE(32) break;
    default: CLSKD_ABF_FUSE(64) break;
  }
#undef CLSKD_ABF_FUSE
  CLSKD_LAUNCH_CHECK("abf_conv1_fuse");
  return CLSKD_OK;
}
