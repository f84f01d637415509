// fp32-accurate implicit-GEMM convolution on the bf16 MFMA pipe (round 4): "3 x bf16" split
// products for the fp32 layers of the DCCRN student, the ConvSTFT / ConviSTFT framing GEMMs
// and the LSTM projections (tools_for_model.py:236-262, 303-330; conv_stft.py framing).
//
// gfx950 has no reduced-precision fp32 MFMA (no xf32): exact fp32 products run at
// v_mfma_f32_32x32x2_f32's 64 FLOP/clk/SIMD, 1/16 of the bf16 rate, and the fp32 engines hold
// 30-75 TF/s on these layers.  Each fp32 operand x is split when it is staged into LDS:
//     hi = bf16_rne(x),  lo = bf16_rne(x - hi)      (x - hi is exact in fp32)
// so x = hi + lo + r with |r| <= 2^-18 |x|, and
//     x * w  ~=  hi*whi + hi*wlo + lo*whi           (dropped: lo*wlo <= 2^-18 |x w|, r terms)
// — three v_mfma_f32_32x32x16_bf16 per 16-deep K step instead of eight 32x32x2 fp32 MFMAs, each
// product of two bf16 values exact in the fp32 accumulator.  Per-product relative error is
// bounded by ~3 * 2^-18 (1.1e-5), typically a few 1e-6, against 2^-11 for the TF32 matmuls the
// reference's own training script enables (distill.py:234); accumulation is fp32 as in the
// exact engine.  The split is a library policy for fp32 descriptors (knob CLSKD_F32_SPLIT);
// tests/test_gpu_split.py holds it to torch fp64 and the fp32 goldens.
//
// Structure: persistent workgroups (NW waves, tile = 32*NW rows x 32*NT columns, one wave per
// 32-row block with NT accumulator column blocks), a continuous stream of 16-deep K-tiles across
// the workgroup's tile list: the next K-tile's fp32 operands (the vec4 K-table gather of
// conv_igemm.hip) are loaded into registers while the current one's MFMAs run, then split and
// written to the other LDS stage as hi / lo bf16 planes (32-B rows, 16-B halves XOR-swizzled by
// (row >> 3) & 1: conflict-free fragment reads); one barrier per K-tile.  Row tables are double
// buffered per tile.  The cross terms accumulate in a second register set (two independent
// MFMA chains).  Epilogue: bias-initialised accumulators, fused BatchNorm statistics per
// workgroup (fp64) as partials or as the folded finalize (bnfold.h).
#include <mutex>
#include <unordered_map>
#include <stdlib.h>

#include "bnfold.h"
#include "common.h"

namespace clskd {

namespace sp3 {
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// 16-B chunk swizzle of a plane row (BK bf16 k's = BK / 8 chunks): conflict-free 16-lane
// fragment reads (BK 16: rows of 32 B, 8 rows cover the 64 banks; BK 32: rows of 64 B, 4 rows)
template <int BK>
__device__ __forceinline__ int swz(int row) {
  return BK == 16 ? (row >> 3) & 1 : BK == 32 ? (row >> 2) & 3 : (row >> 1) & 7;
}

// hi / lo bf16 split of 4 fp32 values (RNE both)
__device__ __forceinline__ void split4(const f32x4 v, s16x4& hi, s16x4& lo) {
  bf16x4 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = (__bf16)v[i];
    l[i] = (__bf16)(v[i] - (float)h[i]);
  }
  hi = __builtin_bit_cast(s16x4, h);
  lo = __builtin_bit_cast(s16x4, l);
}

template <typename T>
__device__ __forceinline__ T sel4(int s, T a0, T a1, T a2, T a3) {
  const T lo = (s & 1) ? a1 : a0;
  const T hi = (s & 1) ? a3 : a2;
  return (s & 2) ? hi : lo;
}
}  // namespace sp3

struct SplitArgs {
  clskd_conv_desc d;
  int32_t kt_taps, kt_cpt;  // K-tile visiting order (channel-block-major, as conv_igemm.hip)
  int32_t n_mt, ntiles;     // M-tiles; tiles = n_mt x N-tiles
  int32_t nblk128;          // statistics slots (ceil(M / 128))
  BnFoldArgs f;
};

// NS LDS stages: 2 = the next K-tile is written to the other stage (one barrier per K-tile);
// 1 = it is written in place after a second barrier (half the LDS: more workgroups per CU to
// hide the register-staged gather's latency, which bounds this engine: ~1 µs per K-tile round)
// PD = 2 (round 5): the gather of K-tile k + 2 is issued while K-tile k computes (two register
// sets), so a K-tile's loads have a whole K-tile round more to land before they are split into
// LDS — the engine waited about one gather latency per round at PD = 1 (needs >= 2 K-tiles)
template <int NT, int NW, int BK, int NS, int PD = 1>
__global__ __launch_bounds__(NW * 64) void conv_split3_kernel(const SplitArgs args) {
  using namespace sp3;
  const clskd_conv_desc& d = args.d;
  constexpr int BM = 32 * NW, BN = 32 * NT, NTH = NW * 64;
  constexpr int QR = BK / 4;                      // k-quads per row of a K-tile
  constexpr int ROWB = BK * 2;                    // bytes of a plane row (BK bf16)
  constexpr int RSTEP = NTH / QR;                 // rows per pass of the A gather
  constexpr int NRA = BM / RSTEP;                 // A float4 loads per thread per K-tile
  constexpr int NBL = (BN * QR + NTH - 1) / NTH;  // B float4 loads per thread per K-tile
  constexpr int PA = BM * ROWB, PB = BN * ROWB;   // bytes of one bf16 plane
  static_assert(BK == 16 || BK == 32 || BK == 64, "K-tile depth");
  static_assert(NS == 1 || NS == 2, "LDS stages");
  static_assert(NRA * RSTEP == BM, "A gather covers the tile");
  // cross-term chain: NT >= 2 interleaves independent column accumulators already
  constexpr bool XACC = NT == 1;
  __shared__ __attribute__((aligned(16))) unsigned char sA[NS][2][PA];  // [stage][hi, lo]
  __shared__ __attribute__((aligned(16))) unsigned char sB[NS][2][PB];
  __shared__ int4 rinfo[2][BM];  // fi0, ti0, valid
  __shared__ int rbase[2][4][BM];
  __shared__ int64_t orow[2][BM];
  extern __shared__ int2 ctab[];  // [K/4] k-quad entries: element offset, dF | dT | segment

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t FoTo = (int64_t)d.Fo * d.To;
  const int nk = d.K / BK;
  const bool fold = args.f.acc != nullptr;

  // ---- this workgroup's tile list (XCD-aware contiguous runs, as conv_gemm8) ----------------
  const int grid = gridDim.x, b = blockIdx.x;
  int t_first, t_step, ntl;
  if ((grid & 7) == 0 && args.ntiles >= grid) {
    const int c = b & 7, s = b >> 3, cpx = grid >> 3;
    const int q = args.ntiles >> 3, r = args.ntiles & 7;
    const int len = q + (c < r ? 1 : 0), start = c * q + (c < r ? c : r);
    t_first = start + s;
    t_step = cpx;
    ntl = s < len ? (len - s + cpx - 1) / cpx : 0;
  } else {
    t_first = b;
    t_step = grid;
    ntl = b < args.ntiles ? (args.ntiles - b + grid - 1) / grid : 0;
  }
  if (d.stats) {  // slots no workgroup owns (grid <= nblk128) are zero
    for (int64_t s = (int64_t)b + grid; s < args.nblk128; s += grid)
      for (int i = tid; i < d.N * 2; i += NTH) d.stats[s * d.N * 2 + i] = 0.0;
  }
  if (ntl == 0) {
    if (fold)
      bnfold_commit(args.f, 0, [](int, double& S, double& Q) { S = Q = 0.0; },
                    reinterpret_cast<int*>(&sA[0][0][0]), b, grid);
    return;
  }
  auto tile_mt = [&](int j) { return (t_first + j * t_step) % args.n_mt; };
  auto tile_nt = [&](int j) { return (t_first + j * t_step) / args.n_mt; };

  auto build_table = [&](int j, int buf) {
    for (int i = tid; i < BM; i += NTH) {
      const int64_t m = (int64_t)tile_mt(j) * BM + i;
      const bool valid = m < M;
      const int64_t mm = valid ? m : 0;
      const int64_t bb = mm / FoTo;
      const int64_t r = mm - bb * FoTo;
      const int fo = (int)(r / d.To);
      const int to = (int)(r - (int64_t)fo * d.To);
      const int fi0 = fo * d.stride_f, ti0 = to * d.stride_t;
      rinfo[buf][i] = make_int4(fi0, ti0, valid ? 1 : 0, 0);
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
        rbase[buf][sg][i] = (int)(bb * d.seg[sg].sB + (int64_t)fi0 * d.seg[sg].sF + (int64_t)ti0 * d.seg[sg].sT);
      orow[buf][i] = valid ? bb * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT : -1;
    }
  };
  for (int q = tid; q < d.K / 4; q += NTH) {
    const clskd_ktab_entry e = d.ktab[q * 4];
    const int sg = d.kseg[q * 4];
    ctab[q] = make_int2(e.off, (int)(((unsigned)e.dF & 0xFFFFu) | (((unsigned)e.dT & 0xFFu) << 16) |
                                     ((unsigned)sg << 24)));
  }
  build_table(0, 0);
  if (ntl > 1) build_table(1, 1);
  __syncthreads();

  // ---- per-thread gather geometry of the stream's current tile -------------------------------
  const int kq = tid % QR;
  int rfi[NRA], rti[NRA], rvl[NRA], arb[NRA][4];
  int geo = -1, geo_n0 = 0;
  auto load_geometry = [&](int j) {
#pragma unroll
    for (int i = 0; i < NRA; ++i) {
      const int row = tid / QR + RSTEP * i;
      const int4 ri = rinfo[j & 1][row];
      rfi[i] = ri.x;
      rti[i] = ri.y;
      rvl[i] = ri.z;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) arb[i][sg] = rbase[j & 1][sg][row];
    }
    geo_n0 = tile_nt(j) * BN;
    geo = j;
  };
  const float* sp0 = d.seg[0].ptr;
  const float* sp1 = d.seg[1].ptr;
  const float* sp2 = d.seg[2].ptr;
  const float* sp3 = d.seg[3].ptr;
  const float* wgt = reinterpret_cast<const float*>(d.weight);
  f32x4 ra[NRA], rb[NBL], ra2[NRA], rb2[NBL];  // ra2 / rb2: the second set (PD = 2)
  auto load_kt = [&](int kt, f32x4 (&xa)[NRA], f32x4 (&xb)[NBL]) {
    const int2 ce = ctab[kt * QR + kq];
    const int sg = (int)((unsigned)ce.y >> 24);
    const int dF = (int)(short)(ce.y & 0xFFFF);
    const int dT = (int)(signed char)((ce.y >> 16) & 0xFF);
    const float* sp = sel4(sg, sp0, sp1, sp2, sp3);
    const int Fb = sel4(sg, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F);
    const int Tb = sel4(sg, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T);
#pragma unroll
    for (int i = 0; i < NRA; ++i) {
      const int fi = rfi[i] + dF, ti = rti[i] + dT;
      const int rbs = sel4(sg, arb[i][0], arb[i][1], arb[i][2], arb[i][3]);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (rvl[i] && (unsigned)fi < (unsigned)Fb && (unsigned)ti < (unsigned)Tb)
        v = *reinterpret_cast<const f32x4*>(sp + (int64_t)(rbs + ce.x));
      xa[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + NTH * i;
      const int n = geo_n0 + idx / QR;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx / QR < BN && n < d.N)
        v = *reinterpret_cast<const f32x4*>(wgt + (int64_t)n * d.K + kt * BK + (idx % QR) * 4);
      xb[i] = v;
    }
  };
  // split + write the registers into stage s: k-quad q of a row = 8 B inside chunk q >> 1
  auto store_kt = [&](int s, const f32x4 (&xa)[NRA], const f32x4 (&xb)[NBL]) {
#pragma unroll
    for (int i = 0; i < NRA; ++i) {
      const int row = tid / QR + RSTEP * i;
      const int off = row * ROWB + (((kq >> 1) ^ swz<BK>(row)) << 4) + (kq & 1) * 8;
      s16x4 hi, lo;
      split4(xa[i], hi, lo);
      *reinterpret_cast<s16x4*>(&sA[s][0][off]) = hi;
      *reinterpret_cast<s16x4*>(&sA[s][1][off]) = lo;
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx / QR, q = idx % QR;
      if (row < BN) {
        const int off = row * ROWB + (((q >> 1) ^ swz<BK>(row)) << 4) + (q & 1) * 8;
        s16x4 hi, lo;
        split4(xb[i], hi, lo);
        *reinterpret_cast<s16x4*>(&sB[s][0][off]) = hi;
        *reinterpret_cast<s16x4*>(&sB[s][1][off]) = lo;
      }
    }
  };

  const int kt_taps = args.kt_taps, kt_cpt = args.kt_cpt;
  int it_tap = 0, it_cb = 0;
  auto next_kt = [&]() {
    const int k = it_tap * kt_cpt + it_cb;
    if (++it_tap == kt_taps) {
      it_tap = 0;
      if (++it_cb == kt_cpt) it_cb = 0;
    }
    return k;
  };

  f32x16 acc[NT], accx[XACC ? NT : 1];
  auto init_acc = [&](int j) {
    const int n0 = tile_nt(j) * BN;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = n0 + t * 32 + l32;
      const float bv = (d.bias && n < d.N) ? d.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[t][r] = bv;
        if constexpr (XACC) accx[t][r] = 0.f;
      }
    }
  };

  const int total = ntl * nk;
  load_geometry(0);
  load_kt(next_kt(), ra, rb);
  store_kt(0, ra, rb);
  if (PD == 2 && total > 1) {  // K-tile 1 into the second set
    const int jn = 1 / nk;
    if (jn != geo) load_geometry(jn);
    load_kt(next_kt(), ra2, rb2);
  }
  __syncthreads();

  const int arow = wave * 32 + l32;
  double st_s[NT], st_q[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) st_s[t] = st_q[t] = 0.0;
  float* outp = reinterpret_cast<float*>(d.out);
  int gk = 0;
  for (int j = 0; j < ntl; ++j) {
    init_acc(j);
    for (int kt = 0; kt < nk; ++kt, ++gk) {
      const int s = NS == 2 ? (gk & 1) : 0;
      const bool pf = gk + 1 < total;
      if constexpr (PD == 1) {
        if (pf) {
          const int jn = (gk + 1) / nk;
          if (jn != geo) load_geometry(jn);
          load_kt(next_kt(), ra, rb);
        }
      } else if (gk + 2 < total) {  // K-tile gk + 2 into the set K-tile gk came from
        const int jn = (gk + 2) / nk;
        if (jn != geo) load_geometry(jn);
        if (gk & 1)
          load_kt(next_kt(), ra2, rb2);
        else
          load_kt(next_kt(), ra, rb);
      }
      // the set holding K-tile gk + 1 (PD = 2: loaded one K-tile round ago)
      auto store_next = [&](int st) {
        if (PD == 1 || (gk & 1))
          store_kt(st, ra, rb);
        else
          store_kt(st, ra2, rb2);
      };
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {  // 16-deep MFMA steps: chunk 2 ks + h of a row
        const int aoff = arow * ROWB + (((2 * ks + h) ^ swz<BK>(arow)) << 4);
        const s16x8 ahi = *reinterpret_cast<const s16x8*>(&sA[s][0][aoff]);
        const s16x8 alo = *reinterpret_cast<const s16x8*>(&sA[s][1][aoff]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int brow = t * 32 + l32;
          const int boff = brow * ROWB + (((2 * ks + h) ^ swz<BK>(brow)) << 4);
          const s16x8 bhi = *reinterpret_cast<const s16x8*>(&sB[s][0][boff]);
          const s16x8 blo = *reinterpret_cast<const s16x8*>(&sB[s][1][boff]);
          acc[t] = mfma16<__bf16>(ahi, bhi, acc[t]);
          if constexpr (XACC) {
            accx[t] = mfma16<__bf16>(ahi, blo, accx[t]);
            accx[t] = mfma16<__bf16>(alo, bhi, accx[t]);
          }
        }
        if constexpr (!XACC) {  // cross terms after every column's main term: no back-to-back
#pragma unroll                   // dependent MFMA on one accumulator
          for (int t = 0; t < NT; ++t) {
            const int brow = t * 32 + l32;
            const int boff = brow * ROWB + (((2 * ks + h) ^ swz<BK>(brow)) << 4);
            const s16x8 bhi = *reinterpret_cast<const s16x8*>(&sB[s][0][boff]);
            acc[t] = mfma16<__bf16>(alo, bhi, acc[t]);
          }
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int brow = t * 32 + l32;
            const int boff = brow * ROWB + (((2 * ks + h) ^ swz<BK>(brow)) << 4);
            const s16x8 blo = *reinterpret_cast<const s16x8*>(&sB[s][1][boff]);
            acc[t] = mfma16<__bf16>(ahi, blo, acc[t]);
          }
        }
      }
      if constexpr (NS == 2) {
        if (pf) store_next(s ^ 1);
        __syncthreads();
      } else {
        __syncthreads();  // every wave is done reading the stage
        if (pf) store_next(0);
        __syncthreads();
      }
    }

    // ---- tile epilogue: statistics (valid rows / columns) and predicated stores ---------------
    const int n0 = tile_nt(j) * BN;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = n0 + t * 32 + l32;
      const bool nok = n < d.N;
      const int64_t coff = nok ? (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo : 0;
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t ro = orow[j & 1][row];
        float v = acc[t][r];
        if constexpr (XACC) v += accx[t][r];
        if (nok && ro >= 0) {
          if (d.accumulate) v += outp[ro + coff];  // data-gradient sums (no statistics then)
          sm += v;
          sq = fmaf(v, v, sq);
          outp[ro + coff] = v;
        }
      }
      st_s[t] += (double)sm;
      st_q[t] += (double)sq;
    }
    if (j + 2 < ntl) {  // row table of tile j + 2 into this tile's buffer
      __syncthreads();
      build_table(j + 2, j & 1);
      __syncthreads();
    }
  }

  if (d.stats || fold) {  // workgroup totals: lane halves, then waves in a fixed order
    __syncthreads();
    double* red = reinterpret_cast<double*>(&sA[0][0][0]);  // [NW][BN][2]
    static_assert(NW * BN * 16 + 16 <= (int)sizeof(sA), "statistics scratch fits in sA");
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double s2 = st_s[t] + __shfl_xor(st_s[t], 32, 64);
      const double q2 = st_q[t] + __shfl_xor(st_q[t], 32, 64);
      if (h == 0) {
        red[(wave * BN + t * 32 + l32) * 2] = s2;
        red[(wave * BN + t * 32 + l32) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    auto sum_waves = [&](int n, double& S, double& Q) {
      S = 0.0;
      Q = 0.0;
      for (int w = 0; w < NW; ++w) {
        S += red[(w * BN + n) * 2];
        Q += red[(w * BN + n) * 2 + 1];
      }
    };
    if (fold) {
      bnfold_commit(args.f, d.N, sum_waves, reinterpret_cast<int*>(red + NW * BN * 2), b, grid);
    } else {
      for (int n = tid; n < d.N; n += NTH) {
        double S, Q;
        sum_waves(n, S, Q);
        d.stats[((int64_t)b * d.N + n) * 2] = S;
        d.stats[((int64_t)b * d.N + n) * 2 + 1] = Q;
      }
    }
  }
}

// LDS stages of an instance: two (stores of K-tile k + 1 beside the MFMAs of k, one barrier per
// K-tile) except the 64-deep tiles, which take one stage to fit two or three workgroups per CU —
// unless CLSKD_SPLIT_NS2=1 (default) and nt >= 2: those instances keep one workgroup per CU
// resident anyway (260-404 VGPRs), so their second stage costs no occupancy
static int split_stages(int bk, int nt) {
  if (bk != 64) return 2;
  const int k = knob(KNOB_SPLIT_NS2);  // 2: every 64-deep instance (A/B: nt 1 drops to one WG/CU)
  return (k == 1 && nt >= 2) || k == 2 ? 2 : 1;
}

// Plan: which instance, grid and K order; false = not this kernel (the caller's engines run).
static bool split_plan(const clskd_conv_desc& d, SplitArgs& a, int& nt, int& bk, int& grid,
                       int* cus_out = nullptr) {
  if (d.compute != CLSKD_F32 || d.in_dtype != CLSKD_F32 || d.out_dtype != CLSKD_F32) return false;
  if (d.wlayout != CLSKD_WLAYOUT_NK || !d.vec4) return false;
  if (d.accumulate && (d.stats || d.bn_fold)) return false;  // (the exact engines refuse it too)
  if (d.K % 16 || (int64_t)(d.K / 4) * 8 > 32 * 1024) return false;  // K padded to 16 (host)
  if (d.nseg < 1 || d.nseg > 4 || d.stride_t < 1) return false;
  nt = d.N <= 32 ? 1 : d.N <= 64 ? 2 : 4;
  const int BN = 32 * nt, BM = 128;
  if ((d.stats || d.bn_fold) && d.N > BN) return false;  // statistics: one column tile
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t n_mt = cdiv(M, BM), n_nt = cdiv(d.N, BN);
  if (n_mt * n_nt > (1 << 30)) return false;
  a.d = d;
  a.n_mt = (int)n_mt;
  a.ntiles = (int)(n_mt * n_nt);
  a.nblk128 = (int)cdiv(M, 128);
  // the deepest K-tile K allows: each K-tile round costs about one gather latency, so deeper
  // tiles carry more MFMA work per round (64: single LDS stage, two or three workgroups per CU)
  bk = d.K % 64 == 0 ? 64 : d.K % 32 == 0 ? 32 : 16;
  const int cap_bk = knob(KNOB_SPLIT_BK);  // A/B: the deepest K-tile allowed (0: 64)
  if (cap_bk == 16 || cap_bk == 32) bk = bk < cap_bk ? bk : cap_bk;
  a.kt_taps = 1;
  a.kt_cpt = d.K / bk;
  if (d.ntaps > 1 && d.ctot % bk == 0 && (int64_t)d.ntaps * d.ctot == d.K) {
    a.kt_taps = d.ntaps;
    a.kt_cpt = d.ctot / bk;
  }
  a.f = make_bnfold(d);
  static int ncu = [] {
    int v = 256;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
    return v > 0 ? v : 256;
  }();
  // 4-wave workgroups, as many per CU as LDS holds (up to three): more waves per SIMD hide more
  // of the gather latency
  const size_t tab = (size_t)2 * 128 * (16 + 16 + 8);
  const size_t lds = (size_t)split_stages(bk, nt) * 2 * (size_t)(128 + 32 * nt) * bk * 2 + tab +
                     (size_t)(d.K / 4) * 8;
  const int per_cu = lds * 3 <= 160 * 1024 ? 3 : lds * 2 <= 160 * 1024 ? 2 : 1;
  // CLSKD_SPLIT_GRID caps the CUs the grid spans (A/B inside the concurrent step; tests: many
  // tiles per workgroup, so K-tile prefetch crosses tiles)
  const int gcap = knob(KNOB_SPLIT_GRID);
  const int cus = gcap > 0 && gcap < ncu ? gcap : ncu;
  if (cus_out) *cus_out = cus;
  const int cap = per_cu * cus;
  grid = a.ntiles < cap ? a.ntiles : cap;
  if (d.stats && grid > a.nblk128) return false;  // (never: BM = 128 rows a tile)
  return true;
}

// force: the descriptor asked for split products (CLSKD_F32X3, passed here as CLSKD_F32);
// otherwise the global A/B knob CLSKD_F32_SPLIT routes every fp32 descriptor
bool conv_split3_takes(const clskd_conv_desc& d, bool force) {
  if (!force && knob(KNOB_F32_SPLIT) != 1) return false;
  SplitArgs a;
  int nt = 0, bk = 0, grid = 0;
  return split_plan(d, a, nt, bk, grid);
}

int launch_conv_split3(const clskd_conv_desc& d, hipStream_t st, bool* launched, bool force) {
  *launched = false;
  if (!force && knob(KNOB_F32_SPLIT) != 1) return CLSKD_OK;
  SplitArgs a;
  int nt = 0, bk = 0, grid = 0, cus = 0;
  if (!split_plan(d, a, nt, bk, grid, &cus)) return CLSKD_OK;
  // CLSKD_SPLIT_OCC=1 (default): the grid holds only the workgroups the instance's register
  // occupancy keeps resident (the plan counts LDS only: up to 3 per CU, while 208-404 VGPRs allow
  // 1-2), so every workgroup is resident from the start and walks its tiles as one persistent
  // stream (0: the LDS-sized grid; -0.02..-0.04 ms per C2 step, profiles/r5_split_pd_ab.txt)
  const bool occ = knob(KNOB_SPLIT_OCC) == 1;
  auto occ_cap = [&](const void* k, size_t lds) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> per;
    int nb;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = per.find(k);
      if (it == per.end()) {
        nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, lds) != hipSuccess || nb < 1) nb = 1;
        per[k] = nb;
      } else {
        nb = it->second;
      }
    }
    return grid < nb * cus ? grid : nb * cus;
  };
  const size_t ctab_bytes = (size_t)(d.K / 4) * 8;
  // CLSKD_SPLIT_PD=2: two K-tiles in flight where the stream has two — measured slower inside the
  // C2 step (profiles/r5_split_pd_ab.txt: +0.07 ms even where occupancy is unchanged, +0.23 ms on
  // every instance), so one (1) is the default
  const int pd = knob(KNOB_SPLIT_PD) == 2 && d.K / bk >= 2 ? 2 : 1;
  const int ns = split_stages(bk, nt);
  auto go = [&](auto kern, int NT_, int BK_, int NS_) {
    const void* k = (const void*)kern;
    if (occ) grid = occ_cap(k, ctab_bytes);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), ctab_bytes, st, a);
    note_kernel_fn(k);
    if (pd == 2)
      note_kernel("conv_split3_kernel<%d,4,%d,%d,2>", NT_, BK_, NS_);
    else
      note_kernel("conv_split3_kernel<%d,4,%d,%d>", NT_, BK_, NS_);
  };
#define SP3(NT_, BK_, NS_)                                                                  \
  (pd == 2 ? go(conv_split3_kernel<NT_, 4, BK_, NS_, 2>, NT_, BK_, NS_)                     \
           : go(conv_split3_kernel<NT_, 4, BK_, NS_, 1>, NT_, BK_, NS_))
  if (bk == 64) {
    if (nt == 1) (ns == 2 ? SP3(1, 64, 2) : SP3(1, 64, 1));
    else if (nt == 2) (ns == 2 ? SP3(2, 64, 2) : SP3(2, 64, 1));
    else (ns == 2 ? SP3(4, 64, 2) : SP3(4, 64, 1));
  } else if (bk == 32) {
    if (nt == 1) SP3(1, 32, 2);
    else if (nt == 2) SP3(2, 32, 2);
    else SP3(4, 32, 2);
  } else {
    if (nt == 1) SP3(1, 16, 2);
    else if (nt == 2) SP3(2, 16, 2);
    else SP3(4, 16, 2);
  }
#undef SP3
  *launched = true;
  return CLSKD_OK;
}

}  // namespace clskd
