// Implicit-GEMM convolution engine for BFTC activations (gfx950, fp32 MFMA 32x32x2).
//
// One engine serves every GEMM-shaped op on the DCCRN/CLSKD path (see include/clskd.h):
// complex Conv2d (packed [[Wr,-Wi],[Wi,Wr]] weights), polyphase ConvTranspose2d, ABF 1x1/3x3
// convs, the ConvSTFT/ConviSTFT/MRSTFT framing GEMMs and the LSTM input/output projections.
//
// Tile: BM=128 output rows x BN output channels x BK=16, 256 threads = 4 waves; wave w owns
// rows [32w, 32w+32) x all BN columns as BN/32 accumulators of v_mfma_f32_32x32x2_f32.
// The K loop is register-prefetched one tile ahead into a second LDS buffer (one barrier per
// K-tile).  Inside a K-tile the reduction order is permuted so each lane reads its MFMA
// operands as 8 contiguous floats (two ds_read_b128): step s uses k = 8*(lane>>5) + s.
// LDS rows are 64 B; 16-B chunks are XOR-swizzled by ((row>>2)&3) so the ds_read_b128 lane
// groups hit 16 distinct bank slots.
#include <stdlib.h>

#include "common.h"

namespace clskd {

constexpr int BK = 16;

struct ConvArgs {
  clskd_conv_desc d;
  // K-tile visiting order (as conv_gemm8): kt_taps x kt_cpt K-tiles visited channel-block-major
  // when every 16-deep K-tile lies inside one tap; kt_taps = 1, kt_cpt = K / 16: packed order
  int kt_taps, kt_cpt;
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// select the per-segment value without runtime-indexed arrays (which would go to scratch)
template <typename T>
__device__ __forceinline__ T sel4(int s, T a0, T a1, T a2, T a3) {
  // two levels of value selects (v_cndmask): an if-else chain compiles to exec-mask branches
  const T lo = (s & 1) ? a1 : a0;
  const T hi = (s & 1) ? a3 : a2;
  return (s & 2) ? hi : lo;
}

template <typename OutT>
__device__ __forceinline__ void store_val(OutT* p, float v) { *p = (OutT)v; }

template <int BN, bool VEC4, typename OutT, int NW = 4>
__global__ __launch_bounds__(NW * 64) void conv_igemm_f32(const ConvArgs args) {
  const clskd_conv_desc& d = args.d;
  constexpr int NT = BN / 32;
  constexpr int BM = 32 * NW;        // rows per tile: 32 per wave
  constexpr int NTH = NW * 64;       // threads
  constexpr int RSTEP = NTH / 4;     // A-gather row stride between a thread's two rows
  __shared__ __attribute__((aligned(16))) float As[2][BM * BK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * BK];
  __shared__ int64_t out_row[BM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)tile * BM;
  const int n0 = blockIdx.y * BN;
  const int nk = d.K / BK;  // host pads K to a multiple of BK
  const int64_t FoTo = (int64_t)d.Fo * d.To;

  // ---- per-block tables: output row offsets; (VEC4) per-row gather bases per segment and the
  //      K-chunk table (one int2 per 4 k: element offset, dF | dT | segment) in LDS, so a
  //      gathered float4 costs one LDS read and a few selects instead of 64-bit index math ----
  __shared__ int rowinfo[BM][4];     // fi0, ti0, valid
  __shared__ int rowbase[4][BM];     // element offset of (b, fi0, ti0) in segment s
  if (tid < BM) {
    int64_t m = m0 + tid;
    int64_t off = -1;
    const bool valid = m < M;
    const int64_t mm = valid ? m : 0;
    const int64_t b = mm / FoTo;
    const int64_t r = mm - b * FoTo;
    const int fo = (int)(r / d.To);
    const int to = (int)(r - (int64_t)fo * d.To);
    if (valid) off = b * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT;
    out_row[tid] = off;
    if constexpr (VEC4) {
      const int fi0 = fo * d.stride_f, ti0 = to * d.stride_t;
      rowinfo[tid][0] = fi0;
      rowinfo[tid][1] = ti0;
      rowinfo[tid][2] = valid ? 1 : 0;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg)
        rowbase[sg][tid] = (int)(b * d.seg[sg].sB + (int64_t)fi0 * d.seg[sg].sF + (int64_t)ti0 * d.seg[sg].sT);
    }
  }
  extern __shared__ int2 ctab[];  // VEC4: [K/4] chunk entries (dynamic LDS)
  if constexpr (VEC4) {
    for (int q = tid; q < d.K / 4; q += NTH) {
      const clskd_ktab_entry e = d.ktab[q * 4];
      const int sg = d.kseg[q * 4];
      ctab[q] = make_int2(e.off, (int)(((unsigned)e.dF & 0xFFFFu) | (((unsigned)e.dT & 0xFFu) << 16) |
                                       ((unsigned)sg << 24)));
    }
    __syncthreads();
  }

  // ---- A-gather rows owned by this thread: rows (tid>>2) and (tid>>2)+RSTEP, k-quad (tid&3) --
  const int kq = tid & 3;
  bool rvalid[2];
  int rb[2], rfi[2], rti[2];
  int a_rb[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (tid >> 2) + RSTEP * i;
    if constexpr (VEC4) {
      rfi[i] = rowinfo[row][0];
      rti[i] = rowinfo[row][1];
      rvalid[i] = rowinfo[row][2] != 0;
      rb[i] = 0;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) a_rb[i][sg] = rowbase[sg][row];
    } else {
      int64_t m = m0 + row;
      rvalid[i] = m < M;
      int64_t mm = rvalid[i] ? m : 0;
      int64_t b = mm / FoTo;
      int64_t r = mm - b * FoTo;
      int fo = (int)(r / d.To);
      int to = (int)(r - (int64_t)fo * d.To);
      rb[i] = (int)b;
      rfi[i] = fo * d.stride_f;
      rti[i] = to * d.stride_t;
#pragma unroll
      for (int sg = 0; sg < 4; ++sg) a_rb[i][sg] = 0;
    }
  }
  const float* sp0 = d.seg[0].ptr;
  const float* sp1 = d.seg[1].ptr;
  const float* sp2 = d.seg[2].ptr;
  const float* sp3 = d.seg[3].ptr;

  auto load_a = [&](int kt, f32x4 (&ra)[2]) {
    if constexpr (VEC4) {
      const int2 ce = ctab[kt * (BK / 4) + kq];
      const int sg = (int)((unsigned)ce.y >> 24);
      const int dF = (int)(short)(ce.y & 0xFFFF);
      const int dT = (int)(signed char)((ce.y >> 16) & 0xFF);
      const float* sp = sel4(sg, sp0, sp1, sp2, sp3);
      const int Fb = sel4(sg, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F);
      const int Tb = sel4(sg, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int fi = rfi[i] + dF;
        const int ti = rti[i] + dT;
        const int rbase = sel4(sg, a_rb[i][0], a_rb[i][1], a_rb[i][2], a_rb[i][3]);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (rvalid[i] && (unsigned)fi < (unsigned)Fb && (unsigned)ti < (unsigned)Tb)
          v = *reinterpret_cast<const f32x4*>(sp + (int64_t)(rbase + ce.x));
        ra[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = kt * BK + kq * 4 + q;
          const clskd_ktab_entry e = d.ktab[k];
          const int s = d.kseg[k];
          const float* sp = sel4(s, d.seg[0].ptr, d.seg[1].ptr, d.seg[2].ptr, d.seg[3].ptr);
          const int64_t sB = sel4(s, d.seg[0].sB, d.seg[1].sB, d.seg[2].sB, d.seg[3].sB);
          const int64_t sF = sel4(s, d.seg[0].sF, d.seg[1].sF, d.seg[2].sF, d.seg[3].sF);
          const int64_t sT = sel4(s, d.seg[0].sT, d.seg[1].sT, d.seg[2].sT, d.seg[3].sT);
          const int Fb = sel4(s, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F);
          const int Tb = sel4(s, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T);
          const int fi = rfi[i] + e.dF;
          const int ti = rti[i] + e.dT;
          if (rvalid[i] && fi >= 0 && fi < Fb && ti >= 0 && ti < Tb) {
            v[q] = sp[(int64_t)rb[i] * sB + (int64_t)rfi[i] * sF + (int64_t)rti[i] * sT + e.off];
          }
        }
        ra[i] = v;
      }
    }
  };

  constexpr int NBL = (BN * 4 + NTH - 1) / NTH;  // float4 B loads per thread
  auto load_b = [&](int kt, f32x4 (&rbv)[NBL]) {
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + NTH * i;
      const int n = n0 + (idx >> 2);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if ((idx >> 2) < BN && n < d.N)
        v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(d.weight) + (int64_t)n * d.K +
                                            kt * BK + (idx & 3) * 4);
      rbv[i] = v;
    }
  };

  auto store_tiles = [&](int buf, const f32x4 (&ra)[2], const f32x4 (&rbv)[NBL]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (tid >> 2) + RSTEP * i;
      *reinterpret_cast<f32x4*>(&As[buf][row * BK + swz(row, kq) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx >> 2;
      if (row < BN) *reinterpret_cast<f32x4*>(&Bs[buf][row * BK + swz(row, idx & 3) * 4]) = rbv[i];
    }
  };

  // accumulators start at the bias: no loads are left for the epilogue's store branches
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = n0 + t * 32 + (lane & 31);
    const float bv = (d.bias && n < d.N) ? d.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = bv;
  }

  // packed K-tile of the next load: all taps of a channel block before the next block, so the
  // rows a K-tile gathers (one tap further) were fetched by the CU's previous K-tile
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
  f32x4 ra[2];
  f32x4 rbv[NBL];
  {
    const int k0 = next_kt();
    load_a(k0, ra);
    load_b(k0, rbv);
  }
  store_tiles(0, ra, rbv);
  __syncthreads();

  const int arow = wave * 32 + (lane & 31);
  const int h = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      const int kn = next_kt();
      load_a(kn, ra);
      load_b(kn, rbv);
    }
    const float* as = &As[buf][0];
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(as + arow * BK + swz(arow, 2 * h) * 4);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(as + arow * BK + swz(arow, 2 * h + 1) * 4);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int brow = t * 32 + (lane & 31);
      const float* bs = &Bs[buf][0];
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bs + brow * BK + swz(brow, 2 * h) * 4);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(bs + brow * BK + swz(brow, 2 * h + 1) * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc[t], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc[t], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1, ra, rbv);
    __syncthreads();
  }

  if (d.stats) {  // fused BatchNorm statistics (fp32 per lane, fp64 across lanes/waves)
    // one partial per 128-row block (the fused-statistics contract): waves 4h..4h+3 of a
    // 256-row tile form block 2*tile + h
    __syncthreads();
    double* red = reinterpret_cast<double*>(&As[0][0]);  // [NW waves][BN][2]
    static_assert(NW * BN * 2 * 8 <= 2 * BM * BK * 4, "stats scratch fits in As");
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = t * 32 + (lane & 31);
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (out_row[row] >= 0) {
          const float v = acc[t][r];
          sm += v;
          sq = fmaf(v, v, sq);
        }
      }
      const double ds = (double)sm + (double)__shfl_xor(sm, 32, 64);
      const double dq = (double)sq + (double)__shfl_xor(sq, 32, 64);
      if (h == 0) {
        red[(wave * BN + col) * 2] = ds;
        red[(wave * BN + col) * 2 + 1] = dq;
      }
    }
    __syncthreads();
    const int64_t nblk128 = (M + 127) / 128;
    for (int q = tid; q < BN * (NW / 4); q += NTH) {
      const int c = q % BN, hb = q / BN;
      const int n = n0 + c;
      const int64_t blk = (int64_t)tile * (NW / 4) + hb;
      if (n >= d.N || blk >= nblk128) continue;
      const int w0 = 4 * hb;
      const double S = red[(w0 * BN + c) * 2] + red[((w0 + 1) * BN + c) * 2] +
                       red[((w0 + 2) * BN + c) * 2] + red[((w0 + 3) * BN + c) * 2];
      const double Q = red[(w0 * BN + c) * 2 + 1] + red[((w0 + 1) * BN + c) * 2 + 1] +
                       red[((w0 + 2) * BN + c) * 2 + 1] + red[((w0 + 3) * BN + c) * 2 + 1];
      d.stats[(blk * d.N + n) * 2] = S;
      d.stats[(blk * d.N + n) * 2 + 1] = Q;
    }
  }

  // ---- epilogue: predicated scatter stores (bias already in the accumulators) ----
  OutT* outp = reinterpret_cast<OutT*>(d.out);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = n0 + t * 32 + (lane & 31);
    if (n >= d.N) continue;
    const int64_t coff = (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t ro = out_row[row];
      if (ro >= 0) {
        float v = acc[t][r];
        if constexpr (sizeof(OutT) == 4) {
          if (d.accumulate) v += outp[ro + coff];
        }
        store_val<OutT>(outp + ro + coff, v);
      }
    }
  }
}

int launch_conv_bf16(const clskd_conv_desc& d, hipStream_t st);

int launch_conv_direct(const clskd_conv_desc& d, hipStream_t st);

int launch_conv_pointwise(const clskd_conv_desc& d, hipStream_t st, bool* launched);
int launch_conv_halo_f32(const clskd_conv_desc& d, hipStream_t st, bool* launched);
int launch_conv_split3(const clskd_conv_desc& d, hipStream_t st, bool* launched, bool force);

}  // namespace clskd

using namespace clskd;

namespace clskd {
bool conv_halo_takes(const clskd_conv_desc& d);
bool conv_halo_f32_takes(const clskd_conv_desc& d);
bool conv_gemm8_takes(const clskd_conv_desc& d);
#ifdef CLSKD_EXPERIMENTS
bool conv_halow_takes(const clskd_conv_desc& d);
#endif
bool conv_pointwise_takes(const clskd_conv_desc& d);
bool conv_split3_takes(const clskd_conv_desc& d, bool force);
}  // namespace clskd

// The kernel a descriptor dispatches to folds the BatchNorm finalize (clskd_bn_fold): the
// persistent engines.  Mirrors the dispatch order of clskd_conv2d_fwd.
static bool fold_capable(const clskd_conv_desc& dd) {
  if (dd.wlayout == CLSKD_WLAYOUT_DIRECT || dd.accumulate) return false;
  if (is_lowp(dd.compute)) {
    if (conv_halo_takes(dd)) return true;
#ifdef CLSKD_EXPERIMENTS
    if (conv_halow_takes(dd)) return true;
#endif
    return conv_gemm8_takes(dd) && dd.N <= 256;  // one N-tile (256x256 / 256x128 instances)
  }
  const bool split = dd.compute == CLSKD_F32X3;
  clskd_conv_desc d = dd;  // the fp32 engines see CLSKD_F32 (F32X3 only asks for the split)
  d.compute = CLSKD_F32;
  if (conv_pointwise_takes(d)) return false;
  if (conv_split3_takes(d, split)) return true;
  return knob(KNOB_NO_HALO32) != 1 && conv_halo_f32_takes(d);
}

extern "C" int32_t clskd_conv_fold_capable(const clskd_conv_desc* dp) {
  if (!dp) return 0;
  return fold_capable(*dp) ? 1 : 0;
}

extern "C" int64_t clskd_bn_fold_state_size(int32_t C) {
  return C > 0 ? (int64_t)CLSKD_BN_FOLD_REPL * C * 6 : 0;
}

extern "C" int clskd_conv2d_fwd(const clskd_conv_desc* dp, void* stream) {
  CLSKD_CHECK_ARG(dp != nullptr, "conv2d: null descriptor");
  CLSKD_CHECK_ARG(dp->compute == CLSKD_F32 || dp->compute == CLSKD_BF16 || dp->compute == CLSKD_F16 ||
                      dp->compute == CLSKD_F32X3,
                  "conv2d: unknown compute %d", dp->compute);
  CLSKD_CHECK_ARG(dp->compute != CLSKD_F32X3 || dp->in_dtype == CLSKD_F32,
                  "conv2d: split products (CLSKD_F32X3) take fp32 segments");
  // CLSKD_F32X3 asks for the split engine; every fp32 engine sees the descriptor as CLSKD_F32
  const bool want_split = dp->compute == CLSKD_F32X3;
  clskd_conv_desc dcopy = *dp;
  if (want_split) dcopy.compute = CLSKD_F32;
  const clskd_conv_desc& d = dcopy;
  CLSKD_CHECK_SHAPE(d.B > 0 && d.Fo > 0 && d.To > 0 && d.N > 0 && d.K > 0, "conv2d: empty shape");
  if (const clskd_bn_fold* f = d.bn_fold) {
    CLSKD_CHECK_ARG(!d.stats, "conv2d: bn_fold and stats are exclusive");
    CLSKD_CHECK_ARG(f->acc && f->ticket && f->scale && f->shift, "conv2d: bn_fold null pointer");
    CLSKD_CHECK_SHAPE(f->C > 0 && f->c_off >= 0 && f->c_off + d.N <= f->C && f->count > 0,
                      "conv2d: bn_fold channels [%d, +%d) outside C=%d", f->c_off, d.N, f->C);
    CLSKD_CHECK_ARG(fold_capable(*dp), "conv2d: N=%d K=%d dispatches to a kernel without the folded "
                    "BatchNorm finalize (clskd_conv_fold_capable)", d.N, d.K);
  }
  const bool lowp = is_lowp(d.compute);
  const int kmul = lowp ? 64 : BK;
  CLSKD_CHECK_SHAPE(d.K % kmul == 0, "conv2d: K=%d must be padded to a multiple of %d", d.K, kmul);
  CLSKD_CHECK_SHAPE(!lowp || d.K <= 8192, "conv2d(bf16/f16): K=%d > 8192", d.K);
  CLSKD_CHECK_ARG(d.in_dtype == d.compute,
                  "conv2d: 16-bit MFMA operands come from activations of that type (in_dtype)");
  CLSKD_CHECK_ARG(d.out_dtype == CLSKD_F32 || d.out_dtype == CLSKD_BF16 || d.out_dtype == CLSKD_F16,
                  "conv2d: out_dtype");
  CLSKD_CHECK_ARG(!is_lowp(d.out_dtype) || !lowp || d.out_dtype == d.in_dtype,
                  "conv2d: a 16-bit output of a 16-bit GEMM has the input's type");
  CLSKD_CHECK_SHAPE(d.nseg >= 1 && d.nseg <= CLSKD_MAX_SEGS, "conv2d: nseg=%d", d.nseg);
  CLSKD_CHECK_ARG(d.weight && d.out && d.ktab && d.kseg, "conv2d: null pointer");
  CLSKD_CHECK_SHAPE(d.nlo >= 1, "conv2d: nlo must be >= 1");
  CLSKD_CHECK_ARG(((uintptr_t)d.weight & 15) == 0, "conv2d: weight must be 16-byte aligned");
  for (int s = 0; s < d.nseg; ++s) CLSKD_CHECK_ARG(d.seg[s].ptr != nullptr, "conv2d: null segment %d", s);
  if (is_lowp(d.in_dtype)) {
    for (int s = 0; s < d.nseg; ++s) {
      const clskd_seg& g = d.seg[s];
      CLSKD_CHECK_ARG(((uintptr_t)g.ptr & 15) == 0 && g.sB % 8 == 0 && g.sF % 8 == 0 && g.sT % 8 == 0,
                      "conv2d(bf16/f16): segment %d must be 16-byte aligned with strides %% 8", s);
    }
  } else if (d.vec4) {
    for (int s = 0; s < d.nseg; ++s) {
      const clskd_seg& g = d.seg[s];
      CLSKD_CHECK_ARG(((uintptr_t)g.ptr & 15) == 0 && g.sB % 4 == 0 && g.sF % 4 == 0 && g.sT % 4 == 0,
                      "conv2d: vec4 segment %d not 16-byte aligned", s);
    }
  }
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  CLSKD_CHECK_SHAPE(M < (int64_t)INT32_MAX * 64, "conv2d: too many rows");
  hipStream_t st = as_stream(stream);
  CLSKD_CHECK_SHAPE(d.kvec == 0 || d.kvec == 1 || d.kvec == 2 || d.kvec == 4 || d.kvec == 8,
                    "conv2d: kvec=%d", d.kvec);
  CLSKD_CHECK_ARG(d.wlayout == CLSKD_WLAYOUT_NK || d.wlayout == CLSKD_WLAYOUT_DIRECT,
                  "conv2d: wlayout=%d", d.wlayout);
  CLSKD_CHECK_ARG(!d.accumulate || ((d.compute == CLSKD_F32 || d.compute == CLSKD_BF16) &&
                                     d.out_dtype == CLSKD_F32),
                  "conv2d: accumulate needs fp32 or bf16 compute and an fp32 output (the fp32 "
                  "engines, the direct kernel, the bf16 LDS-DMA engine)");
  if (d.wlayout == CLSKD_WLAYOUT_DIRECT) {
    if (skip_kernel(SKIP_CONV_DIRECT)) return CLSKD_OK;
    const int rc = launch_conv_direct(d, st);
    if (rc != CLSKD_OK) return rc;
    CLSKD_LAUNCH_CHECK("conv2d_direct");
    return CLSKD_OK;
  }
  if (lowp) {
    if (skip_kernel(SKIP_CONV_LOWP)) return CLSKD_OK;
    const int rc = launch_conv_bf16(d, st);
    if (rc != CLSKD_OK) return rc;
    CLSKD_LAUNCH_CHECK("conv2d_bf16");
    return CLSKD_OK;
  }
  if (skip_kernel(SKIP_CONV_F32)) return CLSKD_OK;
  {  // 1x1 channel lifts with short K: the streaming pointwise kernel (conv_pointwise.hip)
    bool launched = false;
    const int rc = launch_conv_pointwise(d, st, &launched);
    if (rc != CLSKD_OK) return rc;
    if (launched) {
      CLSKD_LAUNCH_CHECK("conv2d_pointwise");
      return CLSKD_OK;
    }
  }
  {  // fp32-accurate 3 x bf16 split products on the bf16 MFMA pipe (CLSKD_F32X3 descriptors;
     // every fp32 descriptor with the A/B knob CLSKD_F32_SPLIT=1)
    bool launched = false;
    const int rc = launch_conv_split3(d, st, &launched, want_split);
    if (rc != CLSKD_OK) return rc;
    if (launched) {
      CLSKD_LAUNCH_CHECK("conv2d_split3");
      return CLSKD_OK;
    }
  }
  if (knob(KNOB_NO_HALO32) != 1) {  // narrow tap-structured layers: halo-tiled fp32 kernel
    bool launched = false;
    const int rc = launch_conv_halo_f32(d, st, &launched);
    if (rc != CLSKD_OK) return rc;
    if (launched) {
      CLSKD_LAUNCH_CHECK("conv2d_halo_f32");
      return CLSKD_OK;
    }
  }
  ConvArgs a{d, 1, d.K / BK};
  if (knob(KNOB_G8_KORDER) != 0 && d.vec4 && d.ntaps > 1 && d.ctot % BK == 0 &&
      (int64_t)d.ntaps * d.ctot == d.K) {  // channel-block-major K order (CLSKD_G8_KORDER=0: packed)
    a.kt_taps = d.ntaps;
    a.kt_cpt = d.ctot / BK;
  }
  const size_t ctab_bytes = (size_t)(d.K / 4) * 8;  // VEC4 K-chunk table (dynamic LDS)
  CLSKD_CHECK_SHAPE(!d.vec4 || ctab_bytes <= 32 * 1024, "conv2d(f32): K=%d too long for the chunk table", d.K);
  // 8-wave 256-row tiles (A/B knob CLSKD_F32_WAVES=4|8): half the B staging per FLOP and two
  // waves per SIMD to hide the gather latency
  const int nw = knob(KNOB_F32_WAVES) == 8 ? 8 : 4;
#define LAUNCH(BN_, V_, O_, NW_)                                                             \
  do {                                                                                       \
    hipLaunchKernelGGL((conv_igemm_f32<BN_, V_, O_, NW_>),                                    \
                       dim3((unsigned)cdiv(M, 32 * NW_), (unsigned)cdiv(d.N, BN_)),           \
                       dim3(NW_ * 64), (V_) ? ctab_bytes : 0, st, a);                        \
    note_kernel_fn((const void*)conv_igemm_f32<BN_, V_, O_, NW_>);                           \
    note_kernel("conv_igemm_f32<%d,%s,%s,%d>", BN_, (V_) ? "true" : "false",                  \
                type_name<O_>(), NW_);                                                       \
  } while (0)
#define LAUNCH_NW(BN_, V_, O_) \
  do { if (nw == 8) LAUNCH(BN_, V_, O_, 8); else LAUNCH(BN_, V_, O_, 4); } while (0)
#define LAUNCH_O(BN_, V_)                                                   \
  do {                                                                      \
    if (d.out_dtype == CLSKD_BF16) LAUNCH_NW(BN_, V_, __bf16);              \
    else if (d.out_dtype == CLSKD_F16) LAUNCH_NW(BN_, V_, _Float16);        \
    else LAUNCH_NW(BN_, V_, float);                                         \
  } while (0)
  if (d.N <= 32) {
    if (d.vec4) LAUNCH_O(32, true); else LAUNCH_O(32, false);
  } else if (d.N <= 64) {
    if (d.vec4) LAUNCH_O(64, true); else LAUNCH_O(64, false);
  } else {
    if (d.vec4) LAUNCH_O(128, true); else LAUNCH_O(128, false);
  }
#undef LAUNCH_O
#undef LAUNCH_NW
#undef LAUNCH
  CLSKD_LAUNCH_CHECK("conv2d");
  return CLSKD_OK;
}
