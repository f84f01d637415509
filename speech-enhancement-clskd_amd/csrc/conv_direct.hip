// Direct convolution for narrow GEMMs (few output channels or a short reduction): the layers
// where the implicit-GEMM engines re-read the im2col-expanded A tile through LDS while the
// MFMA units have almost nothing to do — DCCRN's first encoder layer (Cin = 2: K = 20),
// the last decoder layer (N = 2), the student's 8/16-channel layers and the ReviewKD 1x1
// channel lifts (K <= 64).
//
// Same descriptor, K table, output map and fused-BN-statistics protocol as the engines
// (include/clskd.h): one thread per output row (b, fo, to), 128 rows per block, so the
// statistics partials stats[tile][N][2] line up with conv_mblocks().  The K loop is
// uniform across the block: the K table (one entry per channel run of kvec) is staged in LDS,
// the packed weights are read with scalar loads (constant address space) and enter the VALU as
// SGPR operands — v_fma_f32 for fp32 runs, v_dot2c_f32_bf16 (bf16 pairs, fp32 accumulate) for
// bf16 runs.  Each row's A run is read straight from global memory (an L1/L2-resident
// neighbourhood) with a kvec-wide load, prefetched one run ahead.
#include "common.h"

namespace clskd {

struct DirectArgs {
  clskd_conv_desc d;
};

typedef __bf16 bf16x8d __attribute__((ext_vector_type(8)));
typedef float f32x2d __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T sel4d(int s, T a0, T a1, T a2, T a3) {
  return s == 0 ? a0 : (s == 1 ? a1 : (s == 2 ? a2 : a3));
}

template <typename OutT, int VW>
struct VecOf;
template <> struct VecOf<float, 4> { typedef f32x4 T; };
template <> struct VecOf<float, 2> { typedef f32x2d T; };
template <> struct VecOf<__bf16, 8> { typedef bf16x8d T; };
template <> struct VecOf<__bf16, 4> { typedef __bf16 T __attribute__((ext_vector_type(4))); };
template <> struct VecOf<__bf16, 2> { typedef __bf16 T __attribute__((ext_vector_type(2))); };
typedef _Float16 f16x8d __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2d __attribute__((ext_vector_type(2)));
template <> struct VecOf<_Float16, 8> { typedef f16x8d T; };
template <> struct VecOf<_Float16, 4> { typedef _Float16 T __attribute__((ext_vector_type(4))); };
template <> struct VecOf<_Float16, 2> { typedef f16x2d T; };

typedef __bf16 bf16x2d __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4d __attribute__((ext_vector_type(4)));
// uniform weight reads through the constant address space -> scalar (SMEM) loads, SGPR operands
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) float* cf32p;

template <int G, typename InT>
struct XRun;  // one run of G input channels as loaded
template <> struct XRun<8, __bf16> { bf16x8d v; };  // 8 bf16 = 4 packed pairs
template <> struct XRun<8, _Float16> { f16x8d v; };  // 8 IEEE halves = 4 packed pairs

// acc += x[2I] * w.lo + x[2I+1] * w.hi (fp32 accumulate): v_dot2c_f32_bf16 / v_dot2_f32_f16,
// the weight pair as one 32-bit (SGPR) word
template <int I, typename V>
__device__ __forceinline__ float dot2_pair(const V& x, uint32_t wbits, float a) {
  if constexpr (__is_same(V, f16x8d))
    return __builtin_amdgcn_fdot2(__builtin_shufflevector(x, x, 2 * I, 2 * I + 1),
                                  __builtin_bit_cast(f16x2d, wbits), a, false);
  else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 2 * I, 2 * I + 1),
                                           __builtin_bit_cast(bf16x2d, wbits), a, false);
}
template <> struct XRun<4, float> { f32x4 v; };
template <> struct XRun<2, float> { f32x2d v; };
template <> struct XRun<1, float> { float v; };

template <int G, typename InT>
__device__ __forceinline__ void zero_run(XRun<G, InT>& x) {
  if constexpr (G == 8) x.v = decltype(x.v){};
  else if constexpr (G == 4) x.v = f32x4{0.f, 0.f, 0.f, 0.f};
  else if constexpr (G == 2) x.v = f32x2d{0.f, 0.f};
  else x.v = 0.f;
}

template <int NP, int G, typename InT, typename OutT>
__global__ __launch_bounds__(128) void conv_direct_kernel(const DirectArgs args) {
  const clskd_conv_desc& d = args.d;
  extern __shared__ __attribute__((aligned(16))) unsigned char dsm[];
  const int K = d.K;
  const int nrun = K / G;
  int4* kl = reinterpret_cast<int4*>(dsm);                 // [nrun] {off, dF|dT<<16, seg, 0}
  float* red = reinterpret_cast<float*>(dsm + (size_t)nrun * 16);  // [128][NP+1] (stats)

  const int tid = threadIdx.x;
  for (int j = tid; j < nrun; j += 128) {
    const clskd_ktab_entry e = d.ktab[j * G];
    const int sg = d.kseg[j * G];
    const int FT = (int)(uint16_t)sel4d(sg, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F) |
                   (sel4d(sg, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T) << 16);
    kl[j] = make_int4(e.off, (int)(uint16_t)e.dF | ((int)e.dT << 16), sg, FT);
  }
  __syncthreads();

  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t m = (int64_t)tile * 128 + tid;
  const bool valid = m < M;
  const int64_t FoTo = (int64_t)d.Fo * d.To;
  const int64_t mm = valid ? m : 0;
  const int b = (int)(mm / FoTo);
  const int64_t r = mm - (int64_t)b * FoTo;
  const int fo = (int)(r / d.To);
  const int to = (int)(r - (int64_t)fo * d.To);
  const int fi0 = fo * d.stride_f, ti0 = to * d.stride_t;
  // this row's base address in every segment (the K loop only adds the run offset)
  // (segment s's base = rb0 + dl_s; a sum of selected deltas, not an indexed array, so the
  // compiler keeps it in registers)
  auto row_base = [&](int s) {
    return (int64_t)(uintptr_t)d.seg[s].ptr +
           ((int64_t)b * d.seg[s].sB + (int64_t)fi0 * d.seg[s].sF + (int64_t)ti0 * d.seg[s].sT) *
               (int64_t)sizeof(InT);
  };
  const int64_t rb0 = row_base(0);
  const int64_t dl1 = d.nseg > 1 ? row_base(1) - rb0 : 0;
  const int64_t dl2 = d.nseg > 2 ? row_base(2) - rb0 : 0;
  const int64_t dl3 = d.nseg > 3 ? row_base(3) - rb0 : 0;

  // branch-free run load: out-of-bounds taps (and rows past M) read a safe address and are
  // zeroed after the load, so the U loads of an iteration issue back to back
  // global address space: a generic pointer would make these FLAT loads, which count on lgkmcnt
  // too — every wait for a scalar weight load would then drain the whole run of input loads
  using GIn = const __attribute__((address_space(1))) InT;
  GIn* safe = reinterpret_cast<GIn*>((uintptr_t)d.seg[0].ptr);
  auto load = [&](int j, bool run_ok, XRun<G, InT>& x) {
    const int4 e = kl[j];
    const int dF = (int)(int16_t)(e.y & 0xffff), dT = e.y >> 16;
    const int Fb = e.w & 0xffff, Tb = (int)((unsigned)e.w >> 16);
    const int fi = fi0 + dF, ti = ti0 + dT;
    const bool ok = run_ok && valid && fi >= 0 && fi < Fb && ti >= 0 && ti < Tb;
    const int sg = __builtin_amdgcn_readfirstlane(e.z);  // uniform segment of this run
    const int64_t base = rb0 + (sg == 1 ? dl1 : 0) + (sg == 2 ? dl2 : 0) + (sg == 3 ? dl3 : 0);
    GIn* p = ok ? reinterpret_cast<GIn*>(base) + e.x : safe;
    x.v = *reinterpret_cast<const __attribute__((address_space(1))) decltype(x.v)*>(p);
    if constexpr (G == 8) {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      u4 w = __builtin_bit_cast(u4, x.v);
      w = ok ? w : u4{0u, 0u, 0u, 0u};
      x.v = __builtin_bit_cast(decltype(x.v), w);
    } else if constexpr (G == 1) {
      x.v = ok ? x.v : 0.f;
    } else {
#pragma unroll
      for (int g = 0; g < G; ++g) x.v[g] = ok ? x.v[g] : 0.f;
    }
  };

  float acc[NP];
#pragma unroll
  for (int n = 0; n < NP; ++n) acc[n] = (d.bias && n < d.N) ? d.bias[n] : 0.f;

  auto compute = [&](int j, const XRun<G, InT>& xc) {
    const cu32p wrun_u = (cu32p)d.weight + (int64_t)j * (G / 2 > 0 ? G / 2 : 1) * NP;
    const cf32p wrun_f = (cf32p)d.weight + (int64_t)j * G * NP;
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      if constexpr (G == 8) {
        // bf16 x bf16 pairs, fp32 accumulate: v_dot2c_f32_bf16 with the weight pair in an SGPR;
        // direct layout [K/2][NP] u32 pairs: this run's 4*NP words are contiguous
        const cu32p wp = wrun_u + n;
        float a = acc[n];
        a = dot2_pair<0>(xc.v, wp[0], a);
        a = dot2_pair<1>(xc.v, wp[NP], a);
        a = dot2_pair<2>(xc.v, wp[2 * NP], a);
        a = dot2_pair<3>(xc.v, wp[3 * NP], a);
        acc[n] = a;
      } else {
        // direct layout [K][NP] fp32: this run's G*NP weights are contiguous
        const cf32p wp = wrun_f + n;
        if constexpr (G == 1) {
          acc[n] = fmaf(xc.v, wp[0], acc[n]);
        } else {
#pragma unroll
          for (int q = 0; q < G; ++q) acc[n] = fmaf(xc.v[q], wp[q * NP], acc[n]);
        }
      }
    }
  };

  // U runs per iteration: all U loads in flight before the first use.  Runs past the end of
  // the K table (last iteration) repeat the last run with zeroed inputs: +0 contributions.
  constexpr int U = G >= 4 ? 8 : 16;
  for (int j0 = 0; j0 < nrun; j0 += U) {
    XRun<G, InT> x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool run_ok = j0 + u < nrun;
      load(run_ok ? j0 + u : nrun - 1, run_ok, x[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) compute(j0 + u < nrun ? j0 + u : nrun - 1, x[u]);
  }

  // the block's 128 x NP results in LDS (statistics and/or coalesced stores)
  const bool rows_contig = d.N == NP && d.oNlo == 1 && d.nlo >= NP && d.oT == NP &&
                           d.of_mul == 1 && d.of_add == 0 && d.oF == (int64_t)d.To * NP &&
                           d.oB == (int64_t)d.Fo * d.To * NP &&
                           ((uintptr_t)d.out % 16) == 0 && NP * sizeof(OutT) >= 16;
  if (d.stats || rows_contig) {
#pragma unroll
    for (int n = 0; n < NP; ++n) red[tid * (NP + 1) + n] = valid ? acc[n] : 0.f;
    __syncthreads();
  }
  if (d.stats) {  // fused BatchNorm statistics: fp64 column sums over the block's 128 rows
    for (int n = tid; n < d.N; n += 128) {
      double S = 0.0, Q = 0.0;
      for (int q = 0; q < 128; ++q) {
        const double v = (double)red[q * (NP + 1) + n];
        S += v;
        Q = fma(v, v, Q);
      }
      d.stats[((int64_t)tile * d.N + n) * 2] = S;
      d.stats[((int64_t)tile * d.N + n) * 2 + 1] = Q;
    }
  }
  if (rows_contig) {
    // output rows m0 .. m0+127 are one contiguous run of 128*NP elements: 16-B chunks
    constexpr int CH = 16 / sizeof(OutT);  // elements per chunk
    const int64_t m0 = (int64_t)tile * 128;
    const int rows = (int)min((int64_t)128, M - m0);
    OutT* dst = reinterpret_cast<OutT*>(d.out) + m0 * NP;
    typedef typename VecOf<OutT, CH>::T V;
    for (int c = tid; c < rows * NP / CH; c += 128) {
      const int row = (c * CH) / NP, col = (c * CH) % NP;
      V v;
      if (d.accumulate) {  // fp32 out only (host): data-gradient sums, out += conv
        const V o = *reinterpret_cast<const V*>(dst + (int64_t)c * CH);
#pragma unroll
        for (int i = 0; i < CH; ++i) v[i] = (OutT)(red[row * (NP + 1) + col + i] + (float)o[i]);
      } else {
#pragma unroll
        for (int i = 0; i < CH; ++i) v[i] = (OutT)red[row * (NP + 1) + col + i];
      }
      *reinterpret_cast<V*>(dst + (int64_t)c * CH) = v;
    }
    return;
  }

  if (!valid) return;
  OutT* outp = reinterpret_cast<OutT*>(d.out);
  const int64_t ro = (int64_t)b * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT;
  constexpr int VWMAX = 16 / sizeof(OutT);
  constexpr int VW = NP < VWMAX ? NP : VWMAX;
  const bool vec = d.N == NP && d.oNlo == 1 && d.nlo >= NP && d.oB % VW == 0 && d.oF % VW == 0 &&
                   d.oT % VW == 0 && ((uintptr_t)d.out % (VW * sizeof(OutT))) == 0;
  if (vec) {
    typedef typename VecOf<OutT, VW>::T V;
#pragma unroll
    for (int c = 0; c < NP; c += VW) {
      V v;
      if (d.accumulate) {
        const V o = *reinterpret_cast<const V*>(outp + ro + c);
#pragma unroll
        for (int i = 0; i < VW; ++i) v[i] = (OutT)(acc[c + i] + (float)o[i]);
      } else {
#pragma unroll
        for (int i = 0; i < VW; ++i) v[i] = (OutT)acc[c + i];
      }
      *reinterpret_cast<V*>(outp + ro + c) = v;
    }
  } else {
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      if (n < d.N) {
        const int64_t o = ro + (d.nlo >= NP ? (int64_t)n * d.oNlo
                                            : (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo);
        outp[o] = (OutT)(d.accumulate ? acc[n] + (float)outp[o] : acc[n]);
      }
    }
  }
}

static int np_of(int N) {
  return N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : N <= 16 ? 16 : N <= 32 ? 32 : 64;
}

static size_t direct_lds(const clskd_conv_desc& d, int NP, int G) {
  return (size_t)(d.K / G) * 16 + 128 * (NP + 1) * 4;  // K table + result tile
}

// Direct path policy (measured on MI355X against the MFMA engines, tools/conv_census.py):
// it wins for the 2-channel output layers (2-3x), short-K narrow layers and the 2-channel-input
// first encoder layer (K = 20 -> 32, N = 32: the fp32 engine's scalar gather path takes 135 us
// there); with N >= 32 and real K, or N = 16 with long K, the MFMA engines are faster.
// K <= 1024 bounds the LDS K table (16 KB).  accumulate (out += conv, fp32 out, no statistics):
// the data-gradient sums of the narrow decoder / encoder layers (C3 backward: the 2-channel
// mask-gradient gather into the 8-channel decoder input took 195 us per segment on the fp32 MFMA
// engine's scalar gather path).
bool conv_direct_ok(int N, int K) {
  return N >= 1 && K >= 1 && K <= 1024 &&
         (N <= 4 || (N <= 16 && K <= 128) || (N <= 32 && K <= 32));
}

template <int NP, int G, typename InT>
static void launch_np(const clskd_conv_desc& d, hipStream_t st) {
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const size_t lds = direct_lds(d, NP, G);
  DirectArgs a{d};
  if (d.out_dtype == CLSKD_F16) {
    hipLaunchKernelGGL((conv_direct_kernel<NP, G, InT, _Float16>), dim3((unsigned)cdiv(M, 128)),
                       dim3(128), lds, st, a);
    note_kernel_fn((const void*)conv_direct_kernel<NP, G, InT, _Float16>);
  } else if (d.out_dtype == CLSKD_BF16) {
    hipLaunchKernelGGL((conv_direct_kernel<NP, G, InT, __bf16>), dim3((unsigned)cdiv(M, 128)),
                       dim3(128), lds, st, a);
    note_kernel_fn((const void*)conv_direct_kernel<NP, G, InT, __bf16>);
  } else {
    hipLaunchKernelGGL((conv_direct_kernel<NP, G, InT, float>), dim3((unsigned)cdiv(M, 128)),
                       dim3(128), lds, st, a);
    note_kernel_fn((const void*)conv_direct_kernel<NP, G, InT, float>);
  }
  note_kernel("conv_direct_kernel<%d,%d,%s,%s>", NP, G, type_name<InT>(),
              d.out_dtype == CLSKD_BF16 ? "bf16" : d.out_dtype == CLSKD_F16 ? "f16" : "float");
}

template <int G, typename InT>
static void launch_g(const clskd_conv_desc& d, hipStream_t st) {
  if (d.N <= 2) launch_np<2, G, InT>(d, st);
  else if (d.N <= 4) launch_np<4, G, InT>(d, st);
  else if (d.N <= 8) launch_np<8, G, InT>(d, st);
  else if (d.N <= 16) launch_np<16, G, InT>(d, st);
  else if (d.N <= 32) launch_np<32, G, InT>(d, st);
  else launch_np<64, G, InT>(d, st);
}

int launch_conv_direct(const clskd_conv_desc& d, hipStream_t st) {
  CLSKD_CHECK_SHAPE(conv_direct_ok(d.N, d.K), "conv2d(direct): N=%d K=%d outside the direct path",
                    d.N, d.K);
  CLSKD_CHECK_ARG(((uintptr_t)d.weight & 15) == 0, "conv2d(direct): weight must be 16-byte aligned");
  CLSKD_CHECK_ARG(!d.accumulate || (d.out_dtype == CLSKD_F32 && !d.stats && !d.bn_fold),
                  "conv2d(direct): accumulate takes an fp32 output and no statistics");
  int g = d.kvec;
  if (g == 0) g = is_lowp(d.in_dtype) ? 8 : (d.vec4 ? 4 : 1);
  CLSKD_CHECK_SHAPE(d.K % g == 0, "conv2d(direct): K=%d not a multiple of kvec %d", d.K, g);
  if (d.in_dtype == CLSKD_BF16) {
    CLSKD_CHECK_SHAPE(g == 8, "conv2d(direct): bf16 segments need kvec 8");
    launch_g<8, __bf16>(d, st);
  } else if (d.in_dtype == CLSKD_F16) {
    CLSKD_CHECK_SHAPE(g == 8, "conv2d(direct): f16 segments need kvec 8");
    launch_g<8, _Float16>(d, st);
  } else {
    for (int s = 0; s < d.nseg; ++s) {
      const clskd_seg& sg = d.seg[s];
      CLSKD_CHECK_ARG(((uintptr_t)sg.ptr % (4 * g)) == 0 && sg.sB % g == 0 && sg.sF % g == 0 &&
                          sg.sT % g == 0,
                      "conv2d(direct): segment %d not aligned for kvec %d", s, g);
    }
    if (g == 4) launch_g<4, float>(d, st);
    else if (g == 2) launch_g<2, float>(d, st);
    else if (g == 1) launch_g<1, float>(d, st);
    else CLSKD_CHECK_SHAPE(false, "conv2d(direct): fp32 kvec %d unsupported", g);
  }
  return CLSKD_OK;
}

}  // namespace clskd

extern "C" int clskd_conv_direct_np(int32_t N) { return clskd::np_of(N); }
extern "C" int clskd_conv_direct_ok(int32_t N, int32_t K) { return clskd::conv_direct_ok(N, K) ? 1 : 0; }
