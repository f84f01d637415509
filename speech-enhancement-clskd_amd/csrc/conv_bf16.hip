// Implicit-GEMM convolution engine, bf16 MFMA operands / fp32 accumulation (gfx950).
//
// Same descriptor and K-table gather as conv_igemm.hip (include/clskd.h), selected with
// compute = CLSKD_BF16 for the large-K layers (teacher encoder/decoder, ReviewKD 3x3 convs).
// Activations stay fp32 in HBM and are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) while staging
// into LDS; weights are pre-packed bf16 [N][K] with K padded to a multiple of 64.
//
// Tile BM=128 x BN x BK=64, 256 threads = 4 waves, v_mfma_f32_32x32x16_bf16.  Waves are laid out
// 2x2 (BN=128: 64x64 per wave) or 4x1 (BN<=64: 32xBN per wave).  LDS rows are 64 bf16 = 128 B;
// the 16-B chunk index is XOR-swizzled with ((row>>1)&7) so each ds_read_b128 lane group
// (16 rows, same chunk) hits 16 distinct bank slots.  One register-prefetched K-tile in flight,
// two LDS buffers, one barrier per K-tile.
#include "common.h"

namespace clskd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

namespace bf {
constexpr int BM = 128;
constexpr int BK = 64;
constexpr int ROWB = BK * 2;  // bytes per LDS row

__device__ __forceinline__ int chunk_swz(int row, int c) { return c ^ ((row >> 1) & 7); }

template <typename T>
__device__ __forceinline__ T sel4(int s, T a0, T a1, T a2, T a3) {
  return s == 0 ? a0 : (s == 1 ? a1 : (s == 2 ? a2 : a3));
}
}  // namespace bf

struct ConvArgsBF {
  clskd_conv_desc d;
};

template <int BN>
__global__ __launch_bounds__(256) void conv_igemm_bf16(const ConvArgsBF args) {
  using namespace bf;
  const clskd_conv_desc& d = args.d;
  constexpr int WN = (BN == 128) ? 2 : 1;   // waves along N
  constexpr int WM = 4 / WN;                // waves along M
  constexpr int TM = BM / WM / 32;          // 32x32 tiles per wave along M
  constexpr int TN = BN / WN / 32;          // 32x32 tiles per wave along N
  __shared__ __attribute__((aligned(16))) unsigned char As[2][BM * ROWB];
  __shared__ __attribute__((aligned(16))) unsigned char Bs[2][BN * ROWB];
  __shared__ int64_t out_row[BM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nk = d.K / BK;
  const int64_t FoTo = (int64_t)d.Fo * d.To;

  if (tid < BM) {
    int64_t m = m0 + tid;
    int64_t off = -1;
    if (m < M) {
      int64_t b = m / FoTo;
      int64_t r = m - b * FoTo;
      int fo = (int)(r / d.To);
      int to = (int)(r - (int64_t)fo * d.To);
      off = b * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT;
    }
    out_row[tid] = off;
  }

  // A staging: thread -> row (tid>>1), 32 consecutive k (8 quads) at (tid&1)*32
  const int arow = tid >> 1;
  const int ahalf = tid & 1;
  int rb, rfi, rti;
  bool rvalid;
  {
    int64_t m = m0 + arow;
    rvalid = m < M;
    int64_t mm = rvalid ? m : 0;
    int64_t b = mm / FoTo;
    int64_t r = mm - b * FoTo;
    int fo = (int)(r / d.To);
    int to = (int)(r - (int64_t)fo * d.To);
    rb = (int)b;
    rfi = fo * d.stride_f;
    rti = to * d.stride_t;
  }
  const int64_t rowbase0 = (int64_t)rb * d.seg[0].sB + (int64_t)rfi * d.seg[0].sF + (int64_t)rti * d.seg[0].sT;
  const int64_t rowbase1 = (int64_t)rb * d.seg[1].sB + (int64_t)rfi * d.seg[1].sF + (int64_t)rti * d.seg[1].sT;
  const int64_t rowbase2 = (int64_t)rb * d.seg[2].sB + (int64_t)rfi * d.seg[2].sF + (int64_t)rti * d.seg[2].sT;
  const int64_t rowbase3 = (int64_t)rb * d.seg[3].sB + (int64_t)rfi * d.seg[3].sF + (int64_t)rti * d.seg[3].sT;

  auto load_a = [&](int kt, f32x4 (&ra)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = kt * BK + ahalf * 32 + q * 4;
      const clskd_ktab_entry e = d.ktab[k];
      const int s = d.kseg[k];
      const float* sp = sel4(s, d.seg[0].ptr, d.seg[1].ptr, d.seg[2].ptr, d.seg[3].ptr);
      const int64_t rbase = sel4(s, rowbase0, rowbase1, rowbase2, rowbase3);
      const int Fb = sel4(s, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F);
      const int Tb = sel4(s, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T);
      const int fi = rfi + e.dF;
      const int ti = rti + e.dT;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (rvalid && fi >= 0 && fi < Fb && ti >= 0 && ti < Tb)
        v = *reinterpret_cast<const f32x4*>(sp + rbase + e.off);
      ra[q] = v;
    }
  };

  constexpr int NBL = BN * ROWB / 16 / 256;  // 16-B weight chunks per thread (BN*8/256)
  const __bf16* wgt = reinterpret_cast<const __bf16*>(d.weight);
  auto load_b = [&](int kt, u32x4 (&rbv)[NBL > 0 ? NBL : 1]) {
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + 256 * i;  // chunk index: row = idx>>3, chunk = idx&7
      const int n = n0 + (idx >> 3);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (n < d.N) v = *reinterpret_cast<const u32x4*>(wgt + (int64_t)n * d.K + kt * BK + (idx & 7) * 8);
      rbv[i] = v;
    }
  };

  auto store_tiles = [&](int buf, const f32x4 (&ra)[8], const u32x4 (&rbv)[NBL > 0 ? NBL : 1]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kq = ahalf * 8 + q;  // quad index 0..15 within the 64-wide row
      const int c = kq >> 1;
      bf16x4 h;
      h[0] = (__bf16)ra[q][0];
      h[1] = (__bf16)ra[q][1];
      h[2] = (__bf16)ra[q][2];
      h[3] = (__bf16)ra[q][3];
      *reinterpret_cast<bf16x4*>(&As[buf][arow * ROWB + chunk_swz(arow, c) * 16 + (kq & 1) * 8]) = h;
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx >> 3;
      *reinterpret_cast<u32x4*>(&Bs[buf][row * ROWB + chunk_swz(row, idx & 7) * 16]) = rbv[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[8];
  u32x4 rbv[NBL > 0 ? NBL : 1];
  load_a(0, ra);
  load_b(0, rbv);
  store_tiles(0, ra, rbv);
  __syncthreads();

  const int h = lane >> 5;
  const int l32 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      load_a(kt + 1, ra);
      load_b(kt + 1, rbv);
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = 2 * s + h;  // lane half h takes k = 16s + 8h .. +8
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 32 + l32;
        af[i] = *reinterpret_cast<const bf16x8*>(&As[buf][row * ROWB + chunk_swz(row, c) * 16]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 32 + l32;
        bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[buf][row * ROWB + chunk_swz(row, c) * 16]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1, ra, rbv);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + l32;
    if (n >= d.N) continue;
    const float bias = d.bias ? d.bias[n] : 0.f;
    const int64_t coff = (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t ro = out_row[row];
        if (ro >= 0) d.out[ro + coff] = acc[i][j][r] + bias;
      }
    }
  }
}

int launch_conv_bf16(const clskd_conv_desc& d, hipStream_t st) {
  ConvArgsBF a{d};
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const unsigned gx = (unsigned)cdiv(M, bf::BM);
  if (d.N <= 32)
    hipLaunchKernelGGL(conv_igemm_bf16<32>, dim3(gx, (unsigned)cdiv(d.N, 32)), dim3(256), 0, st, a);
  else if (d.N <= 64)
    hipLaunchKernelGGL(conv_igemm_bf16<64>, dim3(gx, (unsigned)cdiv(d.N, 64)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(conv_igemm_bf16<128>, dim3(gx, (unsigned)cdiv(d.N, 128)), dim3(256), 0, st, a);
  return 0;
}

}  // namespace clskd
