// Implicit-GEMM convolution engine for bf16 BFTC activations (gfx950).
//
// Selected by in_dtype = CLSKD_BF16 (descriptor in include/clskd.h): the frozen teacher and the
// ReviewKD fusions keep their activations in bf16, so the A operand can be staged straight from
// HBM into LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane) without a register round trip.
// The K-table gather becomes a per-lane SOURCE address (the LDS destination of one wave
// instruction is linear: 8 rows x 128 B); out-of-bounds taps read a zero page.
//
// Tile BM=128 x BN x BK=64, 8 waves (4 for BN=32), v_mfma_f32_32x32x16_bf16 (fp32 accumulate).
// Three LDS stages, two K-tiles in flight: per K-tile every wave waits on a COUNTED vmcnt (its
// own DMAs for the tile it is about to read), then a raw s_barrier makes every wave's DMA
// visible; no __syncthreads (which would drain vmcnt to 0).  LDS rows are 128 B with the 16-B
// chunk XOR-swizzled by ((row>>1)&7): the DMA applies the inverse permutation on the source
// address, the ds_read_b128 fragment reads apply it on the LDS address (same involution), so
// every read lane group of 16 rows hits 16 distinct bank slots.  All LDS is one dynamic array.
#include <stdlib.h>

#include "common.h"

namespace clskd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ __attribute__((aligned(64))) unsigned char g_zero_page[64];

namespace v2 {
// Tile geometry: BM output rows x BK reduction columns per stage; LDS rows of BK bf16
// (ROWB = 2*BK bytes = CPR 16-B chunks); one DMA wave instruction fills RPD = 64/CPR rows.
// The 16-B chunk index is XOR-swizzled so the 16 rows a ds_read_b128 cycle serves hit 16
// distinct bank slots: 128-B rows pair up per 256-B bank line -> swizzle by (row>>1)&7;
// 64-B rows come four per line -> (row>>2)&3.
template <int BK>
__device__ __forceinline__ int swz(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}

template <typename T>
__device__ __forceinline__ T sel4(int s, T a0, T a1, T a2, T a3) {
  return s == 0 ? a0 : (s == 1 ? a1 : (s == 2 ? a2 : a3));
}

template <typename OutT>
__device__ __forceinline__ void store_out(OutT* p, float v);
template <>
__device__ __forceinline__ void store_out<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void store_out<__bf16>(__bf16* p, float v) { *p = (__bf16)v; }

__host__ __device__ constexpr int stage_bytes(int BM, int BK, int BN) { return (BM + BN) * BK * 2; }

// One 1-KiB LDS-DMA wave instruction: lane l copies 16 B from gsrc to lds_base + 16*l.
// Inline asm (cdna_hip_programming.md §5.7): hipcc neither tracks nor waits for it, so the
// pipeline's counted vmcnt waits are the only synchronisation.  M0 is set and restored inside.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
}  // namespace v2

struct ConvArgsV2 {
  clskd_conv_desc d;
  // K-tile visiting order (as conv_gemm8): channel-block-major when every K-tile lies in one tap
  int kt_taps, kt_cpt;
};

// Counted wait leaving `ahead` younger K-tiles of this wave's DMAs in flight (NG pieces per
// tile, NG - 1 for a wave without a B group in the last round); vmcnt takes immediates only.
template <int NG, int A>
__device__ __forceinline__ void wait_tiles(int ahead, bool fullB) {
  if constexpr (A <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (ahead >= A) {
      if (fullB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A * NG) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(A * (NG - 1)) : "memory");
    } else {
      wait_tiles<NG, A - 1>(ahead, fullB);
    }
  }
}

template <int BM, int BK, int BN, int NW, int NS, typename OutT, int DBG = 0>
__global__ __launch_bounds__(NW * 64) void conv_igemm_bf16_dma(const ConvArgsV2 args) {
  using namespace v2;
  const clskd_conv_desc& d = args.d;
  constexpr int NT = NW * 64;       // threads
  constexpr int ROWB = BK * 2;      // bytes per LDS row
  constexpr int CPR = ROWB / 16;    // 16-B chunks per row
  constexpr int RPD = 64 / CPR;     // rows per 1-KiB DMA wave instruction
  constexpr int WN = BM == 256 ? (BN >= 256 ? 4 : 2) : ((BN >= 128 || NW == 8) ? 2 : 1);
  constexpr int WM = NW / WN;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int SB = stage_bytes(BM, BK, BN);
  constexpr int NGA = BM / RPD / NW;  // A DMA instructions per wave per K-tile
  constexpr int NGB = (BN / RPD + NW - 1) / NW;  // B DMA instructions per wave per K-tile
  constexpr int NG = NGA + NGB;
  static_assert(TM >= 1 && TN >= 1 && NGA >= 1 && NGB >= 1 && WM * WN == NW, "tile / wave split");
  static_assert(BM / WM <= 128 && 128 % (BM / WM) == 0, "a wave's rows stay inside one 128-row half");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* stages = smem;
  int* rowinfo = reinterpret_cast<int*>(smem + NS * SB);        // [BM][4]: fi0, ti0, valid, -
  int* rowbase = rowinfo + BM * 4;                                   // [4 seg][BM] element offsets
  int64_t* out_row = reinterpret_cast<int64_t*>(rowbase + 4 * BM);   // [BM]
  int4* segtab = reinterpret_cast<int4*>(out_row + BM);              // [4]: ptr lo, ptr hi, F, T
  int2* ctab = reinterpret_cast<int2*>(segtab + 4);                  // [K/8] chunk entries

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)tile * BM;
  const int n0 = blockIdx.y * BN;
  const int nk = d.K / BK;
  const int64_t FoTo = (int64_t)d.Fo * d.To;

  // ---- per-block tables -------------------------------------------------------------------
  if (tid < BM) {
    const int64_t m = m0 + tid;
    const bool valid = m < M;
    const int64_t mm = valid ? m : 0;
    const int64_t b = mm / FoTo;
    const int64_t r = mm - b * FoTo;
    const int fo = (int)(r / d.To);
    const int to = (int)(r - (int64_t)fo * d.To);
    const int fi0 = fo * d.stride_f, ti0 = to * d.stride_t;
    rowinfo[tid * 4 + 0] = fi0;
    rowinfo[tid * 4 + 1] = ti0;
    rowinfo[tid * 4 + 2] = valid ? 1 : 0;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      rowbase[s * BM + tid] = (int)(b * d.seg[s].sB + (int64_t)fi0 * d.seg[s].sF + (int64_t)ti0 * d.seg[s].sT);
    out_row[tid] = valid ? b * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT : -1;
  }
  if (tid < 4) {
    const clskd_seg& g = d.seg[tid];
    const uint64_t pv = (uint64_t)(uintptr_t)g.ptr;
    segtab[tid] = make_int4((int)(unsigned)pv, (int)(unsigned)(pv >> 32), g.F, g.T);
  }
  for (int q = tid; q < d.K / 8; q += NT) {
    const clskd_ktab_entry e = d.ktab[q * 8];
    const int s = d.kseg[q * 8];
    ctab[q] = make_int2(e.off, (int)(((unsigned)e.dF & 0xFFFFu) | (((unsigned)e.dT & 0xFFu) << 16) |
                                     ((unsigned)s << 24)));
  }
  __syncthreads();

  const unsigned short* wgt = reinterpret_cast<const unsigned short*>(d.weight);
  const int prow = lane / CPR;  // row within an RPD-row DMA group
  const int ppos = lane % CPR;  // 16-B chunk position within the LDS row

  const uint64_t zero_addr = (uint64_t)(uintptr_t)g_zero_page;
  const unsigned stage_lds0 = __builtin_amdgcn_readfirstlane(lds_addr(stages));
  // Loop-invariant geometry of this lane's A rows (one per DMA group i): the per-K-tile source
  // address then costs ONE LDS read (the K-chunk entry) plus ALU — the issue step is no longer
  // a chain of dependent LDS round trips sitting between the barrier and the MFMAs.
  int a_fi0[NGA], a_ti0[NGA], a_c[NGA];
  bool a_valid[NGA];
  int a_rb[NGA][4];
#pragma unroll
  for (int i = 0; i < NGA; ++i) {
    const int r = (wave * NGA + i) * RPD + prow;
    a_c[i] = ppos ^ swz<BK>(r);
    const int4 ri = reinterpret_cast<const int4*>(rowinfo)[r];
    a_fi0[i] = ri.x;
    a_ti0[i] = ri.y;
    a_valid[i] = ri.z != 0;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) a_rb[i][sg] = rowbase[sg * BM + r];
  }
  // this wave's share of the B row groups: NGB, or NGB - 1 when the groups run out (uniform)
  const bool fullB = (wave + NW * (NGB - 1)) < BN / RPD;
  const uint64_t sp0 = (uint64_t)(uintptr_t)d.seg[0].ptr, sp1 = (uint64_t)(uintptr_t)d.seg[1].ptr;
  const uint64_t sp2 = (uint64_t)(uintptr_t)d.seg[2].ptr, sp3 = (uint64_t)(uintptr_t)d.seg[3].ptr;
  auto issue = [&](int kt, int stage) {
    uint64_t srcA[NGA], srcB[NGB];
#pragma unroll
    for (int i = 0; i < NGA; ++i) {
      const int2 ce = ctab[kt * CPR + a_c[i]];
      const int sg = (int)((unsigned)ce.y >> 24);
      const int dF = (int)(short)(ce.y & 0xFFFF);
      const int dT = (int)(signed char)((ce.y >> 16) & 0xFF);
      const int fi = a_fi0[i] + dF;
      const int ti = a_ti0[i] + dT;
      const int Fb = sel4(sg, d.seg[0].F, d.seg[1].F, d.seg[2].F, d.seg[3].F);
      const int Tb = sel4(sg, d.seg[0].T, d.seg[1].T, d.seg[2].T, d.seg[3].T);
      const bool ok = a_valid[i] && (unsigned)fi < (unsigned)Fb && (unsigned)ti < (unsigned)Tb;
      const uint64_t base = sel4(sg, sp0, sp1, sp2, sp3);
      const int rb = sel4(sg, a_rb[i][0], a_rb[i][1], a_rb[i][2], a_rb[i][3]);
      const int64_t eoff = (int64_t)rb + ce.x;
      srcA[i] = ok ? base + (uint64_t)(eoff * 2) : zero_addr;
    }
#pragma unroll
    for (int i = 0; i < NGB; ++i) {
      // B row groups are dealt round-robin over the waves; a wave past the last group in its
      // final round issues nothing for it (fullB false): no duplicate DMA pieces
      const int rg = (wave + NW * i) < BN / RPD ? (wave + NW * i) : 0;
      const int r = rg * RPD + prow;
      const int c = ppos ^ swz<BK>(r);
      const int n = n0 + r;
      srcB[i] = n < d.N ? (uint64_t)(uintptr_t)(wgt + (int64_t)n * d.K + kt * BK + c * 8) : zero_addr;
    }
    if constexpr (DBG == 1) return;  // timing experiment: no operand traffic
    // the DMAs, back to back
    const unsigned sl = stage_lds0 + stage * SB;
    if constexpr (DBG != 5 && DBG != 8) {  // DBG 5/8: timing experiments, A operand not staged
#pragma unroll
      for (int i = 0; i < NGA; ++i) glds16((const void*)srcA[i], sl + (wave * NGA + i) * 1024);
    }
    if constexpr (DBG != 4 && DBG != 7) {  // DBG 4/7: timing experiments, B operand not staged
#pragma unroll
      for (int i = 0; i < NGB; ++i) {
        if (i < NGB - 1 || fullB) glds16((const void*)srcB[i], sl + BM * ROWB + (wave + NW * i) * 1024);
      }
    }
  };

  // accumulators start at the bias (its loads are waited for here, once, before the pipeline)
  const int h = lane >> 5;
  const int l32 = lane & 31;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + l32;
    const float bv = (d.bias && n < d.N) ? d.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = bv;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // packed K-tile of the next issued K-tile: all taps of a channel block before the next block
  // (the rows a K-tile gathers are one tap from the previous K-tile's: still in L2)
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
  // prologue: NS-1 K-tiles in flight
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(next_kt(), t);

  for (int kt = 0; kt < nk; ++kt) {
    // wait for this wave's DMAs of tile kt; the (up to NS-2) younger tiles stay in flight
    // (per-wave piece count: NG, or NG - 1 for a wave without a B group in the last round)
    const int ahead = min(NS - 2, nk - 1 - kt);
    wait_tiles<NG, NS - 2>(ahead, fullB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NS - 1 < nk) issue(next_kt(), (kt + NS - 1) % NS);
    const unsigned char* sa = stages + (kt % NS) * SB;
    const unsigned char* sb = sa + BM * ROWB;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int c = 2 * s + h;  // lane half h takes k = 16s + 8h .. +8
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 32 + l32;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + row * ROWB + ((c ^ swz<BK>(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * (BN / WN) + j * 32 + l32;
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + row * ROWB + ((c ^ swz<BK>(row)) << 4));
      }
      if constexpr (DBG != 2 && DBG != 7 && DBG != 8) {  // DBG 2/7/8: timing experiments without the MFMAs
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j][0] += (float)af[i][0] * (float)bfr[j][0];
      }
    }
  }

  if (d.stats) {  // fused BatchNorm statistics: one fp64 partial per 128 output rows
    constexpr int HALVES = BM / 128;     // 128-row halves of this tile (host contract)
    constexpr int WPH = WM / HALVES;     // waves (along M) per half
    __syncthreads();  // all DMAs retired (vmcnt(0) on the last K-tile); stage LDS is free
    double* red = reinterpret_cast<double*>(smem);  // [WM][BN][2]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * (BN / WN) + j * 32 + l32;
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (out_row[row] >= 0) {
            const float v = acc[i][j][r];
            sm += v;
            sq = fmaf(v, v, sq);
          }
        }
      double ds = (double)sm + (double)__shfl_xor(sm, 32, 64);
      double dq = (double)sq + (double)__shfl_xor(sq, 32, 64);
      if (h == 0) {
        red[(wm * BN + col) * 2] = ds;
        red[(wm * BN + col) * 2 + 1] = dq;
      }
    }
    __syncthreads();
    const int64_t nblk128 = (M + 127) / 128;
    for (int idx = tid; idx < HALVES * BN; idx += NT) {
      const int hv = idx / BN, c = idx % BN;
      const int n = n0 + c;
      const int64_t blk = (int64_t)tile * HALVES + hv;
      if (n >= d.N || blk >= nblk128) continue;
      double S = 0.0, Q = 0.0;
#pragma unroll
      for (int w = 0; w < WPH; ++w) {
        S += red[((hv * WPH + w) * BN + c) * 2];
        Q += red[((hv * WPH + w) * BN + c) * 2 + 1];
      }
      d.stats[(blk * d.N + n) * 2] = S;
      d.stats[(blk * d.N + n) * 2 + 1] = Q;
    }
  }

  OutT* out = reinterpret_cast<OutT*>(d.out);
  // Vectorised epilogue: each wave stages its (converted) sub-tile in the freed stage LDS and
  // writes it back as 16-B row chunks — 4 dwordx4 stores per lane instead of 16 * TM * TN
  // scalar stores (the store tail was 12-14 % of a 576-deep layer).  Needs a channel-contiguous,
  // 16-B aligned output map; otherwise the scalar scatter below.
  constexpr int CH = 16 / (int)sizeof(OutT);  // channels per 16-B chunk
  constexpr int WR = BM / WM, WC = BN / WN;   // wave sub-tile
  constexpr int WBYTES = WR * WC * (int)sizeof(OutT);
  constexpr bool VEC_FITS = NW * WBYTES <= NS * SB && WC % CH == 0;
  const bool vec = VEC_FITS && DBG != 3 && d.oNlo == 1 && d.nlo >= d.N && d.N % CH == 0 &&
                   (((uintptr_t)d.out) & 15) == 0 && d.oB % CH == 0 && d.oF % CH == 0 &&
                   d.oT % CH == 0;
  if (vec) {
    __syncthreads();  // every wave's last fragment reads and the statistics scratch are done
    OutT* wt = reinterpret_cast<OutT*>(smem + wave * WBYTES);  // [WR][WC]
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          wt[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * WC + j * 32 + l32] = (OutT)acc[i][j][r];
    constexpr int CPRW = WC / CH;  // 16-B chunks per sub-tile row
#pragma unroll
    for (int q0 = 0; q0 < WR * CPRW; q0 += 64) {
      const int q = q0 + lane;
      const int rr = q / CPRW, cc = q % CPRW;
      const int64_t ro = out_row[wm * WR + rr];
      const int n = n0 + wn * WC + cc * CH;
      if (q < WR * CPRW && ro >= 0 && n < d.N) {
        uint4 v = *reinterpret_cast<const uint4*>(wt + rr * WC + cc * CH);
        if constexpr (sizeof(OutT) == 4) {
          if (d.accumulate) {  // data-gradient sums (fp32 out): out += conv
            const f32x4 o = *reinterpret_cast<const f32x4*>(out + ro + n);
            v = __builtin_bit_cast(uint4, __builtin_bit_cast(f32x4, v) + o);
          }
        }
        *reinterpret_cast<uint4*>(out + ro + n) = v;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + l32;
    if (n >= d.N) continue;
    const int64_t coff = (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t ro = out_row[row];
        if (DBG != 3 && ro >= 0) {
          float v = acc[i][j][r];
          if constexpr (sizeof(OutT) == 4)
            if (d.accumulate) v += reinterpret_cast<const float*>(out)[ro + coff];
          store_out<OutT>(out + ro + coff, v);
        }
      }
    }
  }
}

template <int BM, int BK, int BN, int NW, int S, typename OutT, int DBG = 0>
static int launch_v2(const clskd_conv_desc& d, hipStream_t st) {
  using namespace v2;
  const size_t lds = (size_t)S * stage_bytes(BM, BK, BN) + BM * 16 + 4 * BM * 4 + BM * 8 + 64 +
                     (size_t)(d.K / 8) * 8;
  if (lds > 160 * 1024) {
    set_error("conv2d(bf16): K=%d needs %zu B of LDS", d.K, lds);
    return CLSKD_E_SHAPE;
  }
  auto kern = conv_igemm_bf16_dma<BM, BK, BN, NW, S, OutT, DBG>;
  static bool attr_set = false;  // per instantiation
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  ConvArgsV2 a{d, 1, d.K / BK};
  if (knob(KNOB_G8_KORDER) != 0 && d.ntaps > 1 && d.ctot % BK == 0 && (int64_t)d.ntaps * d.ctot == d.K) {
    a.kt_taps = d.ntaps;
    a.kt_cpt = d.ctot / BK;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)cdiv(M, BM), (unsigned)cdiv(d.N, BN)), dim3(NW * 64), lds, st, a);
  note_kernel_fn((const void*)kern);
  note_kernel("conv_igemm_bf16_dma<%d,%d,%d,%d,%d,%s,%d>", BM, BK, BN, NW, S, type_name<OutT>(), DBG);
  return CLSKD_OK;
}

template <int NW, int S>
static int launch_nw(const clskd_conv_desc& d, hipStream_t st) {
  const bool f32out = d.out_dtype == CLSKD_F32;
  if (d.N <= 32) return f32out ? launch_v2<128, 64, 32, 4, S, float>(d, st) : launch_v2<128, 64, 32, 4, S, __bf16>(d, st);
  if (d.N <= 64) return f32out ? launch_v2<128, 64, 64, NW, S, float>(d, st) : launch_v2<128, 64, 64, NW, S, __bf16>(d, st);
  if (d.N <= 128) return f32out ? launch_v2<128, 64, 128, NW, S, float>(d, st) : launch_v2<128, 64, 128, NW, S, __bf16>(d, st);
  // BN = 256: 48 KB per stage, three stages fill the 160 KB LDS
  return f32out ? launch_v2<128, 64, 256, NW, 3, float>(d, st) : launch_v2<128, 64, 256, NW, 3, __bf16>(d, st);
}

// 256-row tiles, BK = 32, 16 waves: a third fewer staged bytes per FLOP than 128 x 256 x 64
template <int S128, int S256>
static int launch_big_s(const clskd_conv_desc& d, hipStream_t st) {
  const bool f32out = d.out_dtype == CLSKD_F32;
  if (d.N <= 64) return f32out ? launch_v2<256, 32, 64, 16, S128, float>(d, st) : launch_v2<256, 32, 64, 16, S128, __bf16>(d, st);
  if (d.N <= 128) return f32out ? launch_v2<256, 32, 128, 16, S128, float>(d, st) : launch_v2<256, 32, 128, 16, S128, __bf16>(d, st);
  return f32out ? launch_v2<256, 32, 256, 16, S256, float>(d, st) : launch_v2<256, 32, 256, 16, S256, __bf16>(d, st);
}

// Four stages for the 256-row tiles (three K-tiles in flight): 2-5 % over three on the
// encoder/ABF layers; five or six measured no better (tools/conv_micro.py, CLSKD sweep).
static int launch_big(const clskd_conv_desc& d, hipStream_t st) { return launch_big_s<4, 4>(d, st); }

// 8 waves (512 threads) per workgroup: twice the LDS-DMA issuers of a 4-wave tile — the
// engine is bound by DMA issue/latency, not MFMA (tools/conv_micro.py: 13-25 % faster for
// BN >= 64).  BN = 32 keeps 4 waves (four 32x32 MFMA tiles).  CLSKD_BF16_WAVES=4 selects the
// 4-wave tiles everywhere (A/B measurements).
int launch_conv_halo(const clskd_conv_desc& d, hipStream_t st, bool* launched);
int launch_conv_gemm8(const clskd_conv_desc& d, hipStream_t st, bool* launched);
#ifdef CLSKD_EXPERIMENTS
int launch_conv_halow(const clskd_conv_desc& d, hipStream_t st, bool* launched);
#endif

int launch_conv_bf16(const clskd_conv_desc& d, hipStream_t st) {
  const bool no_halo = knob(KNOB_NO_HALO) == 1;  // A/B switch: 1 keeps narrow layers on the engine
  // accumulating launches (fp32 out += conv: the split-product data gradients over bf16 hi / lo
  // planes) run the LDS-DMA engine, the one with the read-add-write epilogue
  if (d.accumulate) {
    CLSKD_CHECK_ARG(d.out_dtype == CLSKD_F32 && !d.stats && !d.bn_fold && d.in_dtype == CLSKD_BF16,
                    "conv2d(bf16): accumulate needs an fp32 output, bf16 operands, no statistics");
    return launch_nw<8, 3>(d, st);
  }
  if (!no_halo) {
    bool launched = false;
    const int rc = launch_conv_halo(d, st, &launched);
    if (rc != CLSKD_OK || launched) return rc;
  }
  const int dbg = knob(KNOB_BF16_DEBUG_MODE);
  {
    const int rc = experiment_guard("CLSKD_BF16_DEBUG_MODE", dbg);
    if (rc != CLSKD_OK) return rc;
  }
#ifdef CLSKD_EXPERIMENTS
  if (dbg == 0 && knob(KNOB_G8) < 10) {  // the wide layers: halo tiles with streamed weights
    bool launched = false;
    const int rc = launch_conv_halow(d, st, &launched);
    if (rc != CLSKD_OK || launched) return rc;
  }
#endif
  if (dbg == 0) {
    bool launched = false;
    const int rc = launch_conv_gemm8(d, st, &launched);
    if (rc != CLSKD_OK || launched) return rc;
  }
  // the generic fallback: every bf16 layer neither the halo kernel nor the persistent engine
  // takes (short or ragged clips, halo tiles that do not fit LDS; no launch in the C2-C5
  // censuses).  bf16 only: an f16 layer that reaches it is an error, never a silent bf16
  // computation
  CLSKD_CHECK_ARG(d.in_dtype == CLSKD_BF16,
                  "conv2d(f16): N=%d K=%d nseg=%d fits neither the halo kernel nor conv_gemm8", d.N,
                  d.K, d.nseg);
  const int nw = knob(KNOB_BF16_WAVES) == 4 ? 4 : 8;
  const int stages = knob(KNOB_BF16_STAGES) == 4 ? 4 : 3;  // experiment knob: 3 | 4
  const int tilecfg = knob(KNOB_BF16_TILE);  // A/B knob: 128 | 256 forces one row-tile height
#ifdef CLSKD_EXPERIMENTS
  // timing experiments only: 1 = no DMA, 2 = no MFMA, ... (wrong results)
  if (dbg == 1 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<128, 64, 256, 8, 3, __bf16, 1>(d, st);
  if (dbg == 2 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<128, 64, 256, 8, 3, __bf16, 2>(d, st);
  if (dbg == 1 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 3, __bf16, 1>(d, st);
  if (dbg == 2 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 3, __bf16, 2>(d, st);
  if (dbg == 3 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 3, __bf16, 3>(d, st);
  if (dbg == 4 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<256, 32, 256, 16, 4, __bf16, 4>(d, st);
  if (dbg == 5 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<256, 32, 256, 16, 4, __bf16, 5>(d, st);
  if (dbg == 4 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 4, __bf16, 4>(d, st);
  if (dbg == 5 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 4, __bf16, 5>(d, st);
  if (dbg == 7 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<256, 32, 256, 16, 4, __bf16, 7>(d, st);
  if (dbg == 8 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<256, 32, 256, 16, 4, __bf16, 8>(d, st);
  if (dbg == 7 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 4, __bf16, 7>(d, st);
  if (dbg == 8 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 4, __bf16, 8>(d, st);
  if (dbg == 6 && d.out_dtype == CLSKD_BF16 && d.N > 128) return launch_v2<256, 32, 256, 16, 4, __bf16, 0>(d, st);
  if (dbg == 6 && d.out_dtype == CLSKD_BF16 && d.N > 64) return launch_v2<256, 32, 128, 16, 4, __bf16, 0>(d, st);
#endif
  if (d.N > 32 && d.K % 32 == 0 && tilecfg != 128) {
    // 256-row tiles stage a third fewer bytes per FLOP (measured 1.1-1.25x faster per tile
    // worth of work) but halve the workgroup count: pick them unless the tail rounds eat the
    // gain — a 256-row tile costs ~1.6 rounds-equivalents of a 128-row tile, one workgroup per
    // CU either way.
    static const int ncu = [] {
      int v = 256;
      (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
      return v > 0 ? v : 256;
    }();
    const int64_t M = (int64_t)d.B * d.Fo * d.To;
    const int64_t ny = cdiv(d.N, d.N <= 64 ? 64 : d.N <= 128 ? 128 : 256);
    const int64_t r256 = cdiv(cdiv(M, 256) * ny, ncu), r128 = cdiv(cdiv(M, 128) * ny, ncu);
    if (tilecfg == 256 || 16 * r256 < 10 * r128) return launch_big(d, st);
  }
  if (stages == 4) return nw == 8 ? launch_nw<8, 4>(d, st) : launch_nw<4, 4>(d, st);
  return nw == 8 ? launch_nw<8, 3>(d, st) : launch_nw<4, 3>(d, st);
}

}  // namespace clskd
