// Persistent, software-pipelined bf16 implicit-GEMM convolution for the wide teacher / ReviewKD
// layers (N > 64; gfx950).
//
// Same descriptor contract as the LDS-DMA engine in conv_bf16.hip (K-table gather of bf16 BFTC
// segments, packed [N][K] bf16 weights with K % 64 == 0, bias-initialised fp32 accumulators,
// fused per-128-row BatchNorm partials, out_row map).  What it changes, measured on the
// teacher shapes (tools/conv_micro.py; tools/g8_sweep.sh ablations):
//
//  * The one-tile-per-workgroup engines pay a fixed cost per tile — row tables with int64
//    divisions, the K-table and bias loads, the first K-tile's full memory round trip, the
//    BatchNorm-statistics and store epilogue — with nothing else on the CU to hide it (one
//    workgroup per CU): 12-20 us per tile round against 1.1-1.7 us per K-tile of MFMA work.
//    Here a grid of at most one workgroup per CU walks a list of tiles; the LDS-DMA pipeline
//    runs straight across tile boundaries (the next tile's first K-tile is in flight while the
//    current tile's last one computes and its epilogue runs), and the row tables of tile j+1
//    are built (double-buffered in LDS) while tile j runs.
//  * 8 waves (512 threads), BK = 64, tile BM x BN with each wave owning a 128x64 (256x256) or
//    64x64 (256x128) block of v_mfma_f32_32x32x16_bf16 accumulators; the K-tile is walked in
//    four 16-deep substeps with the NEXT substep's fragments read while the current one's MFMAs
//    run (two fragment register sets), one raw s_barrier per K-tile (DMA visibility + stage
//    reuse; no __syncthreads in the pipeline: its vmcnt(0) would drain the in-flight DMAs), the
//    K-tile's LDS-DMA pieces interleaved between the substeps.
//  * Two LDS stages; 128-B rows with the 16-B chunk XOR-swizzled by (row >> 1) & 7 on the DMA
//    source address and on the fragment read (conflict-free for the 32x32x16 operand reads).
//    One glds piece = 8 rows x 128 B; a lane's chunk position is the same in every piece it
//    issues, so the K-table entry of a K-tile is ONE LDS read per lane.
//  * Tiles are dealt to workgroups XCD-aware: each XCD's workgroups take one contiguous run of
//    M-tiles, so the rows concurrently gathered on an XCD (overlapping through the taps) share
//    its L2.
#include <stdlib.h>

#include <mutex>
#include <unordered_map>

#include "bnfold.h"
#include "common.h"

namespace clskd {

typedef short bf16x8s __attribute__((ext_vector_type(8)));

namespace g8 {

__device__ __attribute__((aligned(64))) unsigned char zero_page[64];

// One 1-KiB LDS-DMA wave instruction: lane l copies 16 B from gsrc to lds_base + 16*l.  Inline
// asm (cdna_hip_programming.md §5.7): hipcc neither tracks nor waits for it, so the counted
// vmcnt waits below are the only synchronisation.
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

// Tap-addressed pieces (TA): the buffer form of the LDS-DMA, four 1-KiB pieces per call.  Lane l
// copies 16 B from rsrc.base + voff[l] to m0 + 16*l (out-of-range offsets, >= num_records = 2^31,
// read as zeros: masked taps and N-tail weight rows cost no address arithmetic).  Piece p lands at
// lds_base + O0 + p * OS; m0 is saved and restored around the group (the compiler does not
// track it).
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned TA_OOB = 0x80000000u;
__device__ __forceinline__ i32x4 ta_rsrc(uint64_t base) {
  i32x4 r;
  r[0] = (int)(uint32_t)base;
  r[1] = (int)((uint32_t)(base >> 32) & 0xFFFFu);  // stride 0: raw buffer
  r[2] = (int)TA_OOB;                               // num_records (bytes)
  r[3] = 0x00020000;                                // gfx9 data format: 32 bits
  return r;
}
template <int O0, int OS>
__device__ __forceinline__ void bdma4(unsigned v0, unsigned v1, unsigned v2, unsigned v3, i32x4 rs,
                                      unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_add_u32 m0, %1, %7\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %3, %2, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %8\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %4, %2, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %9\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %5, %2, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %10\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %6, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_base), "s"(rs), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "n"(O0), "n"(O0 + OS),
        "n"(O0 + 2 * OS), "n"(O0 + 3 * OS)
      : "memory");
}

template <int O0, int OS>
__device__ __forceinline__ void bdma2(unsigned v0, unsigned v1, i32x4 rs, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_add_u32 m0, %1, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %3, %2, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %6\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %4, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_base), "s"(rs), "v"(v0), "v"(v1), "n"(O0), "n"(O0 + OS)
      : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <typename T>
__device__ __forceinline__ T sel4(int s, T a0, T a1, T a2, T a3) {
  return s == 0 ? a0 : (s == 1 ? a1 : (s == 2 ? a2 : a3));
}

// raw workgroup barrier that leaves LDS-DMA in flight: this wave's LDS reads/writes retired
// first (lgkmcnt), then s_barrier; the compiler may not move memory operations across it
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// vmcnt takes immediates only: wait until at most n of this wave's VMEM ops are outstanding
template <int MAXN>
__device__ __forceinline__ void wait_vm(int n) {
  if constexpr (MAXN <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= MAXN) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXN) : "memory");
    else wait_vm<MAXN - 1>(n);
  }
}

// Row table of one tile (double-buffered in LDS).
template <int BM>
struct RowTable {
  int4 info[BM];     // fi0, ti0, valid, -
  int base[4][BM];   // per-segment element offset of the row
  int64_t orow[BM];  // output element offset (-1: past M)
  unsigned inv[BM];  // TA: bit t * nseg + s set when tap t of segment s reads outside the input
};

}  // namespace g8

struct ConvArgsG8 {
  clskd_conv_desc d;
  int n_mt, ntiles;  // M-tiles per N-block, tiles in the list
  // K-tile visiting order: kt_taps x kt_cpt K-tiles, visited channel-block-major (all taps of
  // 64-channel block c, then block c + 1) when every K-tile lies inside one tap (kt_taps = the
  // tap count, kt_cpt = K-tiles per tap); kt_taps = 1, kt_cpt = K / 64 is the packed order.
  int kt_taps, kt_cpt;
  BnFoldArgs f;  // folded BatchNorm finalize (f.acc != nullptr; needs one N-tile: N <= BN)
  // Stream-K (sk_cnt != nullptr): the ntiles x nk K-tile units are split into gridDim.x equal
  // contiguous ranges; a tile whose units fall in two ranges (never more: ntiles >= grid) is
  // finished by the workgroup that arrives second (per-tile ticket), which adds the other's
  // fp32 partial (written through sc1 into its slot of sk_ws) — one commutative add, so the
  // result does not depend on arrival order.  Tickets and ready flags are zero at rest.
  float* sk_ws;        // [grid][2][BM * BN] partial accumulators, register order
  unsigned* sk_ready;  // [grid][2]
  unsigned* sk_cnt;    // [ntiles]
};

typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ void sk_store4(f32x4v v, g8::i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ f32x4v sk_load4(g8::i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
constexpr int SK_SC1 = 16;  // buffer cache-policy bits: sc1 (write-through / L1-bypassing, gfx950)

// BM x BN tile, 8 waves as WM x WN, BK-deep K-tiles (64: 128-B LDS rows; 32: 64-B rows) in NS
// LDS stages (NS - 1 K-tiles in flight), the DMA pieces of a K-tile issued over the first PHI
// 16-deep substeps.  DBG (timing experiments only, wrong results): 1 = no LDS-DMA, 2 = no MFMA,
// 3 = neither, 4 = B operand only (no A gather), 5 = A operand only.  Correct-result variants:
// 6 = s_setprio 1 around each substep's MFMA cluster, 7 = static priority 1 for waves 4-7, 8 = both;
// 9 = no DMA wait inside the stream (timing only: DMA latency vs issue cost).
// TA = 1 (tap-addressed pieces, round 5): for tap-structured layers (K = ntaps x ctot, every
// K-tile inside one tap and segment) each piece's source is a per-(tile, piece) lane offset plus
// a per-K-tile buffer base (kinfo table, uniform), with a per-row tap-validity mask instead of
// per-piece 64-bit bounds arithmetic: ~12 VALU per K-tile instead of ~120.  TA bit 1 (TA = 3):
// the stream-K deal (ConvArgsG8::sk_cnt) compiled in; its bookkeeping costs registers, so only
// the launches that split tiles run that instantiation.
// DBG >= 16 (round 6, TA instances, experiments library only): ablation flags ABL = DBG - 16 —
// 1 no LDS-DMA, 2 no MFMA, 4 no fragment reads (opaque registers), 8 no epilogue (statistics and
// stores), 16 A pieces only, 32 B pieces only, 64 no DMA wait inside the stream, 128 no output
// stores (statistics kept), 256 no statistics (stores kept).  Wrong results.
template <int BM, int BN, int WM, int BK, int NS, int PHI, typename OutT, int DBG = 0, int PF = 1, int NWV = 8,
          int EB = 0, typename InT = __bf16, int PP = 0, int TA = 0>
__global__ __launch_bounds__(NWV * 64) void conv_gemm8_kernel(const ConvArgsG8 args) {
  using namespace g8;
  const clskd_conv_desc& d = args.d;
  constexpr int NW = NWV, NT = NWV * 64;
  constexpr int ROWB = 2 * BK;               // LDS row bytes
  constexpr int CPR = ROWB / 16;             // 16-B chunks per row
  constexpr int RPP = 64 / CPR;              // rows per 1-KiB DMA piece
  constexpr int NSUB = BK / 16;              // 16-deep MFMA substeps per K-tile
  constexpr int WN = NW / WM;
  constexpr int WR = BM / WM, WC = BN / WN;  // wave block
  constexpr int FM = WR / 32, FN = WC / 32;  // 32x32 tiles per wave
  constexpr int NGA = BM / RPP / NW, NGB = BN / RPP / NW;
  constexpr int G = NGA + NGB;               // DMA pieces per wave per K-tile
  constexpr int GP = (G + PHI - 1) / PHI;
  constexpr int SB = (BM + BN) * ROWB;       // stage bytes
  static_assert(BK == 32 || BK == 64, "K-tile depth");
  static_assert(WM * WN == NW && FM >= 1 && FN >= 1, "tile split");
  static_assert((BM / RPP) % NW == 0 && (BN / RPP) % NW == 0 && NGA >= 1, "DMA piece split");
  static_assert(PHI >= 1 && PHI <= NSUB && NSUB % 2 == 0, "issue substeps");
  static_assert(NS >= 2 && WM * BN * 16 <= SB, "statistics scratch fits one stage");
  static_assert(!(TA & 1) || (BK == 64 && NGA == 4 && (NGB == 4 || NGB == 2) && PHI == 2 && PP == 0 &&
                               (DBG == 0 || DBG >= 16)),
                "tap-addressed pieces: 256-row tiles, two issue substeps");
  constexpr int ABL = DBG >= 16 ? DBG - 16 : 0;
  constexpr bool NO_DMA = DBG == 1 || DBG == 3 || (ABL & 1);
  constexpr bool NO_MFMA = DBG == 2 || DBG == 3 || (ABL & 2);
  constexpr bool NO_FRAG = (ABL & 4) != 0;
  constexpr bool NO_EPI = (ABL & 8) != 0;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* stages = smem;
  RowTable<BM>* tabs = reinterpret_cast<RowTable<BM>*>(smem + NS * SB);  // [2]
  float* bias_l = reinterpret_cast<float*>(tabs + 2);                    // [N]
  int2* ctab = reinterpret_cast<int2*>(bias_l + ((d.N + 3) & ~3));       // [K/8]
  int4* kinfo = reinterpret_cast<int4*>(ctab);  // TA: [K/BK] {A base lo, hi, mask bit, -}

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int nk = d.K / BK;
  const int64_t FoTo = (int64_t)d.Fo * d.To;

  // ---- this workgroup's tile list (XCD-aware contiguous runs) ------------------------------
  const int grid = gridDim.x, b = blockIdx.x;
  int t_first = 0, t_step = 1, ntl;
  const bool sk = (TA & 2) != 0 && PP == 0 && args.sk_cnt != nullptr;  // compile-time off unless TA bit 1
  // stream-K: logical index (the workgroups of one XCD take consecutive ranges), the K-tile
  // range [kb0, nk) of the first tile and [0, ke1) of the last
  const int lidx = (grid & 7) == 0 ? (b & 7) * (grid >> 3) + (b >> 3) : b;
  int kb0 = 0, ke1 = nk;
  if (sk) {
    const int64_t U = (int64_t)args.ntiles * nk;
    const int64_t u0 = U * lidx / grid, u1 = U * (lidx + 1) / grid;
    ntl = 0;
    if (u1 > u0) {
      t_first = (int)(u0 / nk);
      kb0 = (int)(u0 - (int64_t)t_first * nk);
      const int tl = (int)((u1 - 1) / nk);
      ke1 = (int)(u1 - (int64_t)tl * nk);
      ntl = tl - t_first + 1;
    }
  } else if ((grid & 7) == 0 && args.ntiles >= grid) {
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
  const bool fold = args.f.acc != nullptr;
  if (ntl == 0) {  // whole workgroup: no barrier is left waiting
    if (fold)  // it still takes its ticket (a zero contribution); flag in the (unused) stages
      bnfold_commit(args.f, 0, [](int, double& S, double& Q) { S = Q = 0.0; },
                    reinterpret_cast<int*>(smem), b, grid);
    return;
  }
  auto tile_mt = [&](int j) { return (t_first + j * t_step) % args.n_mt; };
  auto tile_nt = [&](int j) { return (t_first + j * t_step) / args.n_mt; };

  auto build_table = [&](int j, int buf) {
    RowTable<BM>& tb = tabs[buf];
    if (tid < BM) {
      const int64_t m = (int64_t)tile_mt(j) * BM + tid;
      const bool valid = m < M;
      const int64_t mm = valid ? m : 0;
      const int64_t bb = mm / FoTo;
      const int64_t r = mm - bb * FoTo;
      const int fo = (int)(r / d.To);
      const int to = (int)(r - (int64_t)fo * d.To);
      const int fi0 = fo * d.stride_f, ti0 = to * d.stride_t;
      tb.info[tid] = make_int4(fi0, ti0, valid ? 1 : 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        tb.base[s][tid] = (int)(bb * d.seg[s].sB + (int64_t)fi0 * d.seg[s].sF + (int64_t)ti0 * d.seg[s].sT);
      tb.orow[tid] = valid ? bb * d.oB + (int64_t)(fo * d.of_mul + d.of_add) * d.oF + (int64_t)to * d.oT : -1;
      if constexpr ((TA & 1) != 0) {
        unsigned m = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          if (t < d.ntaps) {
#pragma unroll
            for (int sg = 0; sg < 2; ++sg) {
              if (sg < d.nseg) {
                const int fi = fi0 + d.tap_df[t], ti = ti0 + d.tap_dt[t];
                const bool ok = valid && (unsigned)fi < (unsigned)d.seg[sg].F && (unsigned)ti < (unsigned)d.seg[sg].T;
                m |= (ok ? 0u : 1u) << (t * d.nseg + sg);
              }
            }
          }
        }
        tb.inv[tid] = m;
      }
    }
  };

  // ---- layer tables: K-chunk entries, bias; row tables of the first two tiles ---------------
  if constexpr ((TA & 1) != 0) {
    // per packed K-tile: the A buffer base (segment pointer + the K-tile's first entry's element
    // offset: tap displacement + channel) and the row-mask bit of its (tap, segment)
    for (int q = tid; q < nk; q += NT) {
      const clskd_ktab_entry e = d.ktab[q * BK];
      const int s = d.kseg[q * BK];
      const int t = (q * BK) / d.ctot;
      const uint64_t a = (uint64_t)(uintptr_t)(s ? d.seg[1].ptr : d.seg[0].ptr) + (uint64_t)(int64_t)e.off * 2u;
      kinfo[q] = make_int4((int)(uint32_t)a, (int)(uint32_t)(a >> 32), t * d.nseg + s, s);
    }
  } else {
    for (int q = tid; q < d.K / 8; q += NT) {
      const clskd_ktab_entry e = d.ktab[q * 8];
      const int s = d.kseg[q * 8];
      ctab[q] = make_int2(e.off, (int)(((unsigned)e.dF & 0xFFFFu) | (((unsigned)e.dT & 0xFFu) << 16) |
                                       ((unsigned)s << 24)));
    }
  }
  for (int n = tid; n < d.N; n += NT) bias_l[n] = d.bias ? d.bias[n] : 0.f;
  build_table(0, 0);
  if (ntl > 1) build_table(1, 1);
  __syncthreads();

  // ---- per-lane DMA geometry (reloaded when the DMA stream moves on to another tile) ---------
  // Piece i of this wave covers tile rows (i*NW + wave)*RPP .. +RPP; lane -> row lane/CPR, LDS
  // chunk position lane%CPR, source chunk position ^ swizzle(row):
  //   BK 64: swizzle (row >> 1) & 7 = (wave & 1) * 4 + lane / 16
  //   BK 32: swizzle (row >> 2) & 3 = (lane / 16) & 3
  // Per A piece: (fi0, ti0) packed in one register (an invalid row carries fi0 = -32768, out of
  // every bound) and the row's element offset in segments 0 and 1 (the kernel takes <= 2).
  const int csrc = BK == 64 ? ((lane & 7) ^ (((wave & 1) << 2) + (lane >> 4))) : ((lane & 3) ^ ((lane >> 4) & 3));
  const int prow = lane / CPR;
  int a_ft[NGA], a_rb0[NGA], a_rb1[NGA];
  int b_n0 = 0, geo_tile = -1;
  // TA: per piece the row's tap-invalid mask and byte offsets (chunk swizzle folded in) into
  // each segment; the weight rows' byte offsets (out of range past N)
  unsigned a_inv[NGA], a_vb0[NGA], a_vb1[NGA], b_vo[NGB];  // dead unless TA
  const unsigned short* wgt = reinterpret_cast<const unsigned short*>(d.weight);
  auto load_geometry = [&](int j) {
    const RowTable<BM>& tb = tabs[j & 1];
    if constexpr ((TA & 1) != 0) {
#pragma unroll
      for (int i = 0; i < NGA; ++i) {
        const int r = (i * NW + wave) * RPP + prow;
        a_inv[i] = tb.inv[r];
        a_vb0[i] = (unsigned)tb.base[0][r] * 2u + (unsigned)csrc * 16u;
        a_vb1[i] = (unsigned)tb.base[1][r] * 2u + (unsigned)csrc * 16u;
      }
#pragma unroll
      for (int i = 0; i < NGB; ++i) {
        const int n = tile_nt(j) * BN + (i * NW + wave) * RPP + prow;
        b_vo[i] = n < d.N ? ((unsigned)n * (unsigned)d.K + (unsigned)csrc * 8u) * 2u : TA_OOB;
      }
      geo_tile = j;
      return;
    }
#pragma unroll
    for (int i = 0; i < NGA; ++i) {
      const int r = (i * NW + wave) * RPP + prow;
      const int4 ri = tb.info[r];
      a_ft[i] = (int)(((unsigned)(ri.z ? ri.x : -32768) << 16) | ((unsigned)ri.y & 0xFFFFu));
      a_rb0[i] = tb.base[0][r];
      a_rb1[i] = tb.base[1][r];
    }
    b_n0 = tile_nt(j) * BN + wave * RPP + prow;
    geo_tile = j;
  };

  const uint64_t zero_addr = (uint64_t)(uintptr_t)g8::zero_page;
  const unsigned stage_lds0 = __builtin_amdgcn_readfirstlane(lds_addr(stages));
  const uint64_t sp0 = (uint64_t)(uintptr_t)d.seg[0].ptr, sp1 = (uint64_t)(uintptr_t)d.seg[1].ptr;
  struct KEnt {
    int off, dF, dT, Fb, Tb, s1;
  };
  auto kdecode = [&](int2 ce) -> KEnt {
    KEnt e;
    e.s1 = (int)((unsigned)ce.y >> 24);
    e.off = ce.x;
    e.dF = (int)(short)(ce.y & 0xFFFF);
    e.dT = (int)(signed char)((ce.y >> 16) & 0xFF);
    e.Fb = e.s1 ? d.seg[1].F : d.seg[0].F;
    e.Tb = e.s1 ? d.seg[1].T : d.seg[0].T;
    return e;
  };
  // source address of piece g (A pieces first, then B) of K-tile kt (of the geometry's tile)
  auto piece_src = [&](int g, int kt, const KEnt& e) -> uint64_t {
    if (g < NGA) {
      const int fi = (a_ft[g] >> 16) + e.dF;
      const int ti = (int)(short)(a_ft[g] & 0xFFFF) + e.dT;
      const bool ok = (unsigned)fi < (unsigned)e.Fb && (unsigned)ti < (unsigned)e.Tb;
      const int rb = e.s1 ? a_rb1[g] : a_rb0[g];
      const uint64_t base = e.s1 ? sp1 : sp0;
      const uint64_t a = base + (uint64_t)(int64_t)(rb + e.off) * 2u;
      const uint64_t msk = 0ull - (uint64_t)ok;  // branch-free select of the zero page
      return (a & msk) | (zero_addr & ~msk);
    }
    const int n = b_n0 + (g - NGA) * NW * RPP;
    const uint64_t a = (uint64_t)(uintptr_t)wgt +
                       ((uint64_t)(uint32_t)n * (uint32_t)d.K + (uint32_t)(kt * BK + csrc * 8)) * 2u;
    const uint64_t msk = 0ull - (uint64_t)(n < d.N);
    return (a & msk) | (zero_addr & ~msk);
  };
  auto dst = [&](int g, int s) -> unsigned {
    const unsigned sl = stage_lds0 + s * SB;
    return g < NGA ? sl + (g * NW + wave) * 1024 : sl + BM * ROWB + ((g - NGA) * NW + wave) * 1024;
  };

  const int h = lane >> 5, l32 = lane & 31;
  f32x16 acc[FM][FN];
  auto k_begin = [&](int j) { return j == 0 ? kb0 : 0; };  // K-tile range of tile j (stream-K)
  auto k_end = [&](int j) { return j == ntl - 1 ? ke1 : nk; };
  auto init_acc = [&](int j) {
    const int nb = tile_nt(j) * BN;
    const bool with_bias = k_begin(j) == 0;  // a split tile's bias is in its first piece only
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      const int n = nb + wn * WC + jj * 32 + l32;
      const float bv = (n < d.N && with_bias) ? bias_l[n] : 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = bv;
    }
  };
  init_acc(0);

  // fragment reads of substep s (k = 16s .. 16s+15) of the stage at `sa`
  auto swz = [](int row) { return BK == 64 ? ((row >> 1) & 7) : ((row >> 2) & 3); };
  auto read_frags = [&](const unsigned char* sa, int s, bf16x8s (&af)[FM], bf16x8s (&bfr)[FN]) {
    if constexpr (NO_FRAG) {  // ablation: opaque registers instead of LDS reads
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" : "=v"(af[i]));
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) asm volatile("" : "=v"(bfr[jj]));
      return;
    }
    const unsigned char* sb = sa + BM * ROWB;
    const int c = 2 * s + h;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * WR + i * 32 + l32;
      af[i] = *reinterpret_cast<const bf16x8s*>(sa + row * ROWB + ((c ^ swz(row)) << 4));
    }
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      const int row = wn * WC + jj * 32 + l32;
      bfr[jj] = *reinterpret_cast<const bf16x8s*>(sb + row * ROWB + ((c ^ swz(row)) << 4));
    }
  };
  auto mfmas = [&](const bf16x8s (&af)[FM], const bf16x8s (&bfr)[FN]) {
    if constexpr (!NO_MFMA) {
      if constexpr (DBG == 6 || DBG == 8) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
          acc[i][jj] = mfma16<InT>(af[i], bfr[jj], acc[i][jj]);
      if constexpr (DBG == 6 || DBG == 8) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) asm volatile("" ::"v"(bfr[jj]));
    }
  };

  // ---- stream of K-tiles over the tile list: K-tile w belongs to tile w / nk ---------------------
  int total = 0;
  for (int j = 0; j < ntl; ++j) total += k_end(j) - k_begin(j);
  // packed K-tile of the next issued stream K-tile: the stream visits each tile's K-tiles
  // channel-block-major (tap q of block c = packed K-tile q * kt_cpt + c), so consecutive K-tiles
  // gather rows shifted by one tap — the rows the CU (and its XCD) fetched one K-tile earlier
  // are still in L2; the packed tap-major order came back to a row only after kt_cpt K-tiles.
  const int kt_taps = args.kt_taps, kt_cpt = args.kt_cpt;
  int it_tap = kb0 % kt_taps, it_cb = kb0 / kt_taps;  // visit index kb0 (stream-K start)
  int it_tile = 0, kt_tile = 0;  // tile of the K-tile next_kt() returned (no division per K-tile)
  auto next_kt = [&]() {
    const int k = it_tap * kt_cpt + it_cb;
    kt_tile = it_tile;
    if (++it_tap == kt_taps) {
      it_tap = 0;
      if (++it_cb == kt_cpt) {
        it_cb = 0;
        ++it_tile;
      }
    }
    return k;
  };
  // issue every piece of stream K-tile w into its stage (geometry moved to its tile first)
  // TA: the uniform per-K-tile state (A / B buffer resources, mask bit, segment)
  struct TaK {
    i32x4 ra, rb;
    unsigned bit;
    bool s1;
  };
  auto ta_k = [&](int kt) -> TaK {
    const int4 ki = kinfo[kt];
    const unsigned lo = __builtin_amdgcn_readfirstlane(ki.x), hi = __builtin_amdgcn_readfirstlane(ki.y);
    const unsigned bit = __builtin_amdgcn_readfirstlane(ki.z);
    const unsigned s1 = __builtin_amdgcn_readfirstlane(ki.w);
    TaK t;
    t.ra = ta_rsrc(((uint64_t)hi << 32) | lo);
    t.rb = ta_rsrc((uint64_t)(uintptr_t)wgt + (uint64_t)kt * (BK * 2));
    t.bit = bit;
    t.s1 = s1 != 0;
    return t;
  };
  // TA: pieces of part p (0: the four A pieces, 1: the four B pieces) into stage sn
  auto ta_issue = [&](int part, const TaK& k, int sn) {
    const unsigned sl = stage_lds0 + sn * SB + wave * 1024;
    if (part == 0) {
      unsigned v[NGA];
#pragma unroll
      for (int i = 0; i < NGA; ++i)
        v[i] = (k.s1 ? a_vb1[i] : a_vb0[i]) | (((a_inv[i] >> k.bit) & 1u) << 31);
      bdma4<0, NW * 1024>(v[0], v[1], v[2], v[3], k.ra, sl);
    } else {
      if constexpr (NGB == 4)
        bdma4<BM * ROWB, NW * 1024>(b_vo[0], b_vo[1], b_vo[2 % NGB], b_vo[3 % NGB], k.rb, sl);
      else
        bdma2<BM * ROWB, NW * 1024>(b_vo[0], b_vo[1 % NGB], k.rb, sl);
    }
  };
  auto issue_all = [&](int w) {
    const int kt = next_kt(), jt = kt_tile;
    if (jt != geo_tile) load_geometry(jt);
    if constexpr ((TA & 1) != 0) {
      const TaK k = ta_k(kt);
      ta_issue(0, k, w % NS);
      ta_issue(1, k, w % NS);
    } else {
      const KEnt e = kdecode(ctab[kt * CPR + csrc]);
#pragma unroll
      for (int g = 0; g < G; ++g) glds16((const void*)piece_src(g, kt, e), dst(g, w % NS));
    }
  };
  if (!NO_DMA) {
#pragma unroll
    for (int w = 0; w < NS - 1; ++w)
      if (w < total) issue_all(w);
  }
  g8::wait_vm<(NS - 2) * G>(min(NS - 2, total - 1) * G);
  raw_barrier();

  constexpr int NSET = PF + 1;
  static_assert(PF >= 1 && PF < NSUB, "fragment prefetch distance");
  bf16x8s fa[NSET][FM], fb[NSET][FN];
  auto read_head = [&](const unsigned char* sa) {  // the first PF substeps of a K-tile
#pragma unroll
    for (int s = 0; s < PF; ++s) read_frags(sa, s, fa[s], fb[s]);
  };
  if constexpr (!PP) read_head(stages);
  if constexpr (DBG == 7 || DBG == 8)
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  int gk = 0;  // stream index of the K-tile being computed
  double fS = 0.0, fQ = 0.0;  // fold: thread tid < HALVES*BN owns (half tid / BN, column tid % BN)
  for (int j = 0; j < ntl; ++j) {
    if constexpr (PP) {
      // Ping-pong K loop (cdna_hip_programming.md §5 8-phase template, T3-T5): every 16-deep
      // substep is a phase {LOAD: this substep's fragments + this wave's share of the next
      // K-tile's LDS-DMA pieces; barrier; MFMA cluster at priority 1; barrier}.  Waves w and
      // w + 4 share a SIMD; group 1 (waves 4-7) runs one barrier behind group 0, so on every
      // SIMD one wave's MFMA cluster covers the other wave's LDS reads, DMA issue and address
      // VALU.  The groups re-align (group 0's extra barrier) for the tile epilogue.
      static_assert(NS == 2 && NWV == 8 && PF == 1, "ping-pong: two stages, 8 waves");
      const bool lag = wave >= 4;
      if (lag) raw_barrier();
      for (int kt = 0; kt < nk; ++kt, ++gk) {
        const unsigned char* sa = stages + (gk % NS) * SB;
        const int wi = gk + 1;  // the K-tile whose pieces this K-tile issues
        const bool do_issue = wi < total;
        int kti = 0;
        KEnt e{};
        if (do_issue) {
          const int jt = wi / nk;
          kti = next_kt();
          if (jt != geo_tile) load_geometry(jt);
          e = kdecode(ctab[kti * CPR + csrc]);
        }
        const int sn = wi % NS;
        constexpr int GH = (G + 1) / 2;  // pieces per issuing phase (phases 0 and 1)
#pragma unroll
        for (int s = 0; s < NSUB; ++s) {
          read_frags(sa, s, fa[0], fb[0]);
          if (s < 2 && do_issue) {
#pragma unroll
            for (int g = s * GH; g < (s + 1) * GH && g < G; ++g)
              glds16((const void*)piece_src(g, kti, e), dst(g, sn));
          }
          // the next K-tile's pieces (issued in phases 0-1) landed before the barrier that
          // every wave passes ahead of the next K-tile's first fragment read
          if (s == NSUB - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          raw_barrier();
          __builtin_amdgcn_s_setprio(1);
          mfmas(fa[0], fb[0]);
          __builtin_amdgcn_s_setprio(0);
          raw_barrier();
        }
      }
      if (!lag) raw_barrier();  // re-align the groups: the epilogue runs in lockstep
    } else
    for (int kt = 0, nkj = k_end(j) - k_begin(j); kt < nkj; ++kt, ++gk) {
      const unsigned char* sa = stages + (gk % NS) * SB;
      // the K-tile issued during this one: stream gk + NS - 1
      const int wi = gk + NS - 1;
      const bool do_issue = wi < total && !NO_DMA;
      int kti = 0;
      KEnt e{};
      TaK tk{};
      if (do_issue) {
        kti = next_kt();
        const int jt = kt_tile;
        if (jt != geo_tile) load_geometry(jt);
        if constexpr ((TA & 1) != 0)
          tk = ta_k(kti);
        else
          e = kdecode(ctab[kti * CPR + csrc]);
      }
      const int sn = wi % NS;
      auto issue = [&](int part) {
        if constexpr ((TA & 1) != 0) {
          if (part < PHI && do_issue && !((ABL & 16) && part == 1) && !((ABL & 32) && part == 0))
            ta_issue(part, tk, sn);
          return;
        }
        if (part < PHI && do_issue) {
#pragma unroll
          for (int g = part * GP; g < (part + 1) * GP && g < G; ++g) {
            if ((DBG == 4 && g < NGA) || (DBG == 5 && g >= NGA)) continue;  // A- / B-only timing
            glds16((const void*)piece_src(g, kti, e), dst(g, sn));
          }
        }
      };
      // PF + 1 fragment register sets: substep s + PF is read while substep s computes; the
      // sched_barriers pin that (the scheduler would otherwise hoist every read and spill)
      // the next K-tile's pieces (this wave's) landed — younger K-tiles stay in flight; then
      // every wave's are visible and every wave is done reading this K-tile's stage
      auto k_boundary = [&]() {
        if ((DBG == 9 || (ABL & 64)) && gk + 1 < total) {  // timing only: never wait for the DMA inside the stream
        } else if ((DBG >= 4 && DBG <= 5) || gk + 1 >= total) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          g8::wait_vm<(NS - 2) * G>(min(NS - 2, total - 2 - gk) * G);
        }
        raw_barrier();
        if (kt + 1 < nkj) read_head(stages + ((gk + 1) % NS) * SB);
      };
      // EB: the boundary sits before the last substep's MFMAs (its fragments are already in
      // registers), so the next K-tile's head reads return under those MFMAs instead of after
      // the barrier with the MFMA pipe idle
      static_assert(!EB || (NSUB - 1) % NSET >= PF, "EB: the last substep's set must not be a head set");
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        if (EB && s == NSUB - 1) k_boundary();
        if (s + PF < NSUB) read_frags(sa, s + PF, fa[(s + PF) % NSET], fb[(s + PF) % NSET]);
        mfmas(fa[s % NSET], fb[s % NSET]);
        issue(s);  // behind the MFMAs: the K-entry read / address ALU overlap them
        __builtin_amdgcn_sched_barrier(0);
      }
      if (!EB) k_boundary();
    }

    // ---- tile epilogue: the stage of the K-tile just computed is free ------------------------
    unsigned char* scratch = stages + ((gk - 1) % NS) * SB;
    const RowTable<BM>& tb = tabs[j & 1];
    const int64_t m0 = (int64_t)tile_mt(j) * BM;
    const int n0 = tile_nt(j) * BN;
    bool finish = true;
    if (sk) {
      // stream-K: a tile split between this range and a neighbouring one (lidx - 1 when this
      // piece does not start at K-tile 0, else lidx + 1)
      const bool split = k_begin(j) > 0 || k_end(j) < nk;
      const int X = t_first + j;
      const int other = k_begin(j) > 0 ? lidx - 1 : lidx + 1;
      // slots: the piece at the start of a range (it does not begin at K-tile 0) uses slot 0, the
      // piece at its end slot 1 (ranges are >= nk units long: never both in one tile)
      const bool at_start = k_begin(j) > 0;
      const int my_slot = lidx * 2 + (at_start ? 0 : 1);
      const int o_slot = other * 2 + (at_start ? 1 : 0);
      int* flag = reinterpret_cast<int*>(scratch);
      bool last = true;
      if (split) {
        if (tid == 0) {
          const unsigned t = __hip_atomic_fetch_add(args.sk_cnt + X, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *flag = t != 0;  // second arrival: finish the tile
        }
        raw_barrier();
        last = *flag != 0;
        raw_barrier();  // every wave has read the flag before the scratch stage is reused
      }
      const i32x4 wrs = ta_rsrc((uint64_t)(uintptr_t)args.sk_ws);
      constexpr int SLAB = BM * BN * 4;
      // a lane's 16-B chunk: lane * 16 (the only per-lane part) + a uniform (SGPR) offset
      const int lvo = lane * 16;
      auto soff = [&](int slot, int i, int jj, int q) {
        return __builtin_amdgcn_readfirstlane(slot * SLAB + (((wave * FM + i) * FN + jj) * 4 + q) * 1024);
      };
      if (!last) {
        // publish: write-through stores, every wave drained, then one ready flag
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int jj = 0; jj < FN; ++jj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              f32x4v v;
              v[0] = acc[i][jj][4 * q];
              v[1] = acc[i][jj][4 * q + 1];
              v[2] = acc[i][jj][4 * q + 2];
              v[3] = acc[i][jj][4 * q + 3];
              sk_store4(v, wrs, lvo, soff(my_slot, i, jj, q), SK_SC1);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        raw_barrier();
        if (tid == 0) __hip_atomic_store(args.sk_ready + my_slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        finish = false;
      } else if (split) {
        // the other piece's ticket came first: its partial is published (or about to be: that
        // workgroup is running and waits for nothing) — poll its flag, then sc1 loads
        if (tid == 0) {
          while (__hip_atomic_load(args.sk_ready + o_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
            __builtin_amdgcn_s_sleep(2);
          __hip_atomic_store(args.sk_ready + o_slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(args.sk_cnt + X, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        raw_barrier();
      }
      // the add runs on every path (straight-line code: the accumulators stay in place): a tile
      // finished here without a partial reads out-of-range offsets, i.e. zeros, and moves nothing
      const int lsrc = (split && last) ? lvo : (int)TA_OOB;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
#pragma unroll
          for (int q = 0; q < 4; q += 2) {
            const f32x4v v0 = sk_load4(wrs, lsrc, soff(o_slot, i, jj, q), SK_SC1);
            const f32x4v v1 = sk_load4(wrs, lsrc, soff(o_slot, i, jj, q + 1), SK_SC1);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              acc[i][jj][4 * q + e] += v0[e];
              acc[i][jj][4 * q + 4 + e] += v1[e];
            }
            __builtin_amdgcn_sched_barrier(0);
          }
    }
    if (finish && (d.stats || fold) && !NO_EPI && !(ABL & 256)) {  // fused BatchNorm statistics: one fp64 partial per 128 output rows
      constexpr int HALVES = BM / 128;
      constexpr int WPH = WM / HALVES;  // waves along M per 128-row half
      double* red = reinterpret_cast<double*>(scratch);  // [WM][BN][2]
      // rows of this lane's accumulators: wm*WR + 4h + (a compile-time offset); the ones at or
      // past `lim` lie beyond M (only in the last M-tile: a uniform branch skips the checks)
      const int64_t left = M - m0 - wm * WR - 4 * h;
      const int lim = left < BM ? (int)left : BM;
      const bool full = __builtin_amdgcn_readfirstlane(M - m0 >= BM ? 1 : 0) != 0;
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const int col = wn * WC + jj * 32 + l32;
        float sm = 0.f, sq = 0.f;
        if (full) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float v = acc[i][jj][r];
              sm += v;
              sq = fmaf(v, v, sq);
            }
        } else {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float v = (i * 32 + (r & 3) + 8 * (r >> 2)) < lim ? acc[i][jj][r] : 0.f;
              sm += v;
              sq = fmaf(v, v, sq);
            }
        }
        const double ds = (double)sm + (double)__shfl_xor(sm, 32, 64);
        const double dq = (double)sq + (double)__shfl_xor(sq, 32, 64);
        if (h == 0) {
          red[(wm * BN + col) * 2] = ds;
          red[(wm * BN + col) * 2 + 1] = dq;
        }
      }
      raw_barrier();
      if (fold) {  // the workgroup's running sums (tiles in list order)
        if (tid < HALVES * BN) {
          const int hv = tid / BN, c = tid % BN;
#pragma unroll
          for (int w = 0; w < WPH; ++w) {
            fS += red[((hv * WPH + w) * BN + c) * 2];
            fQ += red[((hv * WPH + w) * BN + c) * 2 + 1];
          }
        }
      }
      const int64_t nblk128 = (M + 127) / 128;
      for (int idx = tid; idx < (fold ? 0 : HALVES * BN); idx += NT) {
        const int hv = idx / BN, c = idx % BN;
        const int n = n0 + c;
        const int64_t blk = m0 / 128 + hv;
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
      raw_barrier();  // the statistics scratch is read before the output staging reuses it
    }

    // output: each wave stages one 32x32 accumulator tile at a time in its slice of the scratch
    // stage and writes it back as 16-B row chunks (else direct stores: a wave instruction then
    // still writes 32 consecutive channels of two rows)
    OutT* out = reinterpret_cast<OutT*>(d.out);
    constexpr int CH = 16 / (int)sizeof(OutT);
    constexpr int UB = 32 * 32 * (int)sizeof(OutT);  // bytes per staged tile
    static_assert(NW * UB <= SB, "epilogue staging");
    const bool vec = d.oNlo == 1 && d.nlo >= d.N && d.N % CH == 0 && (((uintptr_t)d.out) & 15) == 0 &&
                     d.oB % CH == 0 && d.oF % CH == 0 && d.oT % CH == 0;
    if (!finish || NO_EPI || (ABL & 128)) {
      // the other piece's workgroup writes this tile (or the ablation skips the stores)
    } else if (vec) {
      OutT* wt = reinterpret_cast<OutT*>(scratch + wave * UB);  // [32][32], this wave's
      constexpr int CPRW = 32 / CH;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) {
#pragma unroll
          for (int r = 0; r < 16; ++r) wt[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + l32] = (OutT)acc[i][jj][r];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: tile written
#pragma unroll
          for (int q0 = 0; q0 < 32 * CPRW; q0 += 64) {
            const int q = q0 + lane;
            const int rr = q / CPRW, cc = q % CPRW;
            const int64_t ro = tb.orow[wm * WR + i * 32 + rr];
            const int n = n0 + wn * WC + jj * 32 + cc * CH;
            if (ro >= 0 && n < d.N)
              *reinterpret_cast<uint4*>(out + ro + n) = *reinterpret_cast<const uint4*>(wt + rr * 32 + cc * CH);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: tile read back
        }
    } else {
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const int n = n0 + wn * WC + jj * 32 + l32;
        if (n >= d.N) continue;
        const int64_t coff = (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t ro = tb.orow[row];
            if (ro >= 0) out[ro + coff] = (OutT)acc[i][jj][r];
          }
      }
    }
    if (j + 1 < ntl) {
      // every wave is done with tile j's row table and the scratch stage: build tile j+2's table
      // into the freed buffer (the DMA stream reaches tile j+2 only after >= 1 more barrier)
      raw_barrier();
      if (j + 2 < ntl) build_table(j + 2, j & 1);
      raw_barrier();
      init_acc(j + 1);
      if constexpr (!PP) read_head(stages + (gk % NS) * SB);
    }
  }
  if (fold) {  // the two 128-row halves in a fixed order, then the folded finalize
    static_assert(BM / 128 * BN <= NT, "one (half, column) pair per thread");
    constexpr int HALVES = BM / 128;
    double* fin = reinterpret_cast<double*>(stages);  // [HALVES][BN][2]; every stage is free
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < HALVES * BN) {
      fin[tid * 2] = fS;
      fin[tid * 2 + 1] = fQ;
    }
    __syncthreads();
    int* flag = reinterpret_cast<int*>(fin + HALVES * BN * 2);
    bnfold_commit(args.f, d.N, [&](int n, double& S, double& Q) {
      S = 0.0;
      Q = 0.0;
#pragma unroll
      for (int hv = 0; hv < HALVES; ++hv) {
        S += fin[(hv * BN + n) * 2];
        Q += fin[(hv * BN + n) * 2 + 1];
      }
    }, flag, b, grid);
  }
}

// ---- stream-K workspace: one per HIP stream (launches on one stream are ordered; two streams'
// launches may run together, so they never share partial slabs, tickets or flags).  Allocated
// at the first launch on a stream outside graph capture (or by clskd_stream_prepare).  A launch
// made during graph capture never takes the stream's own workspace: a graph's replays run on
// other streams (the executor's, hipGraphLaunch's) and two graphs captured on one stream may be
// replayed concurrently (clskd.graph.AheadStepExecutor), so a workspace baked into a capture no
// longer belongs to one stream's ordered launches.  A capture gets workspaces of its own instead:
// clskd_capture_scope_begin (before the capture starts) allocates one per stream the capture will
// launch on and binds them to the calling thread; launches captured on another stream, or with no
// scope bound, run the data-parallel deal.  The scope's owner frees it with the graph.
constexpr int SK_MAX_GRID = 256, SK_MAX_TILES = 1 << 16;
struct SkWs {
  float* ws;           // [SK_MAX_GRID][2][256 * 256] fp32
  unsigned* ready;     // [SK_MAX_GRID][2], then the tickets [SK_MAX_TILES]; zero at rest
};
// Whether this thread's last conv_gemm8 launch ran the stream-K deal (clskd_conv_last_stream_k).
static thread_local int g_last_sk = 0;
static void note_stream_k(bool on) { g_last_sk = on ? 1 : 0; }

static std::mutex g_sk_mu;
static std::unordered_map<hipStream_t, SkWs> g_sk;
// a graph capture's own workspaces (clskd_capture_scope_begin), bound to the capturing thread
struct SkScope {
  std::unordered_map<hipStream_t, SkWs> ws;
};
static thread_local SkScope* g_sk_scope = nullptr;

// zero at rest: the flags and tickets are cleared before the workspace is handed out
static bool sk_alloc(SkWs& w, hipStream_t st, bool sync) {
  const size_t wsb = (size_t)SK_MAX_GRID * 2 * 256 * 256 * 4, fb = (size_t)(SK_MAX_GRID * 2 + SK_MAX_TILES) * 4;
  w = SkWs{};
  if (hipMalloc(&w.ws, wsb) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (hipMalloc(&w.ready, fb) != hipSuccess || hipMemsetAsync(w.ready, 0, fb, st) != hipSuccess ||
      (sync && hipStreamSynchronize(st) != hipSuccess)) {
    (void)hipGetLastError();
    (void)hipFree(w.ws);
    if (w.ready) (void)hipFree(w.ready);
    w = SkWs{};
    return false;
  }
  return true;
}

static const SkWs* sk_workspace(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (cs != hipStreamCaptureStatusNone) {  // the capture's own workspace, if it has one
    if (!g_sk_scope) return nullptr;
    auto it = g_sk_scope->ws.find(st);
    return it == g_sk_scope->ws.end() ? nullptr : &it->second;
  }
  std::lock_guard<std::mutex> lk(g_sk_mu);
  auto it = g_sk.find(st);
  if (it != g_sk.end()) return &it->second;
  SkWs w{};
  if (!sk_alloc(w, st, false)) return nullptr;
  return &(g_sk[st] = w);
}

template <int BM, int BN, int WM, int BK, int NS, int PHI, typename OutT, int DBG = 0, int PF = 1, int NWV = 8,
          int EB = 0, typename InT = __bf16, int PP = 0, int TA = 0>
static int launch_g8(const clskd_conv_desc& d, hipStream_t st) {
  using namespace g8;
  constexpr int SB = (BM + BN) * 2 * BK;
  if (d.bn_fold && d.N > BN) {  // the fold epilogue keeps one channel per tile column
    set_error("conv2d(bf16 g8): folded BatchNorm needs N=%d <= the %d-column tile", d.N, BN);
    return CLSKD_E_ARG;
  }
  const size_t lds = NS * (size_t)SB + 2 * sizeof(RowTable<BM>) + (size_t)((d.N + 3) & ~3) * 4 +
                     (size_t)(d.K / 8) * 8;
  if (lds > 160 * 1024) {
    set_error("conv2d(bf16 g8): K=%d N=%d needs %zu B of LDS", d.K, d.N, lds);
    return CLSKD_E_SHAPE;
  }
  auto kern = conv_gemm8_kernel<BM, BN, WM, BK, NS, PHI, OutT, DBG, PF, NWV, EB, InT, PP, TA>;
  static bool attr_set = false;  // per instantiation
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  static const int ncu = [] {
    int v = 256;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
    return v > 0 ? v : 256;
  }();
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int64_t n_mt = cdiv(M, BM), n_nt = cdiv(d.N, BN);
  const int64_t ntiles = n_mt * n_nt;
  // one tile per workgroup when they all fit; otherwise whole XCD groups of workgroups for the
  // contiguous-run tile deal
  // CLSKD_G8_GRID caps the workgroup count (leaves CUs to concurrent streams; A/B knob)
  const int cap = knob(KNOB_G8_GRID) > 0 ? knob(KNOB_G8_GRID) : ncu;
  const int ncap = cap > 0 && cap < ncu ? cap : ncu;
  const int grid = ntiles <= ncap ? (int)ntiles : (ncap >= 8 ? (ncap & ~7) : ncap);
  ConvArgsG8 a{d, (int)n_mt, (int)ntiles, 1, d.K / BK, make_bnfold(d), nullptr, nullptr, nullptr};
  // stream-K when the data-parallel deal leaves a partial last round: the K-tile units split
  // evenly over the grid.  Each workgroup hands one fp32 partial (BM x BN x 4 B) to a neighbour
  // and takes one back; every workgroup does so at about the same time, so the grid moves
  // grid x 2 partials through memory in two bursts (64 MB each for 256 x 256 tiles on 256 CUs):
  // SK_COST = 12 K-tiles, fitted to the teacher layers (profiles/r5_g8_sk_ab.txt: enc3, 2.5
  // rounds, measured 5 % slower with stream-K, enc4 / dec1 at 1.26 rounds 12-17 % faster)
  // A capped grid (CLSKD_G8_GRID: the concurrent four-stream step) keeps the data-parallel deal:
  // there the other streams' kernels fill the CUs a partial last round leaves idle, and the
  // partial hand-off is extra memory traffic (measured: C2 step 5.36 vs 5.30 ms with stream-K,
  // profiles/r5_g8_sk_ab.txt).  CLSKD_G8_SK=2 (tests) splits on any grid.
  const int skm = knob(KNOB_G8_SK);
  if (TA == 1 && (skm == 2 || (skm == 1 && ncap == ncu)) && grid >= 8 && grid <= SK_MAX_GRID && (grid & 7) == 0 &&
      ntiles >= grid && ntiles <= SK_MAX_TILES && ntiles % grid != 0) {
    constexpr int64_t SK_COST = 12;
    const int64_t nk = d.K / BK;
    // CLSKD_G8_SK=2 (tests, A/B): whenever the deal splits, whatever the cost model says
    if (skm == 2 || cdiv(ntiles * nk, (int64_t)grid) + SK_COST < cdiv(ntiles, (int64_t)grid) * nk) {
      if (const SkWs* w = sk_workspace(st)) {
        a.sk_ws = w->ws;
        a.sk_ready = w->ready;
        a.sk_cnt = w->ready + SK_MAX_GRID * 2;
      }
    }
  }
  // channel-block-major K order when every K-tile lies inside one tap (CLSKD_G8_KORDER=0: packed)
  if (knob(KNOB_G8_KORDER) != 0 && d.ntaps > 1 && d.ctot % BK == 0 && (int64_t)d.ntaps * d.ctot == d.K) {
    a.kt_taps = d.ntaps;
    a.kt_cpt = d.ctot / BK;
  }
  const void* kfn = (const void*)kern;
  if constexpr (TA == 1) {
    if (a.sk_cnt) {  // the stream-K instantiation
      auto kern_sk = conv_gemm8_kernel<BM, BN, WM, BK, NS, PHI, OutT, DBG, PF, NWV, EB, InT, PP, 3>;
      static bool attr_sk = false;
      if (!attr_sk) {
        (void)hipFuncSetAttribute((const void*)kern_sk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_sk = true;
      }
      kfn = (const void*)kern_sk;
      hipLaunchKernelGGL(kern_sk, dim3((unsigned)grid), dim3(NWV * 64), lds, st, a);
    }
  }
  if (kfn == (const void*)kern) hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NWV * 64), lds, st, a);
  note_kernel_fn(kfn);
  if constexpr (TA != 0)  // every template argument, as rocprofv3 names the instance (TA 3: stream-K)
    note_kernel("conv_gemm8_kernel<%d,%d,%d,%d,%d,%d,%s,%d,%d,%d,%d,%s,%d,%d>", BM, BN, WM, BK, NS, PHI,
                type_name<OutT>(), DBG, PF, NWV, EB, type_name<InT>(), PP, a.sk_cnt ? 3 : 1);
  else if constexpr (__is_same(InT, _Float16))
    note_kernel("conv_gemm8_kernel<%d,%d,%d,%d,%d,%d,%s,%d,%d,%d,%d,f16%s>", BM, BN, WM, BK, NS, PHI,
                type_name<OutT>(), DBG, PF, NWV, EB, PP ? ",pp" : "");
  else
    note_kernel("conv_gemm8_kernel<%d,%d,%d,%d,%d,%d,%s,%d,%d,%d,%d%s>", BM, BN, WM, BK, NS, PHI,
                type_name<OutT>(), DBG, PF, NWV, EB, PP ? ",bf16,pp" : "");
  note_stream_k(a.sk_cnt != nullptr);
  return CLSKD_OK;
}

// Tap-addressed pieces (TA) apply: a tap-structured K table whose every 64-deep K-tile lies
// inside one tap and one segment, at most 32 (tap, segment) mask bits, and every row's / weight
// row's byte offset below 2^31 (buffer offsets; 2^31 and above read as zeros).
static bool g8_ta_ok(const clskd_conv_desc& d) {
  if (knob(KNOB_G8_TA) == 0 || d.ntaps < 1 || d.ntaps > 16 || d.nseg < 1 || d.nseg > 2) return false;
  if (d.ctot % 64 != 0 || (int64_t)d.ntaps * d.ctot != d.K) return false;
  if (d.nseg == 2 && d.seg_c[0] % 64 != 0) return false;
  for (int s = 0; s < d.nseg; ++s) {
    const clskd_seg& g = d.seg[s];
    if (g.sB < 0 || g.sF < 0 || g.sT < 0) return false;
    const int64_t last = (int64_t)(d.B - 1) * g.sB + (int64_t)(d.Fo - 1) * d.stride_f * g.sF +
                         (int64_t)(d.To - 1) * d.stride_t * g.sT + 64;
    if (last * 2 >= ((int64_t)1 << 31) - 64) return false;
  }
  return (int64_t)d.N * d.K * 2 < ((int64_t)1 << 31) - 64;
}

// Entry from launch_conv_bf16 for N > 64 bf16 layers.  *launched = false leaves the layer to the
// older engine (CLSKD_G8=0 selects that everywhere; an A/B switch).  CLSKD_G8 = 10*cfg + dbg
// selects timing-experiment variants (bf16 outputs only); read per launch (tests switch it).
// Whether launch_conv_gemm8 would take the layer (default mode).
bool conv_gemm8_takes(const clskd_conv_desc& d) {
  return knob(KNOB_G8) != 0 && d.N > 64 && d.K % 64 == 0 && d.nseg <= 2 &&
         (int64_t)d.B * d.Fo * d.To < ((int64_t)1 << 31) && (int64_t)d.Fo * d.stride_f < 32768 &&
         (int64_t)d.To * d.stride_t < 32768;
}

int launch_conv_gemm8(const clskd_conv_desc& d, hipStream_t st, bool* launched) {
  *launched = false;
  const int mode = knob(KNOB_G8);
  if (mode >= 10) {
    const int rc = experiment_guard("CLSKD_G8", mode);
    if (rc != CLSKD_OK) return rc;
  }
  if (mode == 0 || d.N <= 64 || d.K % 64 != 0 || d.nseg > 2 || (int64_t)d.B * d.Fo * d.To >= ((int64_t)1 << 31) ||
      (int64_t)d.Fo * d.stride_f >= 32768 || (int64_t)d.To * d.stride_t >= 32768)  // 16-bit row origins
    return CLSKD_OK;
  const bool f32 = d.out_dtype == CLSKD_F32;
  *launched = true;
#ifdef CLSKD_EXPERIMENTS
  if (mode >= 100 && !f32 && d.in_dtype == CLSKD_BF16 && g8_ta_ok(d)) {
    // TA ablations (round 6): CLSKD_G8 = 100 + ABL flags (see the kernel's DBG >= 16 note)
#define G8A(ABL_)                                                                               \
  case ABL_:                                                                                    \
    if (d.N <= 128) return launch_g8<256, 128, 4, 64, 2, 2, __bf16, 16 + ABL_, 1, 8, 1, __bf16, 0, 1>(d, st); \
    return launch_g8<256, 256, 2, 64, 2, 2, __bf16, 16 + ABL_, 1, 8, 1, __bf16, 0, 1>(d, st);
    switch (mode - 100) {
      G8A(0) G8A(1) G8A(2) G8A(3) G8A(4) G8A(6) G8A(7) G8A(8) G8A(11) G8A(15) G8A(16) G8A(32) G8A(64)
      G8A(128) G8A(256)
      default:
        set_error("CLSKD_G8=%d: unknown ablation", mode);
        return CLSKD_E_ARG;
    }
#undef G8A
  }
  if (mode >= 10 && mode < 100) {
    // rounds 2-4's tile / stage / prefetch variants (CLSKD_G8 = 10 * cfg + dbg) were measured and
    // not adopted; round 6 dropped them from the experiments library
    set_error("CLSKD_G8=%d: the round 2-4 variants are no longer built (TA ablations: 100 + flags)", mode);
    return CLSKD_E_ARG;
  }
#endif
  // default: BK 64, two stages, the K-tile boundary before the last substep (EB; 3-5 % on the
  // N = 256 layers against the boundary after it, CLSKD_G8=10)
  if (d.in_dtype == CLSKD_F16) {  // C4: IEEE-half operands (v_mfma_f32_32x32x16_f16)
    if (g8_ta_ok(d)) {
      if (d.N <= 128)
        return f32 ? launch_g8<256, 128, 4, 64, 2, 2, float, 0, 1, 8, 1, _Float16, 0, 1>(d, st)
                   : launch_g8<256, 128, 4, 64, 2, 2, _Float16, 0, 1, 8, 1, _Float16, 0, 1>(d, st);
      return f32 ? launch_g8<256, 256, 2, 64, 2, 2, float, 0, 1, 8, 1, _Float16, 0, 1>(d, st)
                 : launch_g8<256, 256, 2, 64, 2, 2, _Float16, 0, 1, 8, 1, _Float16, 0, 1>(d, st);
    }
    if (d.N <= 128)
      return f32 ? launch_g8<256, 128, 4, 64, 2, 2, float, 0, 1, 8, 1, _Float16>(d, st)
                 : launch_g8<256, 128, 4, 64, 2, 2, _Float16, 0, 1, 8, 1, _Float16>(d, st);
    return f32 ? launch_g8<256, 256, 2, 64, 2, 2, float, 0, 1, 8, 1, _Float16>(d, st)
               : launch_g8<256, 256, 2, 64, 2, 2, _Float16, 0, 1, 8, 1, _Float16>(d, st);
  }
#ifdef CLSKD_EXPERIMENTS
  // ping-pong K loop (round 4, measured): the 256x256 instance within +-2 % of the phased loop
  // on every C2 layer, the 256x128 instance 10-15 % slower (census, one box) — experiments only
  if (knob(KNOB_G8_PP) == 1) {
    if (d.N <= 128)
      return f32 ? launch_g8<256, 128, 4, 64, 2, 2, float, 0, 1, 8, 1, __bf16, 1>(d, st)
                 : launch_g8<256, 128, 4, 64, 2, 2, __bf16, 0, 1, 8, 1, __bf16, 1>(d, st);
    return f32 ? launch_g8<256, 256, 2, 64, 2, 2, float, 0, 1, 8, 1, __bf16, 1>(d, st)
               : launch_g8<256, 256, 2, 64, 2, 2, __bf16, 0, 1, 8, 1, __bf16, 1>(d, st);
  }
#endif
  if (g8_ta_ok(d)) {
    if (d.N <= 128)
      return f32 ? launch_g8<256, 128, 4, 64, 2, 2, float, 0, 1, 8, 1, __bf16, 0, 1>(d, st)
                 : launch_g8<256, 128, 4, 64, 2, 2, __bf16, 0, 1, 8, 1, __bf16, 0, 1>(d, st);
    return f32 ? launch_g8<256, 256, 2, 64, 2, 2, float, 0, 1, 8, 1, __bf16, 0, 1>(d, st)
               : launch_g8<256, 256, 2, 64, 2, 2, __bf16, 0, 1, 8, 1, __bf16, 0, 1>(d, st);
  }
  if (d.N <= 128) {
    return f32 ? launch_g8<256, 128, 4, 64, 2, 2, float, 0, 1, 8, 1>(d, st)
               : launch_g8<256, 128, 4, 64, 2, 2, __bf16, 0, 1, 8, 1>(d, st);
  }
  return f32 ? launch_g8<256, 256, 2, 64, 2, 2, float, 0, 1, 8, 1>(d, st)
             : launch_g8<256, 256, 2, 64, 2, 2, __bf16, 0, 1, 8, 1>(d, st);
}

}  // namespace clskd

extern "C" int32_t clskd_conv_last_stream_k(void) { return clskd::g_last_sk; }

extern "C" int clskd_stream_prepare(void* stream) {
  return clskd::sk_workspace(reinterpret_cast<hipStream_t>(stream)) ? CLSKD_OK : CLSKD_E_HIP;
}

extern "C" int clskd_capture_scope_begin(void* const* streams, int32_t nstreams, void** scope) {
  using namespace clskd;
  CLSKD_CHECK_ARG(scope && nstreams >= 0 && (nstreams == 0 || streams), "capture_scope_begin: bad arguments");
  CLSKD_CHECK_ARG(g_sk_scope == nullptr, "capture_scope_begin: a scope is already bound to this thread");
  auto* sc = new SkScope();
  for (int i = 0; i < nstreams; ++i) {
    hipStream_t st = reinterpret_cast<hipStream_t>(streams[i]);
    if (sc->ws.count(st)) continue;
    SkWs w{};
    if (!sk_alloc(w, st, true)) {
      for (auto& kv : sc->ws) {
        (void)hipFree(kv.second.ws);
        (void)hipFree(kv.second.ready);
      }
      delete sc;
      set_error("capture_scope_begin: workspace allocation failed");
      return CLSKD_E_HIP;
    }
    sc->ws[st] = w;
  }
  g_sk_scope = sc;
  *scope = sc;
  return CLSKD_OK;
}

extern "C" int clskd_capture_scope_end(void* scope) {
  using namespace clskd;
  CLSKD_CHECK_ARG(scope && g_sk_scope == scope, "capture_scope_end: not the scope bound to this thread");
  g_sk_scope = nullptr;
  return CLSKD_OK;
}

extern "C" int clskd_capture_scope_free(void* scope) {
  using namespace clskd;
  if (!scope) return CLSKD_OK;
  auto* sc = reinterpret_cast<SkScope*>(scope);
  CLSKD_CHECK_ARG(g_sk_scope != sc, "capture_scope_free: the scope is still bound (call capture_scope_end)");
  for (auto& kv : sc->ws) {
    (void)hipFree(kv.second.ws);
    (void)hipFree(kv.second.ready);
  }
  delete sc;
  return CLSKD_OK;
}
