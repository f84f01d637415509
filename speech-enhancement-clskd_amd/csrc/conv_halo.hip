// Halo-tiled bf16 convolution for narrow outputs (N <= 64): the ReviewKD 3x3 convs
// (framework.py:189-191, 64 -> 32/64 channels at the teacher's resolutions), the teacher's
// 32-channel decoder layers and its second encoder layer.
//
// For these layers the implicit-GEMM engine stages the im2col-expanded A operand — every input
// pixel once per tap (6-10x) — and N is too small for that to amortise (staged bytes per FLOP
// = 1/N); the engine is LDS-DMA-bound at 150-350 TF/s.  Here:
//   * the whole weight matrix [N][K] lives in LDS for the kernel's lifetime (persistent
//     workgroups, one per CU), rows padded to an odd number of 16-B chunks so the B-fragment
//     reads of 32 different rows hit 32 distinct bank slots;
//   * an output tile is 8 F-rows x 32 time steps (wave w owns F-row w: one 32x32 MFMA row
//     block); its input halo — (7*stride_f + taps_F) x (31 + taps_T) pixels — is staged once
//     per 32-channel chunk by LDS-DMA (64-B pixel rows, 16-B chunks XOR-swizzled by
//     (pixel>>2)&3, out-of-bounds pixels from a zero page) and reused by every tap;
//   * halo chunks are double-buffered: the DMA of item i+1 runs under the MFMAs of item i;
//   * the epilogue issues a static number of stores per wave (invalid rows go to a sink page),
//     so the next item's counted vmcnt wait never waits for store acknowledgements;
//   * BatchNorm statistics accumulate per workgroup in fp64 across its tiles; workgroup b
//     writes partial slot b and zeroes its share of the remaining ceil(M/128) slots (the
//     partial-slot contract of include/clskd.h is unchanged).
// Same descriptor, output map and bias/stats semantics as the engines.
#include <stdlib.h>

#include "bnfold.h"
#include "common.h"

#ifndef HALO_TRACE
#define HALO_TRACE(i)
#endif

namespace clskd {

typedef __bf16 bf16x8h __attribute__((ext_vector_type(8)));

__device__ __attribute__((aligned(64))) unsigned char g_halo_zero[64];
__device__ __attribute__((aligned(256))) unsigned char g_halo_sink[4096];

namespace halo {
constexpr int FT = 8;      // output F-rows per tile (= waves)
constexpr int TT = 32;     // output time steps per tile
constexpr int NW = 8;      // waves
constexpr int CW = 32;     // channels per chunk: 64-B pixel rows
constexpr int MAXG = 6;    // max LDS-DMA instructions per wave per chunk (48 KiB halo buffer)
constexpr int MAXCH = 32;  // max chunks

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

__device__ __forceinline__ int pswz(int p) { return (p >> 2) & 3; }
}  // namespace halo

struct HaloArgs {
  clskd_conv_desc d;
  int32_t nchunk;
  int32_t chunk_seg[halo::MAXCH];
  int32_t chunk_c0[halo::MAXCH];   // channel offset inside the segment
  int32_t chunk_kofs[halo::MAXCH]; // k offset of the chunk inside one tap's ctot channels
  int32_t dfmin, dtmin;            // halo origin relative to (fo*stride_f, to)
  int32_t HF, HT, NPIX;            // halo extent (pixels) and count
  int32_t NGH;                     // DMA wave-instructions per wave per chunk
  int32_t halo_bytes;              // bytes per halo buffer (NW * NGH KiB)
  int32_t pitch;                   // bytes per weight row in LDS (odd number of 16-B chunks)
  int32_t kc8;                     // 16-B weight chunks per row actually used
  int32_t nfb, ntb, ntiles;        // tile grid: F-blocks, T-blocks, total
  int32_t nblk128;                 // statistics slots (ceil(M/128))
  int32_t tap_pix[16];             // halo pixel offset of tap t for output (0, 0)
  int32_t tap_k[16];               // k offset of tap t (t * ctot)
  BnFoldArgs f;                    // folded BatchNorm finalize (f.acc != nullptr)
  int32_t stats_ld;                // channels per statistics slot row (N, or the full N of a
                                   // column-split launch whose stats pointer is pre-offset)
};

// Kernel arguments are re-read by the compiler under SGPR pressure (s_load inside the loop),
// and scalar loads share lgkmcnt with LDS reads — every fragment wait then degrades to
// lgkmcnt(0).  Values the loop needs are therefore laundered through an opaque VGPR into an
// SGPR (no re-materialisation from the kernarg segment is possible) or staged in LDS.
__device__ __forceinline__ int sconst(int v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int64_t vconst64(int64_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int BN, typename OutT, int NTAPS, typename InT = __bf16>
__global__ __launch_bounds__(512) void conv_halo_kernel(const HaloArgs a) {
  constexpr int DBG = 0;
  using namespace halo;
  const clskd_conv_desc& d = a.d;
  constexpr int NB = BN / 32;  // 32-wide MFMA column tiles
  constexpr int NS = 4 / NB;   // accumulator sets per column tile: 4 MFMA chains per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int halo_bytes = sconst(a.halo_bytes);
  unsigned char* hbuf = smem;                       // [2][halo_bytes]
  unsigned char* wl = smem + 2 * halo_bytes;        // [BN][pitch]
  int4* ctA = reinterpret_cast<int4*>(wl + BN * a.pitch);  // [nchunk] {base lo, base hi, sF, sT}
  int4* ctB = ctA + MAXCH;                                 // [nchunk] {sB, F, T, kofs}
  int* ttab = reinterpret_cast<int*>(ctB + MAXCH);         // [16] tap pixel offset | tap k << 16

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  HALO_TRACE(0);

  // ---- prologue: weights and tables into LDS, stats slots, bias ----------------------------
  // weights: batches of WB independent 16-B loads per thread in flight, then the LDS stores
  // (a load-store loop would serialise one global latency per iteration)
  const unsigned short* wg = reinterpret_cast<const unsigned short*>(d.weight);
  {
    constexpr int WB = 16;
    const int total = BN * a.kc8, kc8 = a.kc8;
    for (int base = tid; base < total; base += 512 * WB) {
      f32x4 v[WB];
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        const int idx = base + j * 512;
        const int n = idx / kc8, c8 = idx - (idx / kc8) * kc8;
        v[j] = (idx < total && n < d.N) ? *reinterpret_cast<const f32x4*>(wg + (int64_t)n * d.K + c8 * 8)
                                        : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        const int idx = base + j * 512;
        const int n = idx / kc8, c8 = idx - (idx / kc8) * kc8;
        if (idx < total) *reinterpret_cast<f32x4*>(wl + n * a.pitch + c8 * 16) = v[j];
      }
    }
  }
  if (tid < a.nchunk) {
    const int sg = a.chunk_seg[tid];
    const clskd_seg& S = d.seg[sg];
    const uint64_t base = (uint64_t)(uintptr_t)(reinterpret_cast<const __bf16*>(S.ptr) + a.chunk_c0[tid]);
    ctA[tid] = make_int4((int)(unsigned)base, (int)(unsigned)(base >> 32), (int)S.sF, (int)S.sT);
    ctB[tid] = make_int4((int)S.sB, S.F, S.T, a.chunk_kofs[tid]);
  }
  if (tid < 16) ttab[tid] = a.tap_pix[tid] | (a.tap_k[tid] << 16);
  if (d.stats) {
    for (int64_t s = (int64_t)blockIdx.x + gridDim.x; s < a.nblk128; s += gridDim.x)
      for (int i = tid; i < d.N * 2; i += 512) d.stats[s * a.stats_ld * 2 + i] = 0.0;
  }
  float bcol[NB];
  int64_t coff[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = nb * 32 + l32;
    bcol[nb] = (d.bias && n < d.N) ? d.bias[n] : 0.f;
    coff[nb] = vconst64(n < d.N ? (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo : -1);
  }
  // loop constants (laundered: never re-loaded from the kernarg segment inside the loop)
  const int nchunk = sconst(a.nchunk), ntb = sconst(a.ntb), nfb = sconst(a.nfb);
  const int NGH = sconst(a.NGH);
  const int Fo = sconst(d.Fo), To = sconst(d.To), sfr = sconst(d.stride_f);
  const int dfmin = sconst(a.dfmin), dtmin = sconst(a.dtmin);
  const int64_t oB = vconst64(d.oB), oF = vconst64(d.oF), oT = vconst64(d.oT);
  const int of_mul = sconst(d.of_mul), of_add = sconst(d.of_add);
  // global address space: a laundered generic pointer would make the epilogue stores FLAT,
  // which count on lgkmcnt too — every fragment wait in the loop degrades to lgkmcnt(0)
  using GOut = __attribute__((address_space(1))) OutT;
  GOut* const outp = reinterpret_cast<GOut*>(vconst64((int64_t)(uintptr_t)d.out));
  // per-lane DMA slot geometry, packed: hf | ht << 8 | src chunk << 16 | valid << 20
  int dmg[MAXG];
  {
    const int HT = a.HT, NPIX = a.NPIX;
#pragma unroll
    for (int i = 0; i < MAXG; ++i) {
      const int slot = (wave * NGH + i) * 64 + lane;
      const int p = slot >> 2;
      const bool ok = i < NGH && p < NPIX;
      const int pp = ok ? p : 0;
      const int hf = pp / HT, ht = pp - (pp / HT) * HT;
      dmg[i] = hf | (ht << 8) | (((slot & 3) ^ pswz(p)) << 16) | ((ok ? 1 : 0) << 20);
    }
  }
  const int prow0 = wave * sfr * sconst(a.HT) + l32;  // halo pixel of (F-row wave, time l32)
  __syncthreads();
  HALO_TRACE(1);

  const uint64_t zero_addr = (uint64_t)(uintptr_t)g_halo_zero;
  const unsigned hlds0 = __builtin_amdgcn_readfirstlane(lds_addr(hbuf));
  const int per = (sconst(a.ntiles) + gridDim.x - 1) / gridDim.x;
  const int tile_begin = blockIdx.x * per;
  const int ntile_blk = max(0, min(sconst(a.ntiles), tile_begin + per) - tile_begin);

  // tile cursors (b, fb, tb) advanced incrementally: no divisions in the loop
  struct Cur { int b, fb, tb; };
  auto cur_of = [&](int tile) {
    Cur c;
    c.tb = tile % ntb;
    const int r = tile / ntb;
    c.fb = r % nfb;
    c.b = r / nfb;
    return c;
  };
  auto advance = [&](Cur& c) {
    if (++c.tb == ntb) {
      c.tb = 0;
      if (++c.fb == nfb) { c.fb = 0; ++c.b; }
    }
  };

  auto issue = [&](const Cur& c, int ch, int buf) {
    if constexpr (DBG == 1) return;  // timing experiment: no halo traffic
    const int4 ea = ctA[ch];
    const int4 eb = ctB[ch];
    const __bf16* base = reinterpret_cast<const __bf16*>(((uint64_t)(unsigned)ea.y << 32) | (unsigned)ea.x) +
                         (int64_t)c.b * eb.x;
    const int fi_lo = c.fb * FT * sfr + dfmin, ti_lo = c.tb * TT + dtmin;
    const unsigned dst = hlds0 + buf * halo_bytes;
#pragma unroll
    for (int i = 0; i < MAXG; ++i) {
      if (i < NGH) {
        const int g = dmg[i];
        const int fi = fi_lo + (g & 0xff), ti = ti_lo + ((g >> 8) & 0xff);
        const bool ok = ((g >> 20) & 1) && (unsigned)fi < (unsigned)eb.y && (unsigned)ti < (unsigned)eb.z;
        const uint64_t src = ok ? (uint64_t)(uintptr_t)(base + (int64_t)fi * ea.z + (int64_t)ti * ea.w +
                                                        ((g >> 16) & 3) * 8)
                                : zero_addr;
        glds16((const void*)src, dst + (wave * NGH + i) * 1024);
      }
    }
  };

  f32x16 acc[NS][NB];
  double st_s[NB], st_q[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) st_s[nb] = st_q[nb] = 0.0;
  int stores_pending = 0;

  Cur cur = cur_of(tile_begin), nxt = cur;
  int nxt_ch = 0, nxt_left = ntile_blk * nchunk;
  int buf = 0;
  if (nxt_left > 0) {
    issue(nxt, 0, 0);
    --nxt_left;
    nxt_ch = 1;
    if (nxt_ch == nchunk) { nxt_ch = 0; advance(nxt); }
  }
  for (int ti = 0; ti < ntile_blk; ++ti) {
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][nb][r] = q == 0 ? bcol[nb] : 0.f;
    for (int ch = 0; ch < nchunk; ++ch) {
      // this chunk's halo was issued one step ago; younger: only the last epilogue's stores
      if (DBG != 3 && stores_pending) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB * 16) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      stores_pending = 0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (nxt_left > 0) {
        issue(nxt, nxt_ch, buf ^ 1);
        --nxt_left;
        if (++nxt_ch == nchunk) { nxt_ch = 0; advance(nxt); }
      }
      const unsigned char* hb = hbuf + buf * halo_bytes;
      const int kofs = ctB[ch].w;
      // taps fully unrolled against a register copy of the packed tap table: the loop's only
      // LDS traffic is fragment reads, so waits stay counted and reads run ahead of the MFMAs
      int4 tq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) tq[i] = reinterpret_cast<const int4*>(ttab)[i];
      // software pipeline over the (compile-time) taps: fragments of tap t+1 are read into the
      // other half of a ping-pong register set before tap t's MFMAs; sched_barrier pins that
      // order so each MFMA waits only for the older reads (counted lgkmcnt, not 0)
      bf16x8h af[2][2], bw[2][2][NB];
      auto load_tap = [&](int t, int sl) {
        const int tv = tq[t >> 2][t & 3];
        const int p = prow0 + (tv & 0xffff);
        const int kb = (tv >> 16) + kofs;
#pragma unroll
        for (int k16 = 0; k16 < 2; ++k16) {
          const int c = k16 * 2 + h;
          af[sl][k16] = *reinterpret_cast<const bf16x8h*>(hb + p * 64 + ((c ^ pswz(p)) << 4));
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            bw[sl][k16][nb] = *reinterpret_cast<const bf16x8h*>(wl + (nb * 32 + l32) * a.pitch +
                                                                (kb + k16 * 16 + h * 8) * 2);
        }
      };
      load_tap(0, 0);
#pragma unroll
      for (int t = 0; t < NTAPS; ++t) {
        if (t + 1 < NTAPS) load_tap(t + 1, (t + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k16 = 0; k16 < 2; ++k16) {
          const int q = ((t & 1) * 2 + k16) % NS;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[q][nb] = mfma16<InT>(af[t & 1][k16], bw[t & 1][k16][nb], acc[q][nb]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      buf ^= 1;
    }
    // ---- tile epilogue: stats + a static number of stores --------------------------------
    const int fo = cur.fb * FT + wave;
    const int to0 = cur.tb * TT;
    const int64_t rowb = (int64_t)cur.b * oB + (int64_t)(fo * of_mul + of_add) * oF;
    GOut* sink = reinterpret_cast<GOut*>((uintptr_t)g_halo_sink) + lane;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const bool nok = coff[nb] >= 0;
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;  // MFMA C row = output time offset
        const int to = to0 + row;
        const bool ok = nok && fo < Fo && to < To;
        float v = acc[0][nb][r];
#pragma unroll
        for (int q = 1; q < NS; ++q) v += acc[q][nb][r];
        if (ok) {
          sm += v;
          sq = fmaf(v, v, sq);
        }
        GOut* dst = ok ? outp + rowb + (int64_t)to * oT + coff[nb] : sink;
        if constexpr (DBG != 3) *dst = (OutT)v;
      }
      st_s[nb] += (double)sm;
      st_q[nb] += (double)sq;
    }
    stores_pending = 1;
    advance(cur);
    HALO_TRACE(2 + ti);
  }
  HALO_TRACE(40);

  if (d.stats || a.f.acc) {  // workgroup partial: lanes (h halves) and waves in a fixed order
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // reuse the halo buffers: [NW][BN][2]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const double s2 = st_s[nb] + __shfl_xor(st_s[nb], 32, 64);
      const double q2 = st_q[nb] + __shfl_xor(st_q[nb], 32, 64);
      if (h == 0) {
        red[(wave * BN + nb * 32 + l32) * 2] = s2;
        red[(wave * BN + nb * 32 + l32) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    if (a.f.acc) {  // folded finalize: waves in the same fixed order
      bnfold_commit(a.f, d.N, [&](int n, double& S, double& Q) {
        S = 0.0;
        Q = 0.0;
        for (int w = 0; w < NW; ++w) {
          S += red[(w * BN + n) * 2];
          Q += red[(w * BN + n) * 2 + 1];
        }
      }, reinterpret_cast<int*>(red + NW * BN * 2), blockIdx.x, gridDim.x);
    } else if (blockIdx.x < a.nblk128) {
      for (int n = tid; n < d.N; n += 512) {
        double S = 0.0, Q = 0.0;
        for (int w = 0; w < NW; ++w) {
          S += red[(w * BN + n) * 2];
          Q += red[(w * BN + n) * 2 + 1];
        }
        d.stats[((int64_t)blockIdx.x * a.stats_ld + n) * 2] = S;
        d.stats[((int64_t)blockIdx.x * a.stats_ld + n) * 2 + 1] = Q;
      }
    }
  }
}

// Plan + eligibility (host).  Returns false (engine path) when the layer does not fit.
static bool halo_plan(const clskd_conv_desc& d, HaloArgs& a, size_t& lds) {
  using namespace halo;
  if (!is_lowp(d.in_dtype) || d.N > 64 || d.ntaps < 1 || d.ntaps > 16 || d.stride_t != 1)
    return false;
  if (d.stride_f < 1 || d.stride_f > 2 || d.ctot < CW) return false;
  a.d = d;
  // chunks: (tap-major K order) segments in order, 32 channels each
  int nch = 0, kofs = 0;
  for (int s = 0; s < d.nseg; ++s) {
    if (d.seg_c[s] % CW) return false;
    for (int c0 = 0; c0 < d.seg_c[s]; c0 += CW) {
      if (nch >= MAXCH) return false;
      a.chunk_seg[nch] = s;
      a.chunk_c0[nch] = c0;
      a.chunk_kofs[nch] = kofs + c0;
      ++nch;
    }
    kofs += d.seg_c[s];
  }
  if (kofs != d.ctot || d.ntaps * d.ctot > d.K) return false;
  a.nchunk = nch;
  int dfmin = 1 << 20, dfmax = -(1 << 20), dtmin = 1 << 20, dtmax = -(1 << 20);
  for (int t = 0; t < d.ntaps; ++t) {
    dfmin = d.tap_df[t] < dfmin ? d.tap_df[t] : dfmin;
    dfmax = d.tap_df[t] > dfmax ? d.tap_df[t] : dfmax;
    dtmin = d.tap_dt[t] < dtmin ? d.tap_dt[t] : dtmin;
    dtmax = d.tap_dt[t] > dtmax ? d.tap_dt[t] : dtmax;
  }
  a.dfmin = dfmin;
  a.dtmin = dtmin;
  a.HF = (FT - 1) * d.stride_f + (dfmax - dfmin + 1);
  a.HT = (TT - 1) + (dtmax - dtmin + 1);
  a.NPIX = a.HF * a.HT;
  for (int t = 0; t < 16; ++t) {
    a.tap_pix[t] = t < d.ntaps ? (d.tap_df[t] - dfmin) * a.HT + (d.tap_dt[t] - dtmin) : 0;
    a.tap_k[t] = t < d.ntaps ? t * d.ctot : 0;
  }
  a.NGH = (int)cdiv((int64_t)a.NPIX * 4, 64 * NW);  // 4 x 16-B slots per pixel
  if (a.NGH > MAXG) return false;
  a.halo_bytes = NW * a.NGH * 1024;
  const int kused = d.ntaps * d.ctot;
  a.kc8 = (kused + 7) / 8;
  a.pitch = (a.kc8 % 2 == 0 ? a.kc8 + 1 : a.kc8) * 16;
  const int BN = d.N <= 32 ? 32 : 64;
  lds = 2 * (size_t)a.halo_bytes + (size_t)BN * a.pitch + 2 * MAXCH * 16 + 16 * 8;
  for (int s = 0; s < d.nseg; ++s)
    if (d.seg[s].sB > INT32_MAX || d.seg[s].sF > INT32_MAX || d.seg[s].sT > INT32_MAX) return false;
  if (lds > 160 * 1024) return false;
  if ((d.stats || d.bn_fold) && (size_t)NW * BN * 16 + 16 > 2 * (size_t)a.halo_bytes) return false;
  a.nfb = (int)cdiv(d.Fo, FT);
  a.ntb = (int)cdiv(d.To, TT);
  const int64_t nt = (int64_t)d.B * a.nfb * a.ntb;
  if (nt < 32 || nt > (1 << 30)) return false;
  a.ntiles = (int)nt;
  a.nblk128 = (int)cdiv((int64_t)d.B * d.Fo * d.To, 128);
  a.stats_ld = d.N;
  a.f = make_bnfold(d);
  return true;
}

static int launch_halo_planned(const HaloArgs& a, size_t lds, hipStream_t st, bool* launched);

// Layers with 32 < N <= 64 whose [64][K] weight block does not fit LDS beside the halo buffers
// (the teacher's 64-channel decoder layer: K = 6 x 256) run as two 32-column launches; each
// re-reads the input halo (~N/K of the staged-bytes saving is kept) but stays on the halo path
// instead of the im2col engine.  Output columns, bias and the statistics slots of the second
// launch are offset by 32 (statistics rows keep the full N as leading dimension).
// Whether launch_conv_halo would take the layer (the same plans, nothing launched).
bool conv_halo_takes(const clskd_conv_desc& d) {
  HaloArgs a;
  size_t lds = 0;
  if (halo_plan(d, a, lds)) return true;
  if (d.N <= 32 || d.N > 64 || d.nlo < d.N || !is_lowp(d.in_dtype)) return false;
  clskd_conv_desc d1 = d, d2 = d;
  d1.N = 32;
  d2.N = d.N - 32;
  HaloArgs a2;
  size_t lds2 = 0;
  return halo_plan(d1, a, lds) && halo_plan(d2, a2, lds2);
}

int launch_conv_halo(const clskd_conv_desc& d, hipStream_t st, bool* launched) {
  HaloArgs a;
  size_t lds = 0;
  *launched = false;
  if (halo_plan(d, a, lds)) return launch_halo_planned(a, lds, st, launched);
  if (d.N <= 32 || d.N > 64 || d.nlo < d.N || !is_lowp(d.in_dtype)) return CLSKD_OK;
  HaloArgs a2;
  size_t lds2 = 0;
  clskd_conv_desc d1 = d, d2 = d;
  d1.N = 32;
  d2.N = d.N - 32;
  d2.weight = reinterpret_cast<const __bf16*>(d.weight) + (int64_t)32 * d.K;
  if (d.bias) d2.bias = d.bias + 32;
  const size_t osz = d.out_dtype == CLSKD_F32 ? 4 : 2;
  d2.out = reinterpret_cast<char*>(d.out) + (int64_t)32 * d.oNlo * (int64_t)osz;
  if (d.stats) d2.stats = d.stats + 64;
  if (!halo_plan(d1, a, lds) || !halo_plan(d2, a2, lds2)) return CLSKD_OK;
  a.stats_ld = a2.stats_ld = d.N;
  if (a.f.acc) {  // column halves: the second one (channels +32) finalizes the layer
    a2.f = a.f;
    a.f.finalize = 0;
    a2.f.c_off += 32;
  }
  bool l1 = false, l2 = false;
  int rc = launch_halo_planned(a, lds, st, &l1);
  if (rc != CLSKD_OK || !l1) return rc;
  rc = launch_halo_planned(a2, lds2, st, &l2);
  if (rc == CLSKD_OK && !l2) {
    set_error("conv halo: second column half not launchable");
    return CLSKD_E_ARG;
  }
  *launched = true;
  return rc;
}

static int launch_halo_planned(const HaloArgs& a, size_t lds, hipStream_t st, bool* launched) {
  const clskd_conv_desc& d = a.d;
  *launched = false;
  static int ncu = [] {
    int v = 256;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
    return v > 0 ? v : 256;
  }();
  // CLSKD_HALO_GRID caps the workgroup count (leaves CUs to concurrent streams; A/B knob)
  const int cap = knob(KNOB_HALO_GRID) > 0 ? knob(KNOB_HALO_GRID) : ncu;
  const int ncap = cap > 0 && cap < ncu ? cap : ncu;
  const int grid = a.ntiles < ncap ? a.ntiles : ncap;
  if (d.stats && grid > a.nblk128) return CLSKD_OK;  // (never for eligible shapes)
  const bool f32out = d.out_dtype == CLSKD_F32;
#define HALO_LAUNCH(BN_, O_, NT_, I_)                                                          \
  do {                                                                                         \
    auto k = conv_halo_kernel<BN_, O_, NT_, I_>;                                               \
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,      \
                              160 * 1024);                                                     \
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, st, a);                                  \
    note_kernel_fn((const void*)k);                                                            \
    if (__is_same(I_, _Float16))                                                               \
      note_kernel("conv_halo_kernel<%d,%s,%d,f16>", BN_, type_name<O_>(), NT_);                \
    else                                                                                       \
      note_kernel("conv_halo_kernel<%d,%s,%d>", BN_, type_name<O_>(), NT_);                    \
  } while (0)
#define HALO_NI(NT_, I_)                                                                       \
  do {                                                                                         \
    if (d.N <= 32) {                                                                           \
      if (f32out) HALO_LAUNCH(32, float, NT_, I_); else HALO_LAUNCH(32, I_, NT_, I_);          \
    } else {                                                                                   \
      if (f32out) HALO_LAUNCH(64, float, NT_, I_); else HALO_LAUNCH(64, I_, NT_, I_);          \
    }                                                                                          \
  } while (0)
#define HALO_NT(NT_)                                                                           \
  do {                                                                                         \
    if (d.in_dtype == CLSKD_F16) HALO_NI(NT_, _Float16); else HALO_NI(NT_, __bf16);            \
  } while (0)
  switch (d.ntaps) {
    case 4: HALO_NT(4); break;
    case 6: HALO_NT(6); break;
    case 9: HALO_NT(9); break;
    case 10: HALO_NT(10); break;
    default: return CLSKD_OK;  // not a built tap count: engine path
  }
#undef HALO_NT
#undef HALO_NI
#undef HALO_LAUNCH
  *launched = true;
  return CLSKD_OK;
}

}  // namespace clskd
