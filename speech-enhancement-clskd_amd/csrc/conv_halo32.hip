// Halo-tiled exact-fp32 convolution for narrow outputs (32 <= N <= 64): the student's encoder
// and decoder layers (ComplexConv2d / ComplexConvTranspose2d polyphase, tools_for_model.py:236-262,
// 303-330) and the fp32 ReviewKD 3x3 convs (framework.py:189-191) of precision='fp32'.
//
// The implicit-GEMM fp32 engine (conv_igemm.hip) gathers the im2col-expanded A operand with
// VALU address arithmetic for every (row, tap, channel) — ~129 instructions beside 8 MFMAs per
// 16-deep K-tile — and runs these layers at 45-75 TF/s of the 157 TF/s fp32 MFMA peak.  At
// fp32 MFMA rates the staging is cheap (an 8x32 output tile of a 64 x 640 layer is ~82k MFMA
// cycles per CU against ~300 KB of input and weights), so the layer is organised like the bf16
// halo kernel (conv_halo.hip) and left to the MFMA pipe:
//   * persistent workgroups (one per CU, 8 waves), tile = 8 output F-rows x 32 time steps, wave
//     w owns F-row w as one 32-row block of v_mfma_f32_32x32x2_f32 (exact fp32 products,
//     fp32 accumulation — the same arithmetic class as the engine);
//   * the whole weight matrix lives in LDS in k-quad order [K/4][NB*32][4] floats: the B
//     fragment of 4 consecutive MFMAs is one 16-B read, and the 32 lanes of a half read 512
//     contiguous bytes (conflict-free);
//   * the input halo — (7*stride_f + taps_F) x (31 + taps_T) pixels — is staged once per
//     8-channel chunk (32-B pixel rows, 16-B halves XOR-swizzled by (pixel>>3)&1) by LDS-DMA,
//     double-buffered, and reused by every tap; an A fragment read (4 channels of one pixel)
//     feeds 4 MFMAs per column block;
//   * the epilogue issues a static number of stores (invalid rows to a sink page) and BatchNorm
//     statistics accumulate per workgroup in fp64 (same partial-slot contract as the engines).
// N = 64 layers whose [64][K] weights do not fit beside the halo buffers run as two 32-column
// launches (the input halo is staged twice; cheap at fp32 MFMA rates).
#include <stdlib.h>

#include "bnfold.h"
#include "common.h"

namespace clskd {

__device__ __attribute__((aligned(64))) unsigned char g_h32_zero[64];
__device__ __attribute__((aligned(256))) unsigned char g_h32_sink[4096];
// DBG == 5 (timing-only): 100 MHz wall-clock marks of workgroup 0, waves 0 and 4 (one SIMD)
__device__ uint64_t g_h32_marks[128];

typedef __attribute__((address_space(1))) float gfloat;

namespace h32 {
constexpr int FT = 8;      // output F-rows per tile (= waves)
constexpr int TT = 32;     // output time steps per tile
constexpr int NW = 8;      // waves
constexpr int CW = 8;      // fp32 channels per chunk: 32-B pixel rows (two 16-B halves)
constexpr int MAXG = 4;    // max LDS-DMA wave-instructions per wave per chunk (32 KiB halo buffer)
constexpr int MAXCH = 64;  // max chunks (ctot <= 512)

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

// 16-B half of pixel p's 32-B row that holds channel group j: conflict-free fragment reads
// (16 consecutive pixels of one half cover all 64 banks)
__device__ __forceinline__ int swz(int p) { return (p >> 3) & 1; }

// loop constants laundered through a VGPR into an SGPR: never re-loaded from the kernarg
// segment inside the loop (scalar loads would share lgkmcnt with the fragment reads)
__device__ __forceinline__ int sconst(int v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int64_t vconst64(int64_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
}  // namespace h32

struct Halo32Args {
  clskd_conv_desc d;
  int32_t nchunk;
  int32_t chunk_seg[h32::MAXCH];
  int32_t chunk_c0[h32::MAXCH];    // channel offset inside the segment
  int32_t chunk_kofs[h32::MAXCH];  // channel offset of the chunk inside one tap's ctot channels
  int32_t dfmin, dtmin;            // halo origin relative to (fo*stride_f, to)
  int32_t HF, HT, NPIX;            // halo extent (pixels) and count
  int32_t NGH;                     // DMA wave-instructions per wave per chunk
  int32_t halo_bytes;              // bytes per halo buffer (NW * NGH KiB)
  int32_t k4;                      // k-quads of resident weights (ntaps * ctot / 4)
  int32_t nfb, ntb, ntiles;        // tile grid: F-blocks, T-blocks, total
  int32_t nblk128;                 // statistics slots (ceil(M/128))
  int32_t tap_pix[16];             // halo pixel offset of tap t for output (0, 0)
  int32_t tap_kq[16];              // k-quad offset of tap t (t * ctot / 4)
  BnFoldArgs f;                    // folded BatchNorm finalize (f.acc != nullptr)
  int32_t stats_ld;                // channels per statistics slot row
};

// DBG (timing-only, experiments build): 1 no halo DMA, 2 fragments read once per chunk instead
// of per tap, 3 no MFMA, 4 no epilogue stores, 5 timeline marks (g_h32_marks), 6 / 7 MFMAs only
// in waves 0-3 / 4-7 (one wave per SIMD)
template <int NB, int NTAPS, int DBG = 0>
__global__ __launch_bounds__(512) void conv_halo_f32_kernel(const Halo32Args a) {
  using namespace h32;
  const clskd_conv_desc& d = a.d;
  constexpr int NBW = NB * 32;        // resident weight columns (zero beyond N)
  // accumulator chains per column block: 2 MFMA chains per wave (64-cycle dependent latency =
  // the issue interval, so alternating two accumulators never stalls)
  constexpr int NS = NB == 1 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int halo_bytes = sconst(a.halo_bytes);
  unsigned char* hbuf = smem;                                 // [2][halo_bytes]
  unsigned char* wl = smem + 2 * halo_bytes;                  // [k4][NBW][4] floats
  int4* ctA = reinterpret_cast<int4*>(wl + a.k4 * NBW * 16);  // [nchunk] {base lo, base hi, sF, sT}
  int4* ctB = ctA + MAXCH;                                    // [nchunk] {sB, F, T, kofs}
  int* ttab = reinterpret_cast<int*>(ctB + MAXCH);            // [16] tap pixel | tap k-quad << 16

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;

  // ---- prologue: weights (k-quad order) and tables into LDS, stats slots, bias -------------
  {
    constexpr int WB = 16;  // independent 16-B loads in flight per thread before the stores
    const float* wg = reinterpret_cast<const float*>(d.weight);
    const int total = a.k4 * NBW;
    const int64_t K = d.K;
    const int N = d.N;
    for (int base = tid; base < total; base += 512 * WB) {
      f32x4 v[WB];
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        const int idx = base + j * 512;
        const int kq = idx / NBW, n = idx % NBW;
        v[j] = (idx < total && n < N) ? *reinterpret_cast<const f32x4*>(wg + n * K + kq * 4)
                                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        const int idx = base + j * 512;
        if (idx < total) *reinterpret_cast<f32x4*>(wl + idx * 16) = v[j];
      }
    }
  }
  if (tid < a.nchunk) {
    const int sg = a.chunk_seg[tid];
    const clskd_seg& S = d.seg[sg];
    const uint64_t base = (uint64_t)(uintptr_t)(S.ptr + a.chunk_c0[tid]);
    ctA[tid] = make_int4((int)(unsigned)base, (int)(unsigned)(base >> 32), (int)S.sF, (int)S.sT);
    ctB[tid] = make_int4((int)S.sB, S.F, S.T, a.chunk_kofs[tid]);
  }
  if (tid < 16) ttab[tid] = a.tap_pix[tid] | (a.tap_kq[tid] << 16);
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
  const int nchunk = sconst(a.nchunk), ntb = sconst(a.ntb), nfb = sconst(a.nfb);
  const int NGH = sconst(a.NGH);
  const int Fo = sconst(d.Fo), To = sconst(d.To), sfr = sconst(d.stride_f);
  const int dfmin = sconst(a.dfmin), dtmin = sconst(a.dtmin);
  const int64_t oB = vconst64(d.oB), oF = vconst64(d.oF), oT = vconst64(d.oT);
  const int of_mul = sconst(d.of_mul), of_add = sconst(d.of_add);
  // global address space: a laundered generic pointer would make the stores FLAT, which count
  // on lgkmcnt too — every fragment wait in the loop would then degrade to lgkmcnt(0)
  gfloat* const outp = reinterpret_cast<gfloat*>(vconst64((int64_t)(uintptr_t)d.out));
  // per-lane DMA slot geometry, packed: hf | ht << 8 | source half << 16 | valid << 20
  int dmg[MAXG];
  {
    const int HT = a.HT, NPIX = a.NPIX;
#pragma unroll
    for (int i = 0; i < MAXG; ++i) {
      const int slot = (wave * NGH + i) * 64 + lane;
      const int p = slot >> 1;
      const bool ok = i < NGH && p < NPIX;
      const int pp = ok ? p : 0;
      const int hf = pp / HT, ht = pp - (pp / HT) * HT;
      dmg[i] = hf | (ht << 8) | (((slot & 1) ^ swz(p)) << 16) | ((ok ? 1 : 0) << 20);
    }
  }
  const int prow0 = wave * sfr * sconst(a.HT) + l32;  // halo pixel of (F-row wave, time l32)
  __syncthreads();
  if constexpr (DBG == 9) return;  // prologue only

  const uint64_t zero_addr = (uint64_t)(uintptr_t)g_h32_zero;
  const unsigned hlds0 = __builtin_amdgcn_readfirstlane(lds_addr(hbuf));
  const int per = (sconst(a.ntiles) + gridDim.x - 1) / gridDim.x;
  const int tile_begin = blockIdx.x * per;
  const int ntile_blk = max(0, min(sconst(a.ntiles), tile_begin + per) - tile_begin);

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
    if constexpr (DBG == 1 || DBG == 8) return;
    const int4 ea = ctA[ch];
    const int4 eb = ctB[ch];
    const float* base = reinterpret_cast<const float*>(((uint64_t)(unsigned)ea.y << 32) | (unsigned)ea.x) +
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
                                                        ((g >> 16) & 1) * 4)
                                : zero_addr;
        glds16((const void*)src, dst + (wave * NGH + i) * 1024);
      }
    }
  };

  f32x16 acc[NS][NB];
  double st_s[NB], st_q[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) st_s[nb] = st_q[nb] = 0.0;
  // A tile's outputs are stored one chunk step late, right after the next halo DMA is issued:
  // vmcnt counts stores, in issue order with the DMA, so stores issued at the tile boundary
  // (before that DMA) would make the next chunk wait for their acknowledgements.
  int stores_pending = 0;  // stores issued in the previous chunk step, younger than its DMA
  bool have_out = false;
  float ov[NB][16];
  int64_t obase = 0;
  unsigned omask = 0;
  auto flush = [&]() {
    gfloat* sink = reinterpret_cast<gfloat*>((uintptr_t)g_h32_sink) + lane;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        gfloat* dst = ((omask >> (nb * 16 + r)) & 1) ? outp + obase + (int64_t)row * oT + coff[nb] : sink;
        if constexpr (DBG != 4 && DBG != 8) *dst = ov[nb][r];
      }
  };

  int mk = 0;
  auto mark = [&]() {
    if constexpr (DBG == 5) {
      if (blockIdx.x == 0 && (wave == 0 || wave == 4) && lane == 0 && mk < 64)
        g_h32_marks[(wave ? 64 : 0) + mk] = wall_clock64();
      ++mk;
    }
  };
  mark();
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
      if (stores_pending) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB * 16) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      stores_pending = 0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      mark();
      if (nxt_left > 0) {
        issue(nxt, nxt_ch, buf ^ 1);
        --nxt_left;
        if (++nxt_ch == nchunk) { nxt_ch = 0; advance(nxt); }
      }
      if (have_out) {
        flush();
        have_out = false;
        stores_pending = 1;
      }
      const unsigned char* hb = hbuf + buf * halo_bytes;
      const int kq0 = (ctB[ch].w >> 2) + h;  // this lane's k-quad inside a tap
      int4 tq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) tq[i] = reinterpret_cast<const int4*>(ttab)[i];
      // software pipeline over the (compile-time) taps: fragments of tap t+1 are read into the
      // other half of a ping-pong register set before tap t's MFMAs
      f32x4 af[2], bw[2][NB];
      auto load_tap = [&](int t, int sl) {
        const int tv = tq[t >> 2][t & 3];
        const int p = prow0 + (tv & 0xffff);
        const int kq = (tv >> 16) + kq0;
        af[sl] = *reinterpret_cast<const f32x4*>(hb + p * 32 + ((h ^ swz(p)) << 4));
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          bw[sl][nb] = *reinterpret_cast<const f32x4*>(wl + (kq * NBW + nb * 32 + l32) * 16);
      };
      load_tap(0, 0);
      if constexpr (DBG == 2) load_tap(1 % NTAPS, 1);
#pragma unroll
      for (int t = 0; t < NTAPS; ++t) {
        if (DBG != 2 && t + 1 < NTAPS) load_tap(t + 1, (t + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = (t * 4 + j) % NS;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            if constexpr (DBG == 3)
              acc[q][nb][j] += af[t & 1][j] * bw[t & 1][nb][j];
            else if (DBG == 6 && wave >= 4)
              acc[q][nb][j] += af[t & 1][j] * bw[t & 1][nb][j];
            else if (DBG == 7 && wave < 4)
              acc[q][nb][j] += af[t & 1][j] * bw[t & 1][nb][j];
            else
              acc[q][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[t & 1][j], bw[t & 1][nb][j],
                                                                acc[q][nb], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DBG == 5) {  // per-tap marks of the first chunk of the first tile
          if (ti == 0 && ch == 1) mark();
        }
      }
      mark();
      buf ^= 1;
    }
    // ---- tile epilogue: stats now, the (static number of) stores one chunk step later -----
    const int fo = cur.fb * FT + wave;
    const int to0 = cur.tb * TT;
    obase = (int64_t)cur.b * oB + (int64_t)(fo * of_mul + of_add) * oF + (int64_t)to0 * oT;
    omask = 0;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const bool nok = coff[nb] >= 0;
      float sm = 0.f, sq = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;  // MFMA C row = output time offset
        const bool ok = nok && fo < Fo && to0 + row < To;
        float v = acc[0][nb][r];
#pragma unroll
        for (int q = 1; q < NS; ++q) v += acc[q][nb][r];
        if (ok) {
          sm += v;
          sq = fmaf(v, v, sq);
        }
        ov[nb][r] = v;
        omask |= (ok ? 1u : 0u) << (nb * 16 + r);
      }
      st_s[nb] += (double)sm;
      st_q[nb] += (double)sq;
    }
    have_out = true;
    advance(cur);
    mark();
  }
  if (have_out) flush();
  mark();

  if (d.stats || a.f.acc) {  // workgroup partial: lanes (h halves) and waves in a fixed order
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // reuse the halo buffers: [NW][NBW][2]
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const double s2 = st_s[nb] + __shfl_xor(st_s[nb], 32, 64);
      const double q2 = st_q[nb] + __shfl_xor(st_q[nb], 32, 64);
      if (h == 0) {
        red[(wave * NBW + nb * 32 + l32) * 2] = s2;
        red[(wave * NBW + nb * 32 + l32) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    if (a.f.acc) {  // folded finalize: waves in the same fixed order
      bnfold_commit(a.f, d.N, [&](int n, double& S, double& Q) {
        S = 0.0;
        Q = 0.0;
        for (int w = 0; w < NW; ++w) {
          S += red[(w * NBW + n) * 2];
          Q += red[(w * NBW + n) * 2 + 1];
        }
      }, reinterpret_cast<int*>(red + NW * NBW * 2), blockIdx.x, gridDim.x);
    } else if (blockIdx.x < a.nblk128) {
      for (int n = tid; n < d.N; n += 512) {
        double S = 0.0, Q = 0.0;
        for (int w = 0; w < NW; ++w) {
          S += red[(w * NBW + n) * 2];
          Q += red[(w * NBW + n) * 2 + 1];
        }
        d.stats[((int64_t)blockIdx.x * a.stats_ld + n) * 2] = S;
        d.stats[((int64_t)blockIdx.x * a.stats_ld + n) * 2 + 1] = Q;
      }
    }
  }
}

// Plan + eligibility (host).  Returns false (engine path) when the layer does not fit.
static bool halo32_plan(const clskd_conv_desc& d, Halo32Args& a, size_t& lds) {
  using namespace h32;
  if (d.in_dtype != CLSKD_F32 || d.compute != CLSKD_F32 || d.out_dtype != CLSKD_F32) return false;
  if (d.accumulate || d.wlayout != CLSKD_WLAYOUT_NK) return false;
  if (d.N < 1 || d.N > 64 || d.ntaps < 1 || d.ntaps > 16 || d.stride_t != 1) return false;
  if (d.stride_f < 1 || d.stride_f > 2 || d.ctot < CW || d.ctot % CW) return false;
  a.d = d;
  int nch = 0, kofs = 0;
  for (int s = 0; s < d.nseg; ++s) {
    const clskd_seg& g = d.seg[s];
    if (d.seg_c[s] % CW) return false;
    if (((uintptr_t)g.ptr & 15) || g.sB % 4 || g.sF % 4 || g.sT % 4) return false;
    if (g.sB > INT32_MAX || g.sF > INT32_MAX || g.sT > INT32_MAX) return false;
    for (int c0 = 0; c0 < d.seg_c[s]; c0 += CW) {
      if (nch >= MAXCH) return false;
      a.chunk_seg[nch] = s;
      a.chunk_c0[nch] = c0;
      a.chunk_kofs[nch] = kofs + c0;
      ++nch;
    }
    kofs += d.seg_c[s];
  }
  if (kofs != d.ctot || d.ntaps * d.ctot > d.K || d.K % 4) return false;
  if (((uintptr_t)d.weight & 15)) return false;
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
  if (a.HF > 255 || a.HT > 255) return false;
  a.NPIX = a.HF * a.HT;
  for (int t = 0; t < 16; ++t) {
    a.tap_pix[t] = t < d.ntaps ? (d.tap_df[t] - dfmin) * a.HT + (d.tap_dt[t] - dtmin) : 0;
    a.tap_kq[t] = t < d.ntaps ? t * d.ctot / 4 : 0;
  }
  if (a.NPIX >= 65536 || (d.ntaps - 1) * d.ctot / 4 >= 32768) return false;
  a.NGH = (int)cdiv((int64_t)a.NPIX * 2, 64 * NW);  // 2 x 16-B slots per pixel
  if (a.NGH > MAXG) return false;
  a.halo_bytes = NW * a.NGH * 1024;
  a.k4 = d.ntaps * d.ctot / 4;
  const int NBW = d.N <= 32 ? 32 : 64;
  lds = 2 * (size_t)a.halo_bytes + (size_t)a.k4 * NBW * 16 + 2 * MAXCH * 16 + 16 * 4;
  if (lds > 160 * 1024) return false;
  if ((d.stats || d.bn_fold) && (size_t)NW * NBW * 16 + 16 > 2 * (size_t)a.halo_bytes) return false;
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

static int launch_halo32_planned(const Halo32Args& a, size_t lds, hipStream_t st, bool* launched) {
  const clskd_conv_desc& d = a.d;
  *launched = false;
  static int ncu = [] {
    int v = 256;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
    return v > 0 ? v : 256;
  }();
  const int grid = a.ntiles < ncu ? a.ntiles : ncu;
  if (d.stats && grid > a.nblk128) return CLSKD_OK;  // (never for eligible shapes)
#define H32_LAUNCH(NB_, NT_, ...)                                                              \
  do {                                                                                         \
    auto k = conv_halo_f32_kernel<NB_, NT_, ##__VA_ARGS__>;                                                 \
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,      \
                              160 * 1024);                                                     \
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, st, a);                                  \
    note_kernel_fn((const void*)k);                                                            \
    note_kernel("conv_halo_f32_kernel<%d,%d>", NB_, NT_);                                      \
  } while (0)
#define H32_NT(NT_)                                                                            \
  do {                                                                                         \
    if (d.N <= 32) H32_LAUNCH(1, NT_); else H32_LAUNCH(2, NT_);                                \
  } while (0)
#ifdef CLSKD_EXPERIMENTS
  if (const int dbg = knob(KNOB_H32_DEBUG_MODE)) {  // timing-only modes on the 64 x 10-tap shape
    if (d.N <= 32 || d.ntaps != 10) return CLSKD_OK;
    switch (dbg) {
      case 1: H32_LAUNCH(2, 10, 1); break;
      case 2: H32_LAUNCH(2, 10, 2); break;
      case 3: H32_LAUNCH(2, 10, 3); break;
      case 4: H32_LAUNCH(2, 10, 4); break;
      case 5: H32_LAUNCH(2, 10, 5); break;
      case 6: H32_LAUNCH(2, 10, 6); break;
      case 7: H32_LAUNCH(2, 10, 7); break;
      case 8: H32_LAUNCH(2, 10, 8); break;
      case 9: H32_LAUNCH(2, 10, 9); break;
      default: return CLSKD_OK;
    }
    *launched = true;
    return CLSKD_OK;
  }
#endif
  switch (d.ntaps) {
    case 4: H32_NT(4); break;
    case 6: H32_NT(6); break;
    case 9: H32_NT(9); break;
    case 10: H32_NT(10); break;
    default: return CLSKD_OK;  // not a built tap count: engine path
  }
#undef H32_NT
#undef H32_LAUNCH
  *launched = true;
  return CLSKD_OK;
}

// fp32 layers with 32 <= N <= 64 and the (tap, segment, channel) K structure whose weights fit
// LDS beside the halo buffers and with at least one full 8-row F tile: the halo kernel;
// *launched = false leaves the layer to the engine.  Measured on the student's C2 layers
// (tools/conv_census.py): enc2 54 vs 60 us, enc3 83 vs 94, decoder 32-channel parities 107 / 80
// vs 138 / 88.  Layers that need the two-launch column split (64 x K >= 512 weights) or have
// Fo < 8 (half the waves idle) measured slower than the engine (e.g. the 4-row encoder layer 119
// vs 64 us); CLSKD_HALO32_SPLIT=1 still takes them (the split path stays parity-tested).
// Whether launch_conv_halo_f32 would take the layer (the same plans, nothing launched).
bool conv_halo_f32_takes(const clskd_conv_desc& d) {
  Halo32Args a;
  size_t lds = 0;
  const int min_n = knob(KNOB_HALO32_MIN_N);
  if (d.N < (min_n > 0 ? min_n : 32)) return false;
  const bool split_ok = knob(KNOB_HALO32_SPLIT) == 1;
  if (!split_ok && d.Fo < h32::FT) return false;
  if (halo32_plan(d, a, lds)) return true;
  if (!split_ok || d.N <= 32 || d.N > 64 || d.nlo < d.N) return false;
  clskd_conv_desc d1 = d, d2 = d;
  d1.N = 32;
  d2.N = d.N - 32;
  Halo32Args a2;
  size_t lds2 = 0;
  return halo32_plan(d1, a, lds) && halo32_plan(d2, a2, lds2);
}

int launch_conv_halo_f32(const clskd_conv_desc& d, hipStream_t st, bool* launched) {
  Halo32Args a;
  size_t lds = 0;
  *launched = false;
  // 16-wide layers run with the 32-column block half idle (zero weight columns, masked stores);
  // CLSKD_HALO32_MIN_N selects the narrowest N taken (A/B knob)
  const int min_n = knob(KNOB_HALO32_MIN_N);
  if (d.N < (min_n > 0 ? min_n : 32)) return CLSKD_OK;
  const bool split_ok = knob(KNOB_HALO32_SPLIT) == 1;
  if (!split_ok && d.Fo < h32::FT) return CLSKD_OK;
  if (halo32_plan(d, a, lds)) return launch_halo32_planned(a, lds, st, launched);
  if (!split_ok || d.N <= 32 || d.N > 64 || d.nlo < d.N) return CLSKD_OK;
  Halo32Args a2;
  size_t lds2 = 0;
  clskd_conv_desc d1 = d, d2 = d;
  d1.N = 32;
  d2.N = d.N - 32;
  d2.weight = reinterpret_cast<const float*>(d.weight) + (int64_t)32 * d.K;
  if (d.bias) d2.bias = d.bias + 32;
  d2.out = reinterpret_cast<float*>(d.out) + (int64_t)32 * d.oNlo;
  if (d.stats) d2.stats = d.stats + 64;
  if (!halo32_plan(d1, a, lds) || !halo32_plan(d2, a2, lds2)) return CLSKD_OK;
  a.stats_ld = a2.stats_ld = d.N;
  if (a.f.acc) {  // column halves: the second one (channels +32) finalizes the layer
    a2.f = a.f;
    a.f.finalize = 0;
    a2.f.c_off += 32;
  }
  bool l1 = false, l2 = false;
  int rc = launch_halo32_planned(a, lds, st, &l1);
  if (rc != CLSKD_OK || !l1) return rc;
  rc = launch_halo32_planned(a2, lds2, st, &l2);
  if (rc == CLSKD_OK && !l2) {
    set_error("conv halo f32: second column half not launchable");
    return CLSKD_E_ARG;
  }
  *launched = true;
  return rc;
}

}  // namespace clskd

// Timeline marks of the last DBG == 5 launch (experiments build only; 100 MHz ticks).
extern "C" int clskd_h32_marks(int64_t* out, int32_t n) {
#ifdef CLSKD_EXPERIMENTS
  CLSKD_CHECK_ARG(out && n > 0 && n <= 128, "h32_marks: n");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(clskd::g_h32_marks), sizeof(int64_t) * n) != hipSuccess) {
    clskd::set_error("h32_marks: copy failed");
    return CLSKD_E_ARG;
  }
  return CLSKD_OK;
#else
  (void)out;
  (void)n;
  clskd::set_error("h32_marks: experiments build only");
  return CLSKD_E_ARG;
#endif
}
