// Halo-tiled bf16 convolution for the WIDE layers (N = 128 / 256): the teacher's encoder 3-5 and
// decoder 0-3 (5x2 / polyphase taps, tools_for_model.py:236-262, 303-330) and the ReviewKD 3x3
// convs with 128 / 256 outputs (framework.py:189-191) — the layers conv_gemm8 runs as an im2col
// implicit GEMM.
//
// conv_gemm8 stages every input pixel once per tap (6-10x) as the A operand: 64 KB of LDS-DMA per
// 256x256x64 K-tile, 32 KB of it gathered input rows.  Its timing ablations (round 4,
// tools/g8_plain.sh: enc3 full 150 us, no DMA 117, no MFMA 104, neither 53) put the DMA staging
// on top of the MFMA work instead of under it, and the measured LDS-DMA gather rate of one CU
// (tools/probe/stage_rate.hip: 49 GB/s with 8 waves, L2-resident rows) is below the 75 GB/s a
// 256x256 tile needs to keep its MFMAs fed.  Here the A operand is staged once per 32-channel
// chunk as a halo and read by every tap through a shifted pixel map (conv_halo.hip's scheme),
// and only the weights stream per (chunk, tap) step:
//   * tile = 256 output pixels (8 F-rows x 32 time steps, or 4 x 64 when Fo = 4) x BN columns;
//     eight 32-row blocks; 8 waves as WM (row blocks) x WN (column blocks), each a
//     FM x FN grid of v_mfma_f32_32x32x16 accumulators (256: 2 x 4 waves, 4 x 2 tiles each);
//   * per chunk: the input halo ((FT-1)*stride_f + taps_F) x (TT-1 + taps_T) pixels x 64 B,
//     LDS-DMA'd into one of two halo buffers while the previous chunk computes (64-B pixel rows,
//     16-B chunks XOR-swizzled by (pixel >> 2) & 3, out-of-bounds pixels from a zero page);
//   * per (chunk, tap) step: the BN x 32 weight slab [n][32 channels] (64-B rows, the same
//     swizzle by n) LDS-DMA'd two steps ahead into a three-stage ring; one counted vmcnt wait and
//     one barrier per step;
//   * persistent workgroups (one per CU) over a contiguous run of tiles; the DMA streams run
//     across tile boundaries; BatchNorm statistics accumulate per workgroup in fp64 (partial slot
//     b, or the folded finalize of bnfold.h), as in conv_halo.
// Staged bytes per 256x256x32 step: 16 KB weights + ~4 KB of input (a 40 KB halo per 10 taps)
// against 32 KB in conv_gemm8.  Same descriptor contract (K ordered tap, segment, channel;
// ntaps / ctot / seg_c / tap_df / tap_dt given), output map, bias and statistics semantics.
#include <stdlib.h>

#include "bnfold.h"
#include "common.h"

namespace clskd {

__device__ __attribute__((aligned(64))) unsigned char g_hw_zero[64];

namespace hw {
constexpr int NW = 8;      // waves
constexpr int CW = 32;     // channels per chunk: 64-B pixel / weight rows
constexpr int MAXG = 7;    // halo DMA instructions per wave per chunk
constexpr int MAXCH = 32;  // chunks
constexpr int BST = 3;     // weight-slab ring stages (two steps in flight)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ int swz(int r) { return (r >> 2) & 3; }  // 64-B rows, 16-B chunks

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

// barrier that leaves LDS-DMA in flight (this wave's LDS reads retired first)
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int sconst(int v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int64_t vconst64(int64_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
}  // namespace hw

struct HwArgs {
  clskd_conv_desc d;
  int32_t nchunk;
  int32_t chunk_seg[hw::MAXCH];
  int32_t chunk_c0[hw::MAXCH];    // channel offset inside the segment
  int32_t chunk_kofs[hw::MAXCH];  // k offset of the chunk inside one tap's ctot channels
  int32_t dfmin, dtmin;           // halo origin relative to (fo*stride_f, to)
  int32_t HF, HT, NPIX;           // halo extent (pixels) and count
  int32_t NGH;                    // halo DMA wave-instructions per wave per chunk
  int32_t halo_bytes;             // bytes per halo buffer (ceil(NPIX / 16) KiB)
  int32_t nfb, ntb, ntiles;       // tile grid: F-blocks, T-blocks, total
  int32_t nblk128;                // statistics slots (ceil(M/128))
  int32_t tap_pix[16];            // halo pixel offset of tap t for output (0, 0)
  int32_t vec;                    // 16-B output row chunks (channel-contiguous, aligned output)
  BnFoldArgs f;
};

// Loop-invariant values the kernel re-reads from LDS where it needs them (the tile epilogue, the
// once-per-chunk halo issue): kept out of the step loop's registers (hipcc keeps hoisted kernel
// arguments live in SGPRs and spills them into VGPR lanes otherwise).
struct HwConsts {
  int64_t oB, oF, oT;
  uint64_t out;
  int32_t Fo, To, of_mul, of_add;
  int32_t nchunk, ntb, nfb, NGH, NPIX, HT, sfr, dfmin, dtmin, ctot, K, N, vec;
};

// BN output columns (128 | 256), WM x (8 / WM) waves, TT time steps per tile row (32 | 64),
// NTAPS taps.
template <int BN, int WM, int TT, typename OutT, int NTAPS, typename InT>
__global__ __launch_bounds__(512) void conv_halow_kernel(const HwArgs a) {
  using namespace hw;
  constexpr int WN = NW / WM;
  constexpr int FM = 8 / WM;               // 32-row blocks per wave
  constexpr int FN = BN / 32 / WN;         // 32-column blocks per wave
  constexpr int FT = 256 / TT;             // F-rows per tile
  constexpr int RBF = TT / 32;             // row blocks per F-row
  constexpr int SLAB = BN * 64;            // bytes per weight slab
  constexpr int GB = SLAB / 1024 / NW;     // weight DMA instructions per wave per step
  static_assert(FM >= 1 && FN >= 1 && GB >= 1 && WM * WN == NW, "tile split");
  static_assert(NTAPS >= 3 && NTAPS <= 16, "taps");
  const clskd_conv_desc& d = a.d;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int halo_bytes = __builtin_amdgcn_readfirstlane(a.halo_bytes);
  unsigned char* hbuf = smem;                                    // [2][halo_bytes]
  unsigned char* wst = smem + 2 * halo_bytes;                    // [BST][SLAB]
  int4* ctA = reinterpret_cast<int4*>(wst + BST * SLAB);         // [MAXCH] {base lo, hi, sF, sT}
  int4* ctB = ctA + MAXCH;                                       // [MAXCH] {sB, F, T, kofs}
  int* ttab = reinterpret_cast<int*>(ctB + MAXCH);               // [16] tap halo pixel offsets
  HwConsts* kc = reinterpret_cast<HwConsts*>(ttab + 16);
  float* bias_l = reinterpret_cast<float*>(kc + 1);              // [BN]
  int64_t* coff_l = reinterpret_cast<int64_t*>(bias_l + BN);     // [BN] (-1: n >= N)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int l32 = lane & 31, h = lane >> 5;

  if (tid < a.nchunk) {
    const int sg = a.chunk_seg[tid];
    const clskd_seg& S = d.seg[sg];
    const uint64_t base = (uint64_t)(uintptr_t)(reinterpret_cast<const InT*>(S.ptr) + a.chunk_c0[tid]);
    ctA[tid] = make_int4((int)(unsigned)base, (int)(unsigned)(base >> 32), (int)S.sF, (int)S.sT);
    ctB[tid] = make_int4((int)S.sB, S.F, S.T, a.chunk_kofs[tid]);
  }
  if (tid < 16) ttab[tid] = a.tap_pix[tid];
  if (tid == 0) {
    HwConsts c;
    c.oB = d.oB;
    c.oF = d.oF;
    c.oT = d.oT;
    c.out = (uint64_t)(uintptr_t)d.out;
    c.Fo = d.Fo;
    c.To = d.To;
    c.of_mul = d.of_mul;
    c.of_add = d.of_add;
    c.nchunk = a.nchunk;
    c.ntb = a.ntb;
    c.nfb = a.nfb;
    c.NGH = a.NGH;
    c.NPIX = a.NPIX;
    c.HT = a.HT;
    c.sfr = d.stride_f;
    c.dfmin = a.dfmin;
    c.dtmin = a.dtmin;
    c.ctot = d.ctot;
    c.K = d.K;
    c.N = d.N;
    c.vec = a.vec;
    *kc = c;
  }
  for (int n = tid; n < BN; n += 512) {
    bias_l[n] = (d.bias && n < d.N) ? d.bias[n] : 0.f;
    coff_l[n] = n < d.N ? (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo : -1;
  }
  if (d.stats) {  // partial slots past the grid are zero (the slot contract of include/clskd.h)
    for (int64_t s = (int64_t)blockIdx.x + gridDim.x; s < a.nblk128; s += gridDim.x)
      for (int i = tid; i < d.N * 2; i += 512) d.stats[s * d.N * 2 + i] = 0.0;
  }
  const int per = (a.ntiles + (int)gridDim.x - 1) / (int)gridDim.x;
  const int tile_begin = blockIdx.x * per;
  const int ntile_blk = max(0, min(a.ntiles, tile_begin + per) - tile_begin);
  const unsigned short* wg = reinterpret_cast<const unsigned short*>(d.weight);
  __syncthreads();

  const int nchunk = __builtin_amdgcn_readfirstlane(kc->nchunk);
  const int ntb = __builtin_amdgcn_readfirstlane(kc->ntb), nfb = __builtin_amdgcn_readfirstlane(kc->nfb);
  const int HT = __builtin_amdgcn_readfirstlane(kc->HT);
  const int rowstep = __builtin_amdgcn_readfirstlane(kc->sfr * HT);  // halo pixels per tile F-row
  const uint64_t zero_addr = (uint64_t)(uintptr_t)g_hw_zero;
  const unsigned hlds0 = __builtin_amdgcn_readfirstlane(hw::lds_addr(hbuf));
  const unsigned wlds0 = __builtin_amdgcn_readfirstlane(hw::lds_addr(wst));
  // halo pixel of (this wave's first row block, time l32); row block i adds rb_pix(i)
  const int pb0 = ((wm * FM) / RBF) * rowstep + ((wm * FM) % RBF) * 32 + l32;
  auto rb_pix = [&](int i) {  // compile-time i: FM row blocks of the wave
    const int rb = wm * FM + i, r0 = wm * FM;
    return (rb / RBF - r0 / RBF) * rowstep + (rb % RBF - r0 % RBF) * 32;
  };

  struct Cur { int b, fb, tb; };
  auto advance = [&](Cur& c) {
    if (++c.tb == ntb) {
      c.tb = 0;
      if (++c.fb == nfb) { c.fb = 0; ++c.b; }
    }
  };
  auto cur_of = [&](int tile) {
    Cur c;
    c.tb = tile % ntb;
    const int r = tile / ntb;
    c.fb = r % nfb;
    c.b = r / nfb;
    return c;
  };
  // halo of chunk ch of tile c into halo buffer hb (pieces: this wave's NGH KiB of the buffer;
  // slot = (wave * NGH + i) * 64 + lane, pixel = slot / 4, 16-B chunk = slot % 4)
  auto issue_halo = [&](const Cur& c, int ch, int hb) -> int {
    const int NGH = __builtin_amdgcn_readfirstlane(kc->NGH);
    const int NPIX = kc->NPIX;
    // pieces past the halo (the last waves' tail) are not issued: the buffer holds
    // ceil(NPIX / 16) KiB, not NW * NGH
    const int nown = max(0, min(NGH, ((NPIX + 15) >> 4) - wave * NGH));
    const int4 ea = ctA[ch];
    const int4 eb = ctB[ch];
    const InT* base = reinterpret_cast<const InT*>(((uint64_t)(unsigned)ea.y << 32) | (unsigned)ea.x) +
                      (int64_t)c.b * eb.x;
    const int fi_lo = c.fb * FT * kc->sfr + kc->dfmin, ti_lo = c.tb * TT + kc->dtmin;
    const float inv_ht = 1.0f / (float)HT;
    const unsigned dst = hlds0 + hb * halo_bytes;
    for (int i = 0; i < nown; ++i) {
      const int slot = (wave * NGH + i) * 64 + lane;
      const int p = slot >> 2;
      const int hf = (int)(((float)p + 0.5f) * inv_ht);
      const int ht = p - hf * HT;
      const int fi = fi_lo + hf, ti = ti_lo + ht;
      const bool ok = p < NPIX && (unsigned)fi < (unsigned)eb.y && (unsigned)ti < (unsigned)eb.z;
      const uint64_t src = ok ? (uint64_t)(uintptr_t)(base + (int64_t)fi * ea.z + (int64_t)ti * ea.w +
                                                      (((slot & 3) ^ swz(p)) << 3))
                              : zero_addr;
      glds16((const void*)src, dst + (wave * NGH + i) * 1024);
    }
    return nown;
  };
  // weight slab of (chunk ch, tap t) into ring stage st: piece q = wave * GB + i covers slab
  // rows 16q .. 16q + 15; lane -> row 16q + lane / 4, 16-B chunk lane % 4
  auto issue_slab = [&](int ch, int t, int st) {
    const int Kw = kc->K, Nn = kc->N;
    const int koff = t * kc->ctot + ctB[ch].w;  // K order (tap, segment, channel)
    const unsigned dst = wlds0 + st * SLAB;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int n = (wave * GB + i) * 16 + (lane >> 2);
      const uint64_t src = n < Nn ? (uint64_t)(uintptr_t)(wg + n * Kw + koff + (((lane & 3) ^ swz(n)) << 3))
                                  : zero_addr;
      glds16((const void*)src, dst + (wave * GB + i) * 1024);
    }
  };

  f32x16 acc[FM][FN];
  double st_s[FN], st_q[FN];
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) st_s[jj] = st_q[jj] = 0.0;

  const int S = nchunk * NTAPS;        // steps per tile
  const int total = ntile_blk * S;     // steps of this workgroup
  // issue cursors: the halo stream (one chunk ahead) and the weight stream (two steps ahead)
  Cur hcur = cur_of(tile_begin);
  int h_ch = 0, h_left = ntile_blk * nchunk, h_buf = 0;
  auto issue_next_halo = [&]() -> int {
    if (h_left <= 0) return 0;
    const int n = issue_halo(hcur, h_ch, h_buf);
    h_buf ^= 1;
    --h_left;
    if (++h_ch == nchunk) { h_ch = 0; advance(hcur); }
    return n;
  };
  int w_ch = 0, w_t = 0, w_issued = 0;
  auto issue_next_slab = [&]() -> int {
    if (w_issued >= total) return 0;
    issue_slab(w_ch, w_t, w_issued % BST);
    ++w_issued;
    if (++w_t == NTAPS) { w_t = 0; if (++w_ch == nchunk) w_ch = 0; }
    return GB;
  };
  if (total > 0) {
    issue_next_halo();   // chunk 0
    issue_next_slab();   // step 0
    issue_next_slab();   // step 1
    hw::wait_vm<MAXG + 2 * GB>(total > 1 ? GB : 0);  // halo 0 and slab 0 landed
  }
  raw_barrier();

  Cur cur = cur_of(tile_begin);
  int gs = 0;
  int hprev = 0;  // halo pieces issued in the previous step (after its slab)
  for (int ti = 0; ti < ntile_blk; ++ti) {
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      const float bv = bias_l[wn * (BN / WN) + jj * 32 + l32];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = bv;
    }
    int t = 0, kch = ti * nchunk;  // kch: the workgroup's chunk count (halo buffer kch & 1)
    for (int s = 0; s < S; ++s, ++gs) {
      // this step's slab and halo are visible; stage (gs + 2) % BST was last read in step gs - 1.
      // Order: fragments of k16 0 -> its 8 MFMAs -> fragments of k16 1 -> the DMA issue of
      // later steps (its issue stalls hide under the queued MFMAs) -> the 8 MFMAs of k16 1
      const unsigned char* ws = wst + (gs % BST) * SLAB;
      const unsigned char* hb = hbuf + (kch & 1) * halo_bytes;
      const int pt = pb0 + ttab[t];  // the tap's halo pixel offset (LDS broadcast)
      bf16x8_t af[2][FM], bw[2][FN];
      auto read_k16 = [&](int k16) {
        const int c = k16 * 2 + h;
        // row block i's pixel = pt + rb_pix(i), rb_pix(i) a multiple of 16: same swizzle
        const unsigned char* a0 = hb + pt * 64 + ((c ^ swz(pt)) << 4);
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[k16][i] = *reinterpret_cast<const bf16x8_t*>(a0 + rb_pix(i) * 64);
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) {
          const int n = wn * (BN / WN) + jj * 32 + l32;
          bw[k16][jj] = *reinterpret_cast<const bf16x8_t*>(ws + n * 64 + ((c ^ swz(n)) << 4));
        }
      };
      auto mfma_k16 = [&](int k16) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int jj = 0; jj < FN; ++jj) acc[i][jj] = mfma16<InT>(af[k16][i], bw[k16][jj], acc[i][jj]);
      };
      read_k16(0);
      mfma_k16(0);
      read_k16(1);
      __builtin_amdgcn_sched_barrier(0);
      const int ib = issue_next_slab();
      const int ih = t == 0 ? issue_next_halo() : 0;
      __builtin_amdgcn_sched_barrier(0);
      mfma_k16(1);
      // the next step's slab (issued one step ago) and, at a chunk's last tap, the next
      // chunk's halo (issued at its first tap) have landed; younger pieces stay in flight
      hw::wait_vm<MAXG + GB>(ib + ih + (t == 1 ? hprev : 0));
      hprev = ih;
      raw_barrier();
      if (++t == NTAPS) {
        t = 0;
        ++kch;
      }
    }
    // ---- tile epilogue: statistics + stores (the accumulators only; the DMA streams of the
    // next tile are already in flight).  The halo buffer of the chunk just finished is free until
    // the next step's halo issue (after the barrier below): each wave stages one 32x32 output tile
    // at a time there and writes it back as 16-B row chunks (channel-contiguous outputs only).
    {
      const int Fo = kc->Fo, To = kc->To;
      const int64_t oB = kc->oB, oF = kc->oF, oT = kc->oT;
      const int of_mul = kc->of_mul, of_add = kc->of_add;
      using GOut = __attribute__((address_space(1))) OutT;
      GOut* const outp = reinterpret_cast<GOut*>(kc->out);
      const int fo0 = cur.fb * FT, to0 = cur.tb * TT;
      constexpr int CH = 16 / (int)sizeof(OutT);       // elements per 16-B chunk
      constexpr int UB = 32 * 32 * (int)sizeof(OutT);  // bytes per staged tile
      constexpr int CPRW = 32 / CH;                    // chunks per staged row
      const int Nn = kc->N;
      OutT* wt = reinterpret_cast<OutT*>(hbuf + ((kch - 1) & 1) * halo_bytes + wave * UB);
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const int nb = wn * (BN / WN) + jj * 32;
        const int64_t coff = coff_l[nb + l32];
        const bool nok = coff >= 0;
        float sm = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int rb = wm * FM + i;
          const int fo = fo0 + rb / RBF;
          const int tb0 = to0 + (rb % RBF) * 32;
          const int64_t rowb = (int64_t)cur.b * oB + (int64_t)(fo * of_mul + of_add) * oF;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
            const float v = acc[i][jj][r];
            if (nok && fo < Fo && tb0 + rr < To) {
              sm += v;
              sq = fmaf(v, v, sq);
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r)
            wt[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + l32] = (OutT)acc[i][jj][r];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: tile written
#pragma unroll
          for (int q0 = 0; q0 < 32 * CPRW; q0 += 64) {
            const int q = q0 + lane;
            const int rr = q / CPRW, cc = q % CPRW;
            const int n = nb + cc * CH;
            if (fo < Fo && tb0 + rr < To && n < Nn)
              *reinterpret_cast<__attribute__((address_space(1))) hw::u32x4*>(
                  outp + rowb + (int64_t)(tb0 + rr) * oT + n) =
                  *reinterpret_cast<const hw::u32x4*>(wt + rr * 32 + cc * CH);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: tile read back
          __builtin_amdgcn_sched_barrier(0);
        }
        st_s[jj] += (double)sm;
        st_q[jj] += (double)sq;
      }
      raw_barrier();  // staging reads done before the next step's halo DMA reuses the buffer
    }
    advance(cur);
  }

  if (d.stats || a.f.acc) {  // workgroup partial: lane halves and row-block waves in a fixed order
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    double* red = reinterpret_cast<double*>(smem);  // reuse the halo buffers: [WM][BN][2]
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      const double s2 = st_s[jj] + __shfl_xor(st_s[jj], 32, 64);
      const double q2 = st_q[jj] + __shfl_xor(st_q[jj], 32, 64);
      if (h == 0) {
        const int col = wn * (BN / WN) + jj * 32 + l32;
        red[(wm * BN + col) * 2] = s2;
        red[(wm * BN + col) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    if (a.f.acc) {
      bnfold_commit(a.f, d.N, [&](int n, double& Sx, double& Qx) {
        Sx = 0.0;
        Qx = 0.0;
        for (int w = 0; w < WM; ++w) {
          Sx += red[(w * BN + n) * 2];
          Qx += red[(w * BN + n) * 2 + 1];
        }
      }, reinterpret_cast<int*>(red + WM * BN * 2), blockIdx.x, gridDim.x);
    } else if (blockIdx.x < a.nblk128) {
      for (int n = tid; n < d.N; n += 512) {
        double Sx = 0.0, Qx = 0.0;
        for (int w = 0; w < WM; ++w) {
          Sx += red[(w * BN + n) * 2];
          Qx += red[(w * BN + n) * 2 + 1];
        }
        d.stats[((int64_t)blockIdx.x * d.N + n) * 2] = Sx;
        d.stats[((int64_t)blockIdx.x * d.N + n) * 2 + 1] = Qx;
      }
    }
  }
}

// Plan + eligibility (host).  Returns false (conv_gemm8 path) when the layer does not fit.
static bool halow_plan(const clskd_conv_desc& d, HwArgs& a, size_t& lds, int& tt, int& bn) {
  using namespace hw;
  if (!is_lowp(d.in_dtype) || d.N <= 64 || d.N > 256 || d.ntaps < 3 || d.ntaps > 16 ||
      d.stride_t != 1 || d.accumulate)
    return false;
  if (d.stride_f < 1 || d.stride_f > 2 || d.ctot < CW || d.Fo < 4) return false;
  if (d.out_dtype != CLSKD_F32 && d.out_dtype != d.in_dtype) return false;
  a.d = d;
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
  if (kofs != d.ctot || d.ntaps * d.ctot != d.K) return false;
  a.nchunk = nch;
  int dfmin = 1 << 20, dfmax = -(1 << 20), dtmin = 1 << 20, dtmax = -(1 << 20);
  for (int t = 0; t < d.ntaps; ++t) {
    dfmin = d.tap_df[t] < dfmin ? d.tap_df[t] : dfmin;
    dfmax = d.tap_df[t] > dfmax ? d.tap_df[t] : dfmax;
    dtmin = d.tap_dt[t] < dtmin ? d.tap_dt[t] : dtmin;
    dtmax = d.tap_dt[t] > dtmax ? d.tap_dt[t] : dtmax;
  }
  tt = d.Fo >= 8 ? 32 : 64;  // 8 x 32 tiles; 4 x 64 when the layer has 4..7 F-rows
  const int FT = 256 / tt;
  bn = d.N <= 128 ? 128 : 256;
  a.dfmin = dfmin;
  a.dtmin = dtmin;
  a.HF = (FT - 1) * d.stride_f + (dfmax - dfmin + 1);
  // halo rows padded so one F-row of the tile is a multiple of 16 pixels (rowstep = stride_f *
  // HT): every row block's pixel then has the same 16-B chunk swizzle as the wave's first one,
  // and its fragment address is the first one's plus a uniform offset (the padding pixels are
  // loaded, never read)
  const int hpad = d.stride_f == 2 ? 8 : 16;
  a.HT = (int)cdiv((tt - 1) + (dtmax - dtmin + 1), hpad) * hpad;
  if (a.HF > 255 || a.HT > 255) return false;
  a.NPIX = a.HF * a.HT;
  for (int t = 0; t < 16; ++t) {
    a.tap_pix[t] = t < d.ntaps ? (d.tap_df[t] - dfmin) * a.HT + (d.tap_dt[t] - dtmin) : 0;
  }
  a.NGH = (int)cdiv((int64_t)a.NPIX * 4, 64 * NW);  // 4 x 16-B slots per pixel
  if (a.NGH > MAXG) return false;
  a.halo_bytes = (int)cdiv(a.NPIX, 16) * 1024;  // whole 1-KiB pieces of 16 pixels
  lds = 2 * (size_t)a.halo_bytes + (size_t)BST * bn * 64 + 2 * MAXCH * 16 + 16 * 4 +
        sizeof(HwConsts) + (size_t)bn * (4 + 8);
  for (int s = 0; s < d.nseg; ++s)
    if (d.seg[s].sB > INT32_MAX || d.seg[s].sF > INT32_MAX || d.seg[s].sT > INT32_MAX) return false;
  if ((int64_t)d.N * d.K >= ((int64_t)1 << 31)) return false;
  if (lds > 160 * 1024) return false;
  if ((d.stats || d.bn_fold) && (size_t)2 * bn * 16 + 16 > 2 * (size_t)a.halo_bytes) return false;
  a.nfb = (int)cdiv(d.Fo, FT);
  a.ntb = (int)cdiv(d.To, tt);
  const int64_t nt = (int64_t)d.B * a.nfb * a.ntb;
  if (nt < 4 || nt > (1 << 30)) return false;
  a.ntiles = (int)nt;
  a.nblk128 = (int)cdiv((int64_t)d.B * d.Fo * d.To, 128);
  a.f = make_bnfold(d);
  const int ch16 = d.out_dtype == CLSKD_F32 ? 4 : 8;
  a.vec = d.oNlo == 1 && d.nlo >= d.N && d.N % ch16 == 0 && (((uintptr_t)d.out) & 15) == 0 &&
          d.oB % ch16 == 0 && d.oF % ch16 == 0 && d.oT % ch16 == 0;
  // the epilogue stages 32x32 output tiles in a free halo buffer and stores 16-B row chunks
  if (!a.vec || (size_t)NW * 32 * 32 * (d.out_dtype == CLSKD_F32 ? 4 : 2) > (size_t)a.halo_bytes)
    return false;
  return true;
}

// Whether launch_conv_halow would take the layer (CLSKD_HALOW=1; default 0 keeps the wide
// layers on conv_gemm8 — A/B switch).
bool conv_halow_takes(const clskd_conv_desc& d) {
  if (knob(KNOB_HALOW) == 0) return false;
  HwArgs a;
  size_t lds = 0;
  int tt = 0, bn = 0;
  if (!halow_plan(d, a, lds, tt, bn)) return false;
  switch (d.ntaps) {
    case 4: case 6: case 9: case 10: return true;
    default: return false;
  }
}

int launch_conv_halow(const clskd_conv_desc& d, hipStream_t st, bool* launched) {
  *launched = false;
  if (knob(KNOB_HALOW) == 0) return CLSKD_OK;
  HwArgs a;
  size_t lds = 0;
  int tt = 0, bn = 0;
  if (!halow_plan(d, a, lds, tt, bn)) return CLSKD_OK;
  static int ncu = [] {
    int v = 256;
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, 0);
    return v > 0 ? v : 256;
  }();
  // persistent grid; with partial statistics slots (one per workgroup) at most ceil(M/128)
  int grid = a.ntiles < ncu ? a.ntiles : ncu;
  if (d.stats && grid > a.nblk128) grid = a.nblk128;
  const bool f32out = d.out_dtype == CLSKD_F32;
#define HW_LAUNCH(BN_, WM_, TT_, O_, NT_, I_)                                                   \
  do {                                                                                          \
    auto k = conv_halow_kernel<BN_, WM_, TT_, O_, NT_, I_>;                                     \
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,       \
                              160 * 1024);                                                      \
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), lds, st, a);                                   \
    note_kernel_fn((const void*)k);                                                             \
    note_kernel("conv_halow_kernel<%d,%d,%d,%s,%d%s>", BN_, WM_, TT_, type_name<O_>(), NT_,     \
                __is_same(I_, _Float16) ? ",f16" : "");                                         \
  } while (0)
#define HW_TT(BN_, WM_, O_, NT_, I_)                                                            \
  do {                                                                                          \
    if (tt == 32) HW_LAUNCH(BN_, WM_, 32, O_, NT_, I_); else HW_LAUNCH(BN_, WM_, 64, O_, NT_, I_); \
  } while (0)
#define HW_NI(NT_, I_)                                                                          \
  do {                                                                                          \
    if (bn == 128) {                                                                            \
      if (f32out) HW_TT(128, 4, float, NT_, I_); else HW_TT(128, 4, I_, NT_, I_);               \
    } else {                                                                                    \
      if (f32out) HW_TT(256, 2, float, NT_, I_); else HW_TT(256, 2, I_, NT_, I_);               \
    }                                                                                           \
  } while (0)
#define HW_NT(NT_)                                                                              \
  do {                                                                                          \
    if (d.in_dtype == CLSKD_F16) HW_NI(NT_, _Float16); else HW_NI(NT_, __bf16);                 \
  } while (0)
  switch (d.ntaps) {
    case 4: HW_NT(4); break;
    case 6: HW_NT(6); break;
    case 9: HW_NT(9); break;
    case 10: HW_NT(10); break;
    default: return CLSKD_OK;  // not a built tap count: conv_gemm8
  }
#undef HW_NT
#undef HW_NI
#undef HW_TT
#undef HW_LAUNCH
  *launched = true;
  return CLSKD_OK;
}

}  // namespace clskd
