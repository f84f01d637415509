// One streaming hop of the DCCRN student (configuration C5) as ONE kernel launch.
//
// The hop-by-hop path (clskd/streaming.py, eager or hipGraph) issues ~70 small launches per
// 6.25 ms hop: ConvSTFT row, 6 encoder convs + BN/PReLU, 2 complex-LSTM steps, the projection,
// 12 polyphase decoder convs + BN/PReLU, mask 'E', the iSTFT row and the overlap-add — each a few
// hundred to a few thousand MACs per stream, so the hop is bound by launch and dependency
// latency (~10 us per node), not by arithmetic (3.8 MMAC per frame, DCCRN.py:149-240).
// Here one workgroup per stream walks the whole hop: every layer's current frame stays in LDS,
// the older frames the causal convolutions and the decoder look-ahead need live in per-stream
// rings in global memory (written by earlier hops, i.e. earlier launches: no cross-workgroup
// synchronisation at all), and the weights (3 MB of fp32 per hop, shared by every stream's
// workgroup through L2) go straight from L2 into registers in k-quad layout [K/4][N][4]: a lane
// owns one output channel and reads four k per 16-B load, a wavefront one contiguous 1 KB run,
// a batch of loads in flight per lane while the previous batch computes.  Each weight quad feeds
// up to 8 output rows and each activation quad (an LDS broadcast) 2 channels, accumulated as
// packed fp32 pairs (v_pk_fma_f32).  Layers whose output count leaves threads idle split K across threads and
// reduce through LDS, and both decoder parities run in the same pass, so every layer keeps all
// NT threads busy.  fp32 throughout, BatchNorm in eval mode (running statistics).
//
// Ring slots: frame f of a ring of depth D lives in slot ((f % D) + D) % D; rings start zeroed
// (the causal / centring zeros of the first frames).  Depths: spectrum 7 (mask of frame t-6),
// encoder output i: 7 - i (decoder 5 - i reads frames t-6+i, t-5+i), decoder input 2, decoder
// output d: 2, iSTFT frames 4 (the 400-sample window spans 4 hops).
#include "common.h"

namespace clskd {
#ifdef CLSKD_EXPERIMENTS
// phase timestamps of stream 0 (thread 0, after each phase's barrier): diagnostic only
__device__ uint64_t g_hop_marks[40];
#define CMARK(i)                                                                          \
  do {                                                                                    \
    if ((i) >= 0 && blockIdx.x == 0 && threadIdx.x == 0) g_hop_marks[i] = wall_clock64(); \
  } while (0)
#else
#define CMARK(i) \
  do {           \
  } while (0)
#endif
namespace shop {

constexpr int NT = 512;    // threads per stream workgroup (8 waves: two per SIMD)
constexpr int HOP = 100, WIN = 400, NBIN = 514, LDEST = 516;
constexpr int WINSZ = 4096;      // conv input window [2][F][Ci] ...
constexpr int ZOFF = WINSZ;      // ... followed by a zero row (out-of-range taps read it)
constexpr int RED = NT * 16;     // split-K partial sums (threads x R x CQ)

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int ring(int f, int D) { return ((f % D) + D) % D; }
// log2 of a power of two (every shape the layer helpers divide by is one: host-checked)
__device__ __forceinline__ int lg2(int v) { return 31 - __builtin_clz(v); }

__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float tanh_f(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * 2.8853900817779268f));
}
// The layer helpers below are out-of-line (one copy of each in the code object: the whole hop
// inlined was 121 KB of straight-line code, refetched from L2 by the instruction cache every hop),
// so their pointers carry explicit address spaces: LDS operands as `lds`, global ones cast to
// `gbl` — a generic pointer would turn every access into a flat one (counted on both vmcnt and
// lgkmcnt, which serialises the weight prefetch).
typedef __attribute__((address_space(3))) float lds;
typedef __attribute__((address_space(1))) const float gbl;
typedef __attribute__((address_space(3))) const f32x4 lds4;
typedef __attribute__((address_space(1))) const f32x4 gbl4;
__device__ __forceinline__ f32x4 ld4(const lds* p) { return *(lds4*)p; }
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ldg4(const float* p) { return *(gbl4*)p; }
__device__ __forceinline__ float ldg(const float* p) { return *(gbl*)p; }
__device__ __forceinline__ lds* L(float* p) { return (lds*)p; }
__device__ __forceinline__ const lds* L(const float* p) { return (const lds*)p; }
__device__ __forceinline__ void fma4(f32x2& acc, const f32x4 w, const f32x4 x) {
  acc = __builtin_elementwise_fma(w.xy, x.xy, acc);
  acc = __builtin_elementwise_fma(w.zw, x.zw, acc);
}

// Weight quads stream from global memory straight into registers, QB float4 per lane per batch
// (KB quads x CQ channels) and NB batches deep: batch b's loads issue NB - 1 batches before it
// computes, and the first NB - 1 batches issue before the layer stages its input (`pre`), so the
// staging round trip and the first weight round trip overlap.  Trip counts are uniform and the
// loads unconditional (indices clamped to the matrix; quads past a slice's end meet the zero row
// instead), so the compiler keeps the batches in flight with counted vmcnt waits.  NB = 3 ran
// the same hop time as NB = 2 (131.6 vs 131.2 us) with 256 VGPRs and spills, so NB = 2.
constexpr int QB = 8, NB = 2;

template <class T, class Load, class Comp, class Pre>
__device__ __forceinline__ void pipeline(int nbat, T (&buf)[NB], Load&& load, Comp&& comp, Pre&& pre) {
#pragma unroll
  for (int u = 0; u < NB - 1; ++u)
    if (u < nbat) load(buf[u], u);
  pre();
  for (int b0 = 0; b0 < nbat; b0 += NB) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int bt = b0 + u;
      if (bt < nbat) {
        if (bt + NB - 1 < nbat) load(buf[(u + NB - 1) % NB], bt + NB - 1);
        comp(buf[u], bt);
      }
    }
  }
}

// Convolution geometry of one layer over the LDS window win [2][F][Ci] (slot 1 = newest frame).
// Tap j: encoder (kf = j/2, kt = j%2) reads row fo*2 + kf - 2 of slot kt; decoder (per parity,
// _DEC_TAPS in model.py) reads row fo + 1 - j/2 of slot 1 - j%2.
struct Geo {
  int F, Ci, lgq, sf, dec;  // lgq = log2(Ci / 4)
};
// (bitwise selects: a conditional expression here became exec-masked branches per row)
__device__ __forceinline__ int pick(bool c, int a, int b) {
  const int m = -(int)c;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ int xrow(const Geo& g, int j, int fo, bool live = true) {
  const int tdf = g.dec ? 1 - (j >> 1) : (j >> 1) - 2;
  const int tsl = g.dec ? 1 - (j & 1) : (j & 1);
  const int fi = fo * g.sf + tdf;
  return pick(live && (unsigned)fi < (unsigned)g.F, (tsl * g.F + fi) << (g.lgq + 2), ZOFF);
}

// out[(fo*of_mul + p)*Co + co] = act(bias_p[co] + sum_k W_p[k][co] x_p(fo, k)) for fo < Fo and
// each of np parities p (W_p: K4_p quads, k-quad layout); coef: BN [scale | shift] + PReLU.
// Thread = (parity, K slice ks, row group fg, channel group cg): R rows fo = fg + FG*r times CQ
// channels co = cg*CQ + q, so each activation quad (an LDS broadcast) feeds CQ channels and each
// weight quad R rows.  S K-slices per output fill the block; partials reduce through `red`
// (np*S*Fo*Co <= NT*R*CQ floats).  PERTAP: taps narrower than a batch (Ci < 4*KB), window
// offsets per quad; else per batch (slices start on whole batches, so one tap per batch).
// stage(): fills win (called with the first weight batches in flight; a barrier follows), here
// also the bias / BN / PReLU parameters go to `prm` (np*Co + 2*Co + 1 floats).
// Requires FG*(Co/CQ)*S a multiple of 64 (the parity is wave-uniform).  Uniform across the block.
template <int R, int CQ, bool PERTAP, class Stage>
__device__ __forceinline__ void conv(const lds* win, const Geo g, int np, int K4a, int K4b, int Fo, int Co,
                                     const float* W0, const float* W1, const float* b0, const float* b1,
                                     const float* coef, const float* alpha, lds* out, int of_mul, lds* red,
                                     lds* prm, int mk, Stage&& stage) {
  constexpr int KB = QB / CQ / (PERTAP ? 2 : 1);  // per-quad offsets cost registers
  constexpr int LR = R == 8 ? 3 : 2, LQ = CQ == 2 ? 1 : 0;
  const int tid = threadIdx.x;
  // every count is a power of two: shifts and masks, no integer divisions
  const int lfo = lg2(Fo), lco = lg2(Co);
  const int lfg = lfo - LR, lcg = lco - LQ;
  const int FG = 1 << lfg, CG = 1 << lcg;
  const int ls = max(0, lg2(NT) - (np == 2 ? 1 : 0) - lfg - lcg);
  const int S = 1 << ls;
  const int lp = lfg + lcg + ls;
  const int p = __builtin_amdgcn_readfirstlane(tid >> lp);
  const int rem = tid & ((1 << lp) - 1);
  const int cg = rem & (CG - 1), fg = (rem >> lcg) & (FG - 1), ks = rem >> (lcg + lfg);
  const bool act = p < np;
  const int pc = act ? p : 0;
  const int k4n = pc ? K4b : K4a;
  int len = (k4n + S - 1) >> ls;
  len = (len + KB - 1) / KB * KB;
  const int nbat = __builtin_amdgcn_readfirstlane(act ? len / KB : 0);
  const int k0 = ks * len, k1 = min(k4n, k0 + len);
  const float* W = (pc ? W1 : W0) + cg * CQ * 4;
  const int stride = Co * 4;
  const int qm = (1 << g.lgq) - 1;
  f32x2 acc[R][CQ];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int q = 0; q < CQ; ++q) acc[r][q] = f32x2{0.f, 0.f};
  struct Batch {
    f32x4 w[KB][CQ];
  };
  Batch buf[NB];
  pipeline(
      nbat, buf,
      [&](Batch& bb, int bt) {
        const int kb = k0 + bt * KB;
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          const float* src = W + (size_t)min(kb + i, k4n - 1) * stride;
#pragma unroll
          for (int q = 0; q < CQ; ++q) bb.w[i][q] = ldg4(src + q * 4);
        }
      },
      [&](const Batch& bb, int bt) {
        const int kb = k0 + bt * KB;
        int off[R];
        if (!PERTAP) {
          const int j = kb >> g.lgq;
#pragma unroll
          for (int r = 0; r < R; ++r) off[r] = xrow(g, j, fg + FG * r, kb < k1);
        }
#pragma unroll
        for (int i = 0; i < KB; ++i) {
          const int k4 = kb + i;
          if (PERTAP) {
            const int j = k4 >> g.lgq;
#pragma unroll
            for (int r = 0; r < R; ++r) off[r] = xrow(g, j, fg + FG * r, k4 < k1);
          }
          const int c = (k4 & qm) << 2;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const f32x4 x = ld4(win + off[r] + c);
#pragma unroll
            for (int q = 0; q < CQ; ++q) fma4(acc[r][q], bb.w[i][q], x);
          }
        }
      },
      [&]() {
        stage();
        for (int q = tid; q < np * Co; q += NT) {
          const float* bp = q >= Co ? b1 : b0;
          prm[q] = bp ? ldg(bp + (q & (Co - 1))) : 0.f;
        }
        if (coef) {
          for (int q = tid; q < 2 * Co; q += NT) prm[np * Co + q] = ldg(coef + q);
          if (tid == 0) prm[np * Co + 2 * Co] = ldg(alpha);
        }
        __syncthreads();
      });
  if (mk >= 0) __syncthreads();
  CMARK(mk);
  auto fin = [&](int pp, int fo, int cc, float v) {
    v += prm[pp * Co + cc];
    if (coef) {
      v = fmaf(v, prm[np * Co + cc], prm[np * Co + Co + cc]);
      v = v >= 0.f ? v : prm[np * Co + 2 * Co] * v;
    }
    out[(fo * of_mul + pp) * Co + cc] = v;
  };
  if (S == 1) {
    if (act)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < CQ; ++q) fin(p, fg + FG * r, cg * CQ + q, acc[r][q].x + acc[r][q].y);
    return;
  }
  if (act)
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int q = 0; q < CQ; ++q)
        red[((p * S + ks) * Fo + fg + FG * r) * Co + cg * CQ + q] = acc[r][q].x + acc[r][q].y;
  __syncthreads();
  CMARK(mk < 0 ? -1 : mk + 1);
  for (int q = tid; q < (np << (lfo + lco)); q += NT) {
    const int pp = q >> (lfo + lco), o = q & ((1 << (lfo + lco)) - 1);
    float v = 0.f;
    for (int s2 = 0; s2 < S; ++s2) v += red[(((pp << ls) + s2) << (lfo + lco)) + o];
    fin(pp, o >> lco, o & (Co - 1), v);
  }
}

// One layer: R = min(Fo, 8) rows and CQ = 2 channels per thread where Co >= 16.  zero: the
// layer's output frame is out of range (staging still runs).
template <class Stage>
__device__ __forceinline__ void conv_layer(const lds* win, const Geo g, int np, int K4a, int K4b, int Fo, int Co,
                                           const float* W0, const float* W1, const float* b0, const float* b1,
                                           const float* coef, const float* alpha, lds* out, int of_mul,
                                           lds* red, lds* prm, bool zero, int mk, Stage&& stage) {
  if (zero) {
    stage();
    const int lfc = lg2(Fo) + lg2(Co);
    for (int q = threadIdx.x; q < (np << lfc); q += NT) {
      const int p = q >> lfc, o = q & ((1 << lfc) - 1);
      out[((o >> lg2(Co)) * of_mul + p) * Co + (o & (Co - 1))] = 0.f;
    }
    return;
  }
#define CONV_ARGS win, g, np, K4a, K4b, Fo, Co, W0, W1, b0, b1, coef, alpha, out, of_mul, red, prm, mk, stage
  if (Fo >= 8) {
    if (Co >= 16) {
      if (g.Ci < 16) conv<8, 2, true>(CONV_ARGS);  // (CQ = 2: KB = 4 quads, a tap of Ci >= 16 spans >= 4)
      else conv<8, 2, false>(CONV_ARGS);
    } else {
      if (g.Ci < 4 * QB) conv<8, 1, true>(CONV_ARGS);
      else conv<8, 1, false>(CONV_ARGS);
    }
  } else {
    // Fo == 4 (host-checked): encoder 5 and decoder 0 of the student, Ci >= 16 and Co >= 16
    conv<4, 2, false>(CONV_ARGS);
  }
#undef CONV_ARGS
}

// y[h*ys + n] = bias[n] + sum_k W[k][n] x[h*xs + k] for n < N, h < nh; W in k-quad layout with
// K4 quads, x in LDS (16-B aligned rows).  Units (K slice, h, n) over the block, rounds of NT
// units with uniform trip counts (idle units compute on clamped indices and do not store);
// with S > 1 slices the partials reduce through `red`.  pre(): stages x (called with the first
// weight batches of round 0 in flight; a barrier follows).  The caller synchronises before
// reading y.
template <class Pre>
__device__ __forceinline__ void gemv(const float* W, const float* bias, const lds* x, int xs, int nh, int K4, int N,
                                     lds* y, int ys, lds* red, const lds* zrow, Pre&& pre) {
  const int tid = threadIdx.x;
  const int M = nh * N;
  // K slices: the least work per thread over rounds of NT units, a round costing its quads
  // plus ~8 quads of fixed work (unit indices, partial store, the pipeline's first round trip);
  // ties: fewer slices.  (Counting quads alone picked 14 rounds of 8 quads for the STFT row.)
  int S = 1, best = 1 << 30;
  for (int s2 = 1; s2 <= 16 && s2 * M <= RED && s2 <= K4; ++s2) {
    const int cost = (s2 * M + NT - 1) / NT * ((K4 + s2 - 1) / s2 + 8);
    if (cost < best) {
      best = cost;
      S = s2;
    }
  }
  const int len = (K4 + S - 1) / S;
  const int nbat = __builtin_amdgcn_readfirstlane((len + QB - 1) / QB);
  const int U = S * M;
  struct Batch {
    f32x4 w[QB];
  };
  for (int u0 = 0; u0 < U; u0 += NT) {
    const int u = min(u0 + tid, U - 1);
    const int ks = u / M, hn = u - ks * M, h = hn / N, n = hn - h * N;
    const lds* xr = x + h * xs;
    const float* Wn = W + n * 4;
    const int k0 = ks * len, k1 = min(K4, k0 + len);
    f32x2 acc = f32x2{0.f, 0.f};
    Batch buf[NB];
    pipeline(
        nbat, buf,
        [&](Batch& bb, int bt) {
#pragma unroll
          for (int i = 0; i < QB; ++i) bb.w[i] = ldg4(Wn + (size_t)min(k0 + bt * QB + i, K4 - 1) * N * 4);
        },
        [&](const Batch& bb, int bt) {
          const int kb = k0 + bt * QB;
#pragma unroll
          for (int i = 0; i < QB; ++i) fma4(acc, bb.w[i], ld4(kb + i < k1 ? xr + (kb + i) * 4 : zrow));
        },
        [&]() {
          if (u0 == 0) {
            pre();
            __syncthreads();
          }
        });
    if (u0 + tid < U) {
      if (S == 1)
        y[h * ys + n] = acc.x + acc.y + (bias ? ldg(bias + n) : 0.f);
      else
        red[u] = acc.x + acc.y;
    }
  }
  if (S == 1) return;
  __syncthreads();
  for (int q = tid; q < M; q += NT) {
    float v = bias ? ldg(bias + q % N) : 0.f;
    for (int s2 = 0; s2 < S; ++s2) v += red[s2 * M + q];
    y[(q / N) * ys + q % N] = v;
  }
}

}  // namespace shop

#define HOP_MARK(i) CMARK(i)

__global__ __launch_bounds__(shop::NT) void stream_hop_kernel(const clskd_stream_hop_args a) {
  using namespace shop;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int t = a.t;
  float* st = a.state + (int64_t)b * a.state_stride;
  const int H = a.H, D4 = a.D4, C6 = a.enc_cout[5], Ch = C6 / 2, G4 = 4 * H;

  __shared__ __attribute__((aligned(16))) float xw[WIN];
  __shared__ __attribute__((aligned(16))) float spec[NBIN + 2];
  __shared__ __attribute__((aligned(16))) float win[WINSZ + 256];
  __shared__ __attribute__((aligned(16))) float curA[1024];
  __shared__ __attribute__((aligned(16))) float curB[1024];  // ping-pong: current frame of a layer
  __shared__ __attribute__((aligned(16))) float decin[256];
  __shared__ __attribute__((aligned(16))) float gx[2][8 * 64];
  __shared__ __attribute__((aligned(16))) float hv[2][2][64];
  __shared__ float cv[2][2][64], act[2][2][4 * 64];
  __shared__ __attribute__((aligned(16))) float rin[2][64];
  __shared__ __attribute__((aligned(16))) float est[LDEST];
  __shared__ __attribute__((aligned(16))) float frame[WIN];
  __shared__ __attribute__((aligned(16))) float red[RED];
  __shared__ __attribute__((aligned(16))) float prm[512];
  __shared__ __attribute__((aligned(16))) float whh[8 * 32 * 36];  // W_hh [2*4H][H + 4], H <= 32

  HOP_MARK(0);
#ifdef CLSKD_EXPERIMENTS
  if (b == 0 && tid == 0) {  // shader-clock rate and one dependent global round trip
    const uint64_t w0 = wall_clock64();
    g_hop_marks[38] = clock64();
    const float v = ldg(a.enc_w[3] + 64 * (t % 16));
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t c0 = clock64();
    g_hop_marks[30] = c0 - (uint64_t)(v == 12345.f);  // (v consumed: the load completes before c0)
    g_hop_marks[31] = w0;
  }
#endif
  for (int i = tid; i < 256; i += NT) win[ZOFF + i] = 0.f;
  const float* zr = win + ZOFF;  // zero row (LDS)
  // ---- input window: shift by one hop, append the new samples (tools_for_model.py:53-67)
  float* gxw = st + a.off_xwin;
  auto stage_x = [&]() {
    for (int i = tid; i < WIN; i += NT)
      xw[i] = i < WIN - HOP ? gxw[i + HOP] : (a.live ? a.x_in[(int64_t)b * HOP + i - (WIN - HOP)] : 0.f);
  };

  float* cur = curA;
  float* nxt = curB;
  if (a.live) {
    // ---- ConvSTFT row of the newest window -> spectrum ring
    gemv(a.stft_w, nullptr, L(xw), 0, 1, WIN / 4, NBIN, L(spec), 0, L(red), L(zr), stage_x);
    __syncthreads();
    HOP_MARK(1);
    // ---- encoder (DCCRN.py:171-176): window [t-1, t], taps (kf - 2, kt), stride 2 in F.
    //      The ring writes of the previous phase's output are issued in the next phase's staging,
    //      behind its first weight loads: gfx950's vmcnt counts stores, so a load issued after a
    //      store would wait for that store's acknowledgement too.
    for (int i = 0; i < 6; ++i) {
      const int Fi = 256 >> i, Fo = Fi / 2, Co = a.enc_cout[i];
      const int Ci = i == 0 ? 4 : a.enc_cin[i];  // encoder 0: (re, im) padded to a quad
      // stage [2][Fi][Ci]: slot 1 = this frame (spectrum / previous layer in LDS), slot 0 = t-1
      auto stage = [&]() {
        if (i == 0) {
          for (int j = tid; j < WIN; j += NT) gxw[j] = xw[j];  // (every read of gxw is behind gemv's barrier)
          float* sring = st + a.off_spec;
          for (int j = tid; j < NBIN; j += NT) sring[ring(t, 7) * NBIN + j] = spec[j];
          const float* sp = st + a.off_spec + ring(t - 1, 7) * NBIN;
          for (int q = tid; q < 4 * Fi; q += NT) {
            const int f = q >> 2, ri = q & 3;
            win[q] = ri < 2 ? sp[(ri ? 258 : 1) + f] : 0.f;
            win[4 * Fi + q] = ri < 2 ? spec[(ri ? 258 : 1) + f] : 0.f;
          }
        } else {
          const int D = 7 - (i - 1);
          float* ep = st + a.off_enc[i - 1];
          const float* rp = ep + (int64_t)ring(t - 1, D) * Fi * Ci;
          float* er = ep + (int64_t)ring(t, D) * Fi * Ci;  // encoder i-1's frame t (its output Fi x Ci)
          for (int q = tid; q < Fi * Ci; q += NT) {
            win[q] = rp[q];
            win[Fi * Ci + q] = cur[q];
            er[q] = cur[q];
          }
        }
      };
      const Geo g{Fi, Ci, 31 - __builtin_clz(Ci / 4), 2, 0};
      conv_layer(L(win), g, 1, 10 * Ci / 4, 0, Fo, Co, a.enc_w[i], nullptr, a.enc_b[i], nullptr, a.enc_coef[i],
                 a.enc_alpha[i], L(nxt), 1, L(red), L(prm), false, i == 0 ? 32 : i == 4 ? 34 : -1, stage);
      __syncthreads();
      HOP_MARK(2 + i);
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    // cur = encoder 5 output [D4][C6] of frame t
    // ---- complex LSTMs (DCCRN.py:178-199), (h, c) carried across hops
    for (int li = 0; li < 2; ++li) {
      const int K = li == 0 ? D4 * Ch : H;
      float* xin = win;  // [2][K]
      float* hs = st + a.off_h + li * 4 * H;  // [ws][half][H]
      float* cs = st + a.off_c + li * 4 * H;
      // gate q = (ws, half, g), W_hh row n = ws*4H + g
      const bool gate = tid < 4 * G4;
      const int lh = lg2(H), lg4 = lh + 2;  // G4 = 4H
      const int q = gate ? tid : 0, ws = q >> (lg4 + 1), half = (q >> lg4) & 1, gg = q & (G4 - 1), n = ws * G4 + gg;
      // gx[half][n] (n < 8H: both weight sets side by side); staged: the input halves (layer 0
      // x[k = f*Ch + c] = enc5[f][half*Ch + c]; layer 1 the combine output), (h, c) and W_hh
      // (rows padded to H + 4 floats: the gate loop's row-per-lane quad reads are conflict-free)
      gemv(a.lstm_w[li], a.lstm_b[li], L(xin), K, 2, K / 4, 8 * H, L(&gx[0][0]), 8 * 64, L(red), L(zr), [&]() {
        if (li == 0) {  // encoder 5's frame t -> its ring (behind the first weight loads)
          float* er = st + a.off_enc[5] + (int64_t)ring(t, 2) * D4 * C6;
          for (int q2 = tid; q2 < D4 * C6; q2 += NT) er[q2] = cur[q2];
        }
        for (int q2 = tid; q2 < (H / 4) * 2 * G4; q2 += NT) {
          const int j4 = q2 >> (lg4 + 1), r = q2 & (2 * G4 - 1);
          *reinterpret_cast<f32x4*>(&whh[r * (H + 4) + j4 * 4]) = ldg4(a.lstm_whh[li] + (size_t)q2 * 4);
        }
        for (int q2 = tid; q2 < 2 * K; q2 += NT) {
          const int lk = lg2(K), lch = lg2(Ch);
          const int half2 = q2 >> lk, k = q2 & (K - 1);
          xin[q2] = li == 0 ? cur[(k >> lch) * C6 + half2 * Ch + (k & (Ch - 1))] : rin[half2][k];
        }
        for (int q2 = tid; q2 < 4 * H; q2 += NT) {
          (&hv[0][0][0])[(q2 >> lh) * 64 + (q2 & (H - 1))] = hs[q2];
          (&cv[0][0][0])[(q2 >> lh) * 64 + (q2 & (H - 1))] = cs[q2];
        }
      });
      __syncthreads();
      // gates as clskd_lstm_cell: a = gx + W_hh[ws][g] . h[ws][half]
      if (gate) {
        f32x2 s2 = f32x2{gx[half][n], 0.f};
        for (int j4 = 0; j4 < H / 4; ++j4) fma4(s2, ld4(L(&whh[n * (H + 4) + j4 * 4])), ld4(L(&hv[ws][half][j4 * 4])));
        const float s = s2.x + s2.y;
        act[ws][half][gg] = (gg >> lh) == 2 ? fmaf(2.f, sigm(2.f * s), -1.f) : sigm(s);
      }
      __syncthreads();
      for (int q2 = tid; q2 < 4 * H; q2 += NT) {
        const int ws2 = q2 >> (lh + 1), half2 = (q2 >> lh) & 1, u = q2 & (H - 1);
        const float* ac = act[ws2][half2];
        const float cn = ac[H + u] * cv[ws2][half2][u] + ac[u] * ac[2 * H + u];
        const float hn = ac[3 * H + u] * tanh_f(cn);
        cs[q2] = cn;
        hs[q2] = hn;
        hv[ws2][half2][u] = hn;
      }
      __syncthreads();
      // real = R(r) - I(i), imag = R(i) + I(r)  (tools_for_model.py:168-169)
      for (int q2 = tid; q2 < 2 * H; q2 += NT) {
        const int half2 = q2 >> lh, u = q2 & (H - 1);
        rin[half2][u] = half2 == 0 ? hv[0][0][u] - hv[1][1][u] : hv[0][1][u] + hv[1][0][u];
      }
      __syncthreads();
      HOP_MARK(8 + li);
    }
    // projection (NavieComplexLSTM r_trans / i_trans): dec_in[f][half*Ch + c], n = c*D4 + f
    float* pj = &act[0][0][0];  // [2][Ch*D4] (the gate scratch is free now)
    for (int half = 0; half < 2; ++half) {
      gemv(a.proj_w[half], a.proj_b[half], L(rin[half]), 0, 1, H / 4, Ch * D4, L(pj + half * Ch * D4), 0, L(red),
           L(zr), []() {});
      __syncthreads();
    }
    for (int q = tid; q < 2 * Ch * D4; q += NT) {
      const int ld4 = lg2(D4), lcd = lg2(Ch) + ld4;
      const int half = q >> lcd, n = q & ((1 << lcd) - 1);
      decin[(n & (D4 - 1)) * C6 + half * Ch + (n >> ld4)] = pj[q];
    }
    __syncthreads();
    HOP_MARK(10);
  } else {
    // drain hop: no new frame; encoder outputs and the decoder input of frame t are zeros
    stage_x();
    __syncthreads();
    for (int i = tid; i < WIN; i += NT) gxw[i] = xw[i];
    for (int i = 0; i < 6; ++i) {
      const int Fo = 128 >> i, Co = a.enc_cout[i];
      float* er = st + a.off_enc[i] + (int64_t)ring(t, 7 - i) * Fo * Co;
      for (int q = tid; q < Fo * Co; q += NT) er[q] = 0.f;
    }
    for (int q = tid; q < D4 * C6; q += NT) {
      cur[q] = 0.f;
      decin[q] = 0.f;
    }
    __syncthreads();
  }

  // ---- decoder (DCCRN.py:201-206): layer d emits frame t-1-d from its input's frames
  //      [t-1-d, t-d] and encoder 5-d's frames [t-1-d, t-d]; both parities in one pass
  const float* in_cur = decin;  // frame t-d of this layer's input
  for (int d = 0; d < 6; ++d) {
    const int F = D4 << d, Ca = a.dec_ca[d], Cb = a.dec_cb[d], Ci = Ca + Cb, Co = a.dec_co[d];
    const int ie = 5 - d, De = 7 - ie;
    const int out_frame = t - 1 - d;
    const bool dead = a.zero_from >= 0 && out_frame >= a.zero_from;
    const float* in_old = d == 0 ? st + a.off_decin + ring(t - 1, 2) * D4 * C6
                                 : st + a.off_dout[d - 1] + (int64_t)ring(t - 1 - d, 2) * F * Ca;
    const float* sk_old = st + a.off_enc[ie] + (int64_t)ring(t - 1 - d, De) * F * Cb;
    const float* sk_new = d == 0 ? cur : st + a.off_enc[ie] + (int64_t)ring(t - d, De) * F * Cb;
    const bool last = d == 5;
    // _DEC_TAPS (model.py): parity 0 -> dF (1, 0, -1), parity 1 -> dF (1, 0); K order per tap
    // (kt = 0, 1) with window slot 1 - kt
    const Geo g{F, Ci, 31 - __builtin_clz(Ci / 4), 1, 1};
    conv_layer(L(win), g, 2, 6 * Ci / 4, 4 * Ci / 4, F, Co, a.dec_w[d][0], a.dec_w[d][1], a.dec_b[d][0],
               a.dec_b[d][1], last ? nullptr : a.dec_coef[d], last ? nullptr : a.dec_alpha[d], L(nxt), 2, L(red),
               L(prm), dead, d == 1 ? 36 : -1, [&]() {
                 // the previous phase's output -> its ring (behind this layer's first weight loads)
                 if (d == 0) {
                   float* dr = st + a.off_decin + ring(t, 2) * D4 * C6;
                   for (int q = tid; q < D4 * C6; q += NT) dr[q] = decin[q];
                 } else {  // decoder d-1's frame t-d: [2 F_{d-1} = F][Co_{d-1} = Ca]
                   float* orr = st + a.off_dout[d - 1] + (int64_t)ring(t - d, 2) * F * Ca;
                   for (int q = tid; q < F * Ca; q += NT) orr[q] = in_cur[q];
                 }
                 const int lci = g.lgq + 2;
                 for (int q = tid; q < F * Ci; q += NT) {
                   const int f = q >> lci, c = q & (Ci - 1);
                   win[q] = c < Ca ? in_old[f * Ca + c] : sk_old[f * Cb + c - Ca];
                   win[F * Ci + q] = c < Ca ? in_cur[f * Ca + c] : sk_new[f * Cb + c - Ca];
                 }
               });
    __syncthreads();
    in_cur = nxt;
    // ping-pong: the next layer writes the other buffer (cur holds encoder 5 only for d == 0)
    nxt = (nxt == curA) ? curB : curA;
    HOP_MARK(11 + d);
  }
  // in_cur = mask of frame t-6: [256][2] (re, im)
  // ---- mask 'E' (DCCRN.py:207-226) on the spectrum of frame t-6 (staged while the first iSTFT
  //      weight batches load), ConviSTFT row, overlap-add
  const float* s6 = st + a.off_spec + ring(t - 6, 7) * NBIN;
  HOP_MARK(17);
  gemv(a.istft_w, nullptr, L(est), 0, 1, LDEST / 4, WIN, L(frame), 0, L(red), L(zr), [&]() {
    for (int f = tid; f < 257; f += NT) {
      const float re = s6[f], im = s6[257 + f];
      const float mags = sqrtf(re * re + im * im + 1e-8f);
      const float phase = atan2f(im, re);
      float mr = 0.f, mi = 0.f;
      if (f > 0) {
        mr = in_cur[(f - 1) * 2];
        mi = in_cur[(f - 1) * 2 + 1];
      }
      const float mm = sqrtf(mr * mr + mi * mi);
      const float rp = mr / (mm + 1e-8f);
      const float ip = mi / (mm + 1e-8f);
      const float mphase = atan2f(ip, rp);
      const float em = tanhf(mm) * mags;
      const float ep = phase + mphase;
      est[f] = em * cosf(ep);
      est[257 + f] = em * sinf(ep);
    }
    if (tid < 2) est[514 + tid] = 0.f;
  });
  __syncthreads();
  HOP_MARK(18);
  float* fr = st + a.off_frames;
  for (int i = tid; i < WIN; i += NT) fr[ring(t, 4) * WIN + i] = frame[i];
  // output samples of this hop: p = n + 300 over the frames t-3 .. t (k = 0 .. 3)
  for (int n = tid; n < HOP; n += NT) {
    const int p = n + 300;
    float acc = 0.f, coff = 0.f;
    for (int k = 0; k < 4; ++k) {
      const int o = p - k * HOP;
      if (o < 0 || o >= WIN) continue;
      const float v = k == 3 ? frame[o] : fr[ring(t - 3 + k, 4) * WIN + o];
      acc += v;
      const float w = a.window[o];
      coff += w * w;
    }
    float v = acc / (coff + 1e-8f);
    v = fminf(fmaxf(v, -1.f), 1.f);
    a.wav_out[(int64_t)b * HOP + n] = v;
  }
  HOP_MARK(19);
#ifdef CLSKD_EXPERIMENTS
  if (b == 0 && tid == 0) g_hop_marks[39] = clock64();
#endif
}

}  // namespace clskd

using namespace clskd;

extern "C" int clskd_stream_hop(const clskd_stream_hop_args* a, void* stream) {
  CLSKD_CHECK_ARG(a && a->state && a->wav_out && a->stft_w && a->istft_w && a->window,
                  "stream_hop: null argument");
  CLSKD_CHECK_ARG(!a->live || a->x_in, "stream_hop: live hop without input");
  CLSKD_CHECK_SHAPE(a->B >= 1 && a->t >= 0, "stream_hop: B=%d t=%d", a->B, a->t);
  auto pow2 = [](int v) { return v >= 1 && (v & (v - 1)) == 0; };
  CLSKD_CHECK_SHAPE(a->H >= 4 && pow2(a->H) && 16 * a->H <= shop::NT && a->D4 >= 1 &&
                        pow2(a->D4) && a->D4 * a->enc_cout[5] <= 256 && a->enc_cout[5] % 2 == 0,
                    "stream_hop: H=%d D4=%d outside the built LDS budget", a->H, a->D4);
  CLSKD_CHECK_SHAPE(a->enc_cin[0] == 2, "stream_hop: encoder 0 takes (re, im), got %d", a->enc_cin[0]);
  // conv_layer's thread plans: R = 8 rows (4 where Fo == 4), CQ = 2 channels where Co >= 16 (or
  // Fo == 4); the plan's (rows / R) * (Co / CQ) per parity must fit the block.
  auto plan_ok = [&](int Fo, int Co, int Ci, int np) {
    const int R = Fo >= 8 ? 8 : 4, CQ = (Fo < 8 || Co >= 16) ? 2 : 1;
    return pow2(Fo) && Fo >= 4 && (Fo >= 8 || (Co >= 16 && Ci >= 16)) && np * (Fo / R) * (Co / CQ) <= shop::NT &&
           Co % CQ == 0;
  };
  for (int i = 0; i < 6; ++i) {
    const int Fi = 256 >> i, Fo = Fi / 2, Co = a->enc_cout[i], Ci = i == 0 ? 4 : a->enc_cin[i];
    CLSKD_CHECK_SHAPE(pow2(Co) && pow2(Ci) && Ci >= 4 && (i == 0 || Ci == a->enc_cout[i - 1]),
                      "stream_hop: enc %d Ci=%d Co=%d", i, Ci, Co);
    CLSKD_CHECK_SHAPE(2 * Fi * Ci <= shop::WINSZ && Fo * Co <= 1024 && Ci <= 256 && plan_ok(Fo, Co, Ci, 1),
                      "stream_hop: encoder %d too wide for the LDS budget", i);
    CLSKD_CHECK_ARG(a->enc_w[i] && a->enc_b[i] && a->enc_coef[i] && a->enc_alpha[i], "stream_hop: enc %d", i);
  }
  for (int d = 0; d < 6; ++d) {
    const int F = a->D4 << d, Ci = a->dec_ca[d] + a->dec_cb[d], Co = a->dec_co[d];
    CLSKD_CHECK_SHAPE(pow2(Co) && pow2(Ci) && Ci >= 4, "stream_hop: dec %d Ci=%d Co=%d", d, Ci, Co);
    CLSKD_CHECK_SHAPE(2 * F * Ci <= shop::WINSZ && 2 * F * Co <= 1024 && Ci <= 256 && plan_ok(F, Co, Ci, 2),
                      "stream_hop: decoder %d too wide for the LDS budget", d);
    CLSKD_CHECK_ARG(a->dec_w[d][0] && a->dec_w[d][1], "stream_hop: dec %d weights", d);
  }
  CLSKD_CHECK_SHAPE(2 * a->D4 * (a->enc_cout[5] / 2) <= shop::WINSZ && (a->D4 * a->enc_cout[5] / 2) % 4 == 0 &&
                        8 * a->H <= 512 && 2 * 4 * a->H <= 1024,
                    "stream_hop: LSTM too wide for the LDS budget");
  hipLaunchKernelGGL(stream_hop_kernel, dim3((unsigned)a->B), dim3(shop::NT), 0, as_stream(stream), *a);
  CLSKD_LAUNCH_CHECK("stream_hop");
  return CLSKD_OK;
}

extern "C" int clskd_stream_hop_marks(int64_t* out, int32_t n) {
#ifdef CLSKD_EXPERIMENTS
  CLSKD_CHECK_ARG(out && n >= 1 && n <= 40, "stream_hop_marks: bad output");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hop_marks), sizeof(int64_t) * n) != hipSuccess) {
    set_error("stream_hop_marks: copy failed");
    return CLSKD_E_HIP;
  }
  return CLSKD_OK;
#else
  (void)out;
  (void)n;
  set_error("stream_hop_marks: phase marks exist only in a -DCLSKD_EXPERIMENTS build");
  return CLSKD_E_ARG;
#endif
}
