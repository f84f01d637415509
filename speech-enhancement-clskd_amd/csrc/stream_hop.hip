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
// synchronisation at all), and the weights — k-major [K][N] copies of the packed fp32 operands
// the offline forward uses — stream through L1/L2 (926 KB per hop, shared by every stream's
// workgroup).  Per output channel a thread keeps up to MAXR output rows in registers, so each
// weight load feeds R FMAs.  fp32 throughout, BatchNorm in eval mode (running statistics).
//
// Ring slots: frame f of a ring of depth D lives in slot ((f % D) + D) % D; rings start zeroed
// (the causal / centring zeros of the first frames).  Depths: spectrum 7 (mask of frame t-6),
// encoder output i: 7 - i (decoder 5 - i reads frames t-6+i, t-5+i), decoder input 2, decoder
// output d: 2, iSTFT frames 4 (the 400-sample window spans 4 hops).
#include "common.h"

namespace clskd {
namespace shop {

constexpr int NT = 512;    // threads per stream workgroup (8 waves: two per SIMD)
constexpr int MAXR = 4;    // output rows per thread and channel
constexpr int HOP = 100, WIN = 400, NBIN = 514, LDEST = 516;
constexpr int WCH = 8192;  // floats per LDS weight chunk (32 KB; two chunks double-buffered)
constexpr int PER = WCH / 4 / NT;  // float4 loads per thread per chunk

__device__ __forceinline__ int ring(int f, int D) { return ((f % D) + D) % D; }

__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float tanh_f(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * 2.8853900817779268f));
}

// Rows [0, K) of a k-major weight matrix Wt [K][N] (fp32; storage padded to whole float4s)
// stream through LDS in chunks of kc rows (kc * N <= WCH, kc a multiple of 4): chunk c + 1 is
// loaded into registers (PER float4 per thread, all in flight at once) while chunk c is
// consumed from LDS, so a hop pays the L2 latency once per 32 KB instead of once per weight.
// compute(w, k0, kn): w = LDS rows k0 .. k0 + kn - 1 ([kn][N]).  Ends with a barrier.
template <class F>
__device__ void wstream(const float* __restrict__ Wt, int K, int N, float* wbuf, F&& compute) {
  const int tid = threadIdx.x;
  int kc = (WCH / N) & ~3;
  if (kc < 4) kc = 4;
  const int nch = (K + kc - 1) / kc;
  f32x4 r[PER];
  auto gload = [&](int c) {
    const int rows = min(kc, K - c * kc);
    const int n4 = (rows * N + 3) / 4;
    const f32x4* src = reinterpret_cast<const f32x4*>(Wt + (size_t)c * kc * N);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = tid + i * NT;
      r[i] = idx < n4 ? src[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
    f32x4* dst = reinterpret_cast<f32x4*>(wbuf + buf * WCH);
#pragma unroll
    for (int i = 0; i < PER; ++i) dst[tid + i * NT] = r[i];
  };
  gload(0);
  sstore(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) gload(c + 1);
    compute(wbuf + (c & 1) * WCH, c * kc, min(kc, K - c * kc));
    if (c + 1 < nch) sstore((c + 1) & 1);
    __syncthreads();
  }
}

// out[(fo*of_mul + of_add)][co] = act(bias[co] + sum_taps sum_c Wt[(tap*Ci + c)*Co + co] *
// win[slot(tap)][fo*sf + dF(tap)][c]) for fo < Fo; win = LDS [2][F][Ci] (slot 0 = older frame);
// out-of-range input rows read `zrow` (Ci zeros in LDS).  coef: BN [scale | shift] + PReLU.
__device__ void conv_layer(const float* win, int F, int Ci, int ntap, const int* tdf, const int* tsl,
                           int sf, int Fo, int Co, int of_mul, int of_add, const float* __restrict__ Wt,
                           const float* __restrict__ bias, const float* __restrict__ coef,
                           const float* __restrict__ alpha, float* out, const float* zrow, bool zero,
                           float* wbuf) {
  const int tid = threadIdx.x;
  const int co = tid % Co, g = tid / Co, G = NT / Co;
  const int R = (Fo + G - 1) / G;
  const bool act = g < G;
  if (zero) {
    if (act)
      for (int r = 0; r < R; ++r) {
        const int fo = g + G * r;
        if (fo < Fo) out[(fo * of_mul + of_add) * Co + co] = 0.f;
      }
    return;
  }
  const float b0 = (act && bias) ? bias[co] : 0.f;
  float acc[MAXR];
#pragma unroll
  for (int r = 0; r < MAXR; ++r) acc[r] = b0;
  wstream(Wt, ntap * Ci, Co, wbuf, [&](const float* w, int k0, int kn) {
    if (!act) return;
    int j = k0 / Ci, c = k0 - j * Ci;
    const float* rows[MAXR];
    auto set_rows = [&]() {
#pragma unroll
      for (int r = 0; r < MAXR; ++r) {
        const int fo = g + G * r;
        const int fi = fo * sf + tdf[j];
        rows[r] = (r < R && fo < Fo && fi >= 0 && fi < F) ? win + ((size_t)tsl[j] * F + fi) * Ci : zrow;
      }
    };
    set_rows();
    for (int q = 0; q < kn; ++q) {
      const float wv = w[q * Co + co];
#pragma unroll
      for (int r = 0; r < MAXR; ++r)
        if (r < R) acc[r] = fmaf(wv, rows[r][c], acc[r]);
      if (++c == Ci && q + 1 < kn) {
        c = 0;
        ++j;
        set_rows();
      }
    }
  });
  if (!act) return;
  float sc = 1.f, sh = 0.f, al = 0.f;
  if (coef) {
    sc = coef[co];
    sh = coef[Co + co];
    al = alpha[0];
  }
#pragma unroll
  for (int r = 0; r < MAXR; ++r) {
    const int fo = g + G * r;
    if (r < R && fo < Fo) {
      float v = acc[r];
      if (coef) {
        v = fmaf(v, sc, sh);
        v = v >= 0.f ? v : al * v;
      }
      out[(fo * of_mul + of_add) * Co + co] = v;
    }
  }
}

// y[h][n] = bias[n] + sum_k Wt[k*N + n] x[h*xs + k] for n < N, h < nh (x in LDS)
__device__ void gemv(const float* __restrict__ Wt, const float* __restrict__ bias, const float* x,
                     int xs, int nh, int K, int N, float* y, int ys, float* wbuf) {
  const int tid = threadIdx.x;
  constexpr int MO = 4;  // outputs per thread: (h, n) = q, q + NT, ...
  float acc[MO];
  int hh[MO], nn[MO];
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    const int q = tid + i * NT;
    hh[i] = q / N;
    nn[i] = q % N;
    acc[i] = (q < nh * N && bias) ? bias[nn[i]] : 0.f;
  }
  wstream(Wt, K, N, wbuf, [&](const float* w, int k0, int kn) {
    for (int kq = 0; kq < kn; ++kq) {
#pragma unroll
      for (int i = 0; i < MO; ++i)
        if (tid + i * NT < nh * N) acc[i] = fmaf(w[kq * N + nn[i]], x[hh[i] * xs + k0 + kq], acc[i]);
    }
  });
#pragma unroll
  for (int i = 0; i < MO; ++i)
    if (tid + i * NT < nh * N) y[hh[i] * ys + nn[i]] = acc[i];
}

}  // namespace shop

__global__ __launch_bounds__(shop::NT) void stream_hop_kernel(const clskd_stream_hop_args a) {
  using namespace shop;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int t = a.t;
  float* st = a.state + (int64_t)b * a.state_stride;
  const int H = a.H, D4 = a.D4, C6 = a.enc_cout[5], Ch = C6 / 2, G4 = 4 * H;

  __shared__ __attribute__((aligned(16))) float xw[WIN];
  __shared__ float spec[NBIN + 2];
  __shared__ __attribute__((aligned(16))) float win[4096];
  __shared__ float curA[1024], curB[1024];  // ping-pong: current frame of a layer
  __shared__ float decin[256];
  __shared__ float zrow[256];
  __shared__ float gx[2][8 * 64];
  __shared__ float hv[2][2][64], cv[2][2][64], act[2][2][4 * 64], rin[2][64];
  __shared__ float est[LDEST];
  __shared__ float frame[WIN];
  __shared__ __attribute__((aligned(16))) float wbuf[2 * WCH];  // weight chunks (wstream)

  for (int i = tid; i < 256; i += NT) zrow[i] = 0.f;
  // ---- input window: shift by one hop, append the new samples (tools_for_model.py:53-67)
  float* gxw = st + a.off_xwin;
  for (int i = tid; i < WIN; i += NT) xw[i] = i < WIN - HOP ? gxw[i + HOP] : (a.live ? a.x_in[(int64_t)b * HOP + i - (WIN - HOP)] : 0.f);
  __syncthreads();
  for (int i = tid; i < WIN; i += NT) gxw[i] = xw[i];

  float* cur = curA;
  float* nxt = curB;
  if (a.live) {
    // ---- ConvSTFT row of the newest window -> spectrum ring
    gemv(a.stft_w, nullptr, xw, 0, 1, WIN, NBIN, spec, 0, wbuf);
    __syncthreads();
    float* sring = st + a.off_spec;
    for (int i = tid; i < NBIN; i += NT) sring[ring(t, 7) * NBIN + i] = spec[i];
    // ---- encoder (DCCRN.py:171-176): window [t-1, t], taps (kf - 2, kt), stride 2 in F
    int enc_tdf[10], enc_tsl[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      enc_tdf[j] = j / 2 - 2;
      enc_tsl[j] = j % 2;
    }
    for (int i = 0; i < 6; ++i) {
      const int Fi = 256 >> i, Ci = a.enc_cin[i], Fo = Fi / 2, Co = a.enc_cout[i];
      // stage [2][Fi][Ci]: slot 1 = this frame (spectrum / previous layer in LDS), slot 0 = t-1
      if (i == 0) {
        const float* sp = st + a.off_spec + ring(t - 1, 7) * NBIN;
        for (int q = tid; q < 2 * Fi; q += NT) {
          const int f = q >> 1, ri = q & 1;
          win[q] = sp[(ri ? 258 : 1) + f];
          win[2 * Fi + q] = spec[(ri ? 258 : 1) + f];
        }
      } else {
        const int D = 7 - (i - 1);
        const float* rp = st + a.off_enc[i - 1] + (int64_t)ring(t - 1, D) * Fi * Ci;
        for (int q = tid; q < Fi * Ci; q += NT) {
          win[q] = rp[q];
          win[Fi * Ci + q] = cur[q];
        }
      }
      __syncthreads();
      shop::conv_layer(win, Fi, Ci, 10, enc_tdf, enc_tsl, 2, Fo, Co, 1, 0, a.enc_w[i], a.enc_b[i],
                       a.enc_coef[i], a.enc_alpha[i], nxt, zrow, false, wbuf);
      __syncthreads();
      float* er = st + a.off_enc[i] + (int64_t)ring(t, 7 - i) * Fo * Co;
      for (int q = tid; q < Fo * Co; q += NT) er[q] = nxt[q];
      float* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    // cur = encoder 5 output [D4][C6] of frame t
    // ---- complex LSTMs (DCCRN.py:178-199), (h, c) carried across hops
    for (int li = 0; li < 2; ++li) {
      const int K = li == 0 ? D4 * Ch : H;
      // input halves: layer 0 x[k = f*Ch + c] = enc5[f][half*Ch + c]; layer 1 the combine output
      float* xin = win;  // [2][K]
      for (int q = tid; q < 2 * K; q += NT) {
        const int half = q / K, k = q % K;
        xin[q] = li == 0 ? cur[(k / Ch) * C6 + half * Ch + (k % Ch)] : rin[half][k];
      }
      float* hs = st + a.off_h + li * 4 * H;  // [ws][half][H]
      float* cs = st + a.off_c + li * 4 * H;
      for (int q = tid; q < 4 * H; q += NT) {
        (&hv[0][0][0])[(q / H) * 64 + q % H] = hs[q];
        (&cv[0][0][0])[(q / H) * 64 + q % H] = cs[q];
      }
      __syncthreads();
      // gx[half][n] (n < 8H: both weight sets side by side)
      gemv(a.lstm_w[li], a.lstm_b[li], xin, K, 2, K, 8 * H, &gx[0][0], 8 * 64, wbuf);
      // W_hh [2][4H][H] into LDS (one chunk)
      {
        const f32x4* src = reinterpret_cast<const f32x4*>(a.lstm_whh[li]);
        for (int q = tid; q < 2 * G4 * H / 4; q += NT) reinterpret_cast<f32x4*>(wbuf)[q] = src[q];
      }
      __syncthreads();
      // gates (ws, half, g) as clskd_lstm_cell: a = gx + W_hh[ws][g] . h[ws][half]
      for (int q = tid; q < 2 * 2 * G4; q += NT) {
        const int ws = q / (2 * G4), half = (q / G4) % 2, gg = q % G4;
        float s = gx[half][ws * G4 + gg];
        const float* w = wbuf + (ws * G4 + gg) * H;
        for (int j = 0; j < H; ++j) s = fmaf(w[j], hv[ws][half][j], s);
        act[ws][half][gg] = (gg / H) == 2 ? fmaf(2.f, sigm(2.f * s), -1.f) : sigm(s);
      }
      __syncthreads();
      for (int q = tid; q < 4 * H; q += NT) {
        const int ws = q / (2 * H), half = (q / H) % 2, u = q % H;
        const float* ac = act[ws][half];
        const float cn = ac[H + u] * cv[ws][half][u] + ac[u] * ac[2 * H + u];
        const float hn = ac[3 * H + u] * tanh_f(cn);
        cs[q] = cn;
        hs[q] = hn;
        hv[ws][half][u] = hn;
      }
      __syncthreads();
      // real = R(r) - I(i), imag = R(i) + I(r)  (tools_for_model.py:168-169)
      for (int q = tid; q < 2 * H; q += NT) {
        const int half = q / H, u = q % H;
        rin[half][u] = half == 0 ? hv[0][0][u] - hv[1][1][u] : hv[0][1][u] + hv[1][0][u];
      }
      __syncthreads();
    }
    // projection (NavieComplexLSTM r_trans / i_trans): dec_in[f][half*Ch + c], n = c*D4 + f
    float* pj = &act[0][0][0];  // [2][Ch*D4] (the gate scratch is free now)
    for (int half = 0; half < 2; ++half)
      gemv(a.proj_w[half], a.proj_b[half], rin[half], 0, 1, H, Ch * D4, pj + half * Ch * D4, 0, wbuf);
    __syncthreads();
    for (int q = tid; q < 2 * Ch * D4; q += NT) {
      const int half = q / (Ch * D4), n = q % (Ch * D4);
      decin[(n % D4) * C6 + half * Ch + n / D4] = pj[q];
    }
    __syncthreads();
  } else {
    // drain hop: no new frame; encoder outputs and the decoder input of frame t are zeros
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
  float* dr = st + a.off_decin + ring(t, 2) * D4 * C6;
  for (int q = tid; q < D4 * C6; q += NT) dr[q] = decin[q];

  // ---- decoder (DCCRN.py:201-206): layer d emits frame t-1-d from its input's frames
  //      [t-1-d, t-d] and encoder 5-d's frames [t-1-d, t-d]
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
    for (int q = tid; q < F * Ci; q += NT) {
      const int f = q / Ci, c = q % Ci;
      win[q] = c < Ca ? in_old[f * Ca + c] : sk_old[f * Cb + c - Ca];
      win[F * Ci + q] = c < Ca ? in_cur[f * Ca + c] : sk_new[f * Cb + c - Ca];
    }
    __syncthreads();
    const bool last = d == 5;
    for (int p = 0; p < 2; ++p) {
      // _DEC_TAPS (model.py): parity 0 -> dF (1, 0, -1), parity 1 -> dF (1, 0); K order per tap
      // (kt = 0, 1) with window slot 1 - kt
      const int nt = p == 0 ? 6 : 4;
      int tdf[6], tsl[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {  // parity p: dF = 1 - j/2 for j < 6 (p = 0) / 4 (p = 1)
        tdf[j] = 1 - j / 2;
        tsl[j] = 1 - (j % 2);
      }
      shop::conv_layer(win, F, Ci, nt, tdf, tsl, 1, F, Co, 2, p, a.dec_w[d][p], a.dec_b[d][p],
                       last ? nullptr : a.dec_coef[d], last ? nullptr : a.dec_alpha[d], nxt, zrow, dead,
                       wbuf);
    }
    __syncthreads();
    if (!last) {
      float* orr = st + a.off_dout[d] + (int64_t)ring(out_frame, 2) * 2 * F * Co;
      for (int q = tid; q < 2 * F * Co; q += NT) orr[q] = nxt[q];
    }
    in_cur = nxt;
    // ping-pong: the next layer writes the other buffer (cur holds encoder 5 only for d == 0)
    nxt = (nxt == curA) ? curB : curA;
    __syncthreads();
  }
  // in_cur = mask of frame t-6: [256][2] (re, im)
  // ---- mask 'E' (DCCRN.py:207-226) on the spectrum of frame t-6, ConviSTFT row, overlap-add
  const float* s6 = st + a.off_spec + ring(t - 6, 7) * NBIN;
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
  __syncthreads();
  gemv(a.istft_w, nullptr, est, 0, 1, LDEST, WIN, frame, 0, wbuf);
  __syncthreads();
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
}

}  // namespace clskd

using namespace clskd;

extern "C" int clskd_stream_hop(const clskd_stream_hop_args* a, void* stream) {
  CLSKD_CHECK_ARG(a && a->state && a->wav_out && a->stft_w && a->istft_w && a->window,
                  "stream_hop: null argument");
  CLSKD_CHECK_ARG(!a->live || a->x_in, "stream_hop: live hop without input");
  CLSKD_CHECK_SHAPE(a->B >= 1 && a->t >= 0, "stream_hop: B=%d t=%d", a->B, a->t);
  CLSKD_CHECK_SHAPE(a->H >= 1 && a->H <= 64 && a->D4 >= 1 && a->D4 * a->enc_cout[5] <= 256,
                    "stream_hop: H=%d D4=%d outside the built LDS budget", a->H, a->D4);
  for (int i = 0; i < 6; ++i) {
    const int Fi = 256 >> i, Co = a->enc_cout[i], Ci = a->enc_cin[i];
    CLSKD_CHECK_SHAPE(Co >= 1 && Co <= shop::NT && (shop::NT % Co) == 0, "stream_hop: enc %d Co=%d", i, Co);
    CLSKD_CHECK_SHAPE(2 * Fi * Ci <= 4096 && (Fi / 2) * Co <= 1024 && Ci <= 256,
                      "stream_hop: encoder %d too wide for the LDS budget", i);
    CLSKD_CHECK_SHAPE((Fi / 2 + shop::NT / Co - 1) / (shop::NT / Co) <= shop::MAXR, "stream_hop: enc %d rows", i);
    CLSKD_CHECK_ARG(a->enc_w[i] && a->enc_b[i] && a->enc_coef[i] && a->enc_alpha[i], "stream_hop: enc %d", i);
  }
  for (int d = 0; d < 6; ++d) {
    const int F = a->D4 << d, Ci = a->dec_ca[d] + a->dec_cb[d], Co = a->dec_co[d];
    CLSKD_CHECK_SHAPE(Co >= 1 && Co <= shop::NT && (shop::NT % Co) == 0, "stream_hop: dec %d Co=%d", d, Co);
    CLSKD_CHECK_SHAPE(2 * F * Ci <= 4096 && 2 * F * Co <= 1024 && Ci <= 256,
                      "stream_hop: decoder %d too wide for the LDS budget", d);
    CLSKD_CHECK_SHAPE((F + shop::NT / Co - 1) / (shop::NT / Co) <= shop::MAXR, "stream_hop: dec %d rows", d);
    CLSKD_CHECK_ARG(a->dec_w[d][0] && a->dec_w[d][1], "stream_hop: dec %d weights", d);
  }
  CLSKD_CHECK_SHAPE(2 * a->D4 * (a->enc_cout[5] / 2) <= 4096 && 8 * a->H * 2 <= 1024 &&
                        2 * 4 * a->H * a->H <= shop::WCH && 2 * 4 * a->H <= shop::MAXR * shop::NT * 4,
                    "stream_hop: LSTM too wide for the LDS budget");
  CLSKD_CHECK_SHAPE(514 <= 4 * shop::NT && 2 * 8 * a->H <= 4 * shop::NT, "stream_hop: gemv outputs");
  hipLaunchKernelGGL(stream_hop_kernel, dim3((unsigned)a->B), dim3(shop::NT), 0, as_stream(stream), *a);
  CLSKD_LAUNCH_CHECK("stream_hop");
  return CLSKD_OK;
}
