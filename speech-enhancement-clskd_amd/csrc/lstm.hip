// Complex-LSTM recurrence (tools_for_model.py:138-174; nn.LSTM gate order i, f, g, o).
//
// The input projections x@W_ih^T (+ b_ih + b_hh) are hoisted into one implicit GEMM per layer
// (conv engine); this kernel runs only the serial part.  One workgroup owns one (weight set,
// sequence) pair for the whole sequence: W_hh lives in VGPRs (4H*H / threads floats per thread,
// 64 for the teacher's H=128), h in LDS, c in the registers of the H cell-update threads.  The
// batch axis is independent, so workgroups never communicate — 2*2B workgroups run concurrently
// (real_lstm/imag_lstm x real/imag inputs x batch).  fp32 throughout; accurate expf/tanhf.
#include "common.h"

namespace clskd {

template <int H>
__global__ __launch_bounds__(8 * H) void lstm_recurrent_kernel(
    const float* __restrict__ gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
    const float* __restrict__ whh, int T, float* __restrict__ out, int64_t o_ws, int64_t o_seq,
    int64_t o_t) {
  constexpr int G = 4 * H;     // gate rows
  constexpr int KS = 2;        // threads per gate row
  constexpr int HK = H / KS;   // weights per thread
  const int tid = threadIdx.x;
  const int g = tid >> 1;
  const int ks = tid & 1;
  const int ws = blockIdx.y;
  const int seq = blockIdx.x;
  __shared__ __attribute__((aligned(16))) float h_s[H];
  __shared__ float pre[G];

  float w[HK];
  const float* wrow = whh + ((int64_t)ws * G + g) * H + ks * HK;
#pragma unroll
  for (int c = 0; c < HK; c += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(wrow + c);
    w[c] = v[0];
    w[c + 1] = v[1];
    w[c + 2] = v[2];
    w[c + 3] = v[3];
  }
  if (tid < H) h_s[tid] = 0.f;
  float cstate = 0.f;
  const float* gp = gx + ws * gx_ws + seq * gx_seq + g;
  float* op = out + ws * o_ws + seq * o_seq;
  float gnext = (ks == 0) ? gp[0] : 0.f;
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const float gcur = gnext;
    if (ks == 0 && t + 1 < T) gnext = gp[(int64_t)(t + 1) * gx_t];
    // four independent FMA chains (latency), summed in a fixed order
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const float* hp = h_s + ks * HK;
#pragma unroll
    for (int c = 0; c < HK; c += 4) {
      const f32x4 hv = *reinterpret_cast<const f32x4*>(hp + c);
      a0 = fmaf(w[c], hv[0], a0);
      a1 = fmaf(w[c + 1], hv[1], a1);
      a2 = fmaf(w[c + 2], hv[2], a2);
      a3 = fmaf(w[c + 3], hv[3], a3);
    }
    float acc = (a0 + a1) + (a2 + a3);
    acc += __shfl_xor(acc, 1, 64);
    if (ks == 0) pre[g] = gcur + acc;
    __syncthreads();
    if (tid < H) {
      const float ig = sigmoidf_(pre[tid]);
      const float fg = sigmoidf_(pre[H + tid]);
      const float gg = tanhf(pre[2 * H + tid]);
      const float og = sigmoidf_(pre[3 * H + tid]);
      cstate = fg * cstate + ig * gg;
      const float hv = og * tanhf(cstate);
      h_s[tid] = hv;
      op[(int64_t)t * o_t + tid] = hv;
    }
    __syncthreads();
  }
}

}  // namespace clskd

using namespace clskd;

extern "C" int clskd_lstm_recurrent(const float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
                                    const float* whh, int32_t nws, int32_t nseq, int32_t T,
                                    int32_t H, float* out, int64_t o_ws, int64_t o_seq,
                                    int64_t o_t, void* stream) {
  CLSKD_CHECK_ARG(gx && whh && out, "lstm: null pointer");
  CLSKD_CHECK_SHAPE(nws >= 1 && nseq >= 1 && T >= 1, "lstm: empty shape");
  CLSKD_CHECK_ARG(((uintptr_t)whh & 15) == 0, "lstm: whh must be 16-byte aligned");
  dim3 grid(nseq, nws);
  hipStream_t st = as_stream(stream);
  switch (H) {
    case 16:
      hipLaunchKernelGGL(lstm_recurrent_kernel<16>, grid, dim3(128), 0, st, gx, gx_ws, gx_seq, gx_t, whh,
                         T, out, o_ws, o_seq, o_t);
      break;
    case 32:
      hipLaunchKernelGGL(lstm_recurrent_kernel<32>, grid, dim3(256), 0, st, gx, gx_ws, gx_seq, gx_t, whh,
                         T, out, o_ws, o_seq, o_t);
      break;
    case 64:
      hipLaunchKernelGGL(lstm_recurrent_kernel<64>, grid, dim3(512), 0, st, gx, gx_ws, gx_seq, gx_t, whh,
                         T, out, o_ws, o_seq, o_t);
      break;
    case 128:
      hipLaunchKernelGGL(lstm_recurrent_kernel<128>, grid, dim3(1024), 0, st, gx, gx_ws, gx_seq, gx_t,
                         whh, T, out, o_ws, o_seq, o_t);
      break;
    default:
      set_error("lstm: hidden size %d not built (16, 32, 64, 128)", H);
      return CLSKD_E_SHAPE;
  }
  CLSKD_LAUNCH_CHECK("lstm_recurrent");
  return CLSKD_OK;
}
