// Complex-LSTM recurrence (tools_for_model.py:138-174; nn.LSTM gate order i, f, g, o).
//
// The input projections x@W_ih^T (+ b_ih + b_hh) are hoisted into one implicit GEMM per layer
// (conv engine); this kernel runs only the serial part.  One workgroup owns one (weight set,
// sequence) pair for the whole sequence: W_hh lives in VGPRs (4H*H / threads floats per thread,
// 64 for the teacher's H=128), h in LDS (double-buffered), c in the registers of the gate-0
// lanes.  The
// batch axis is independent, so workgroups never communicate — 2*2B workgroups run concurrently
// (real_lstm/imag_lstm x real/imag inputs x batch).  fp32 throughout.
#include <stdlib.h>

#include "common.h"

namespace clskd {

typedef float f32x2l __attribute__((ext_vector_type(2)));

// In-row cross-lane moves on the DPP path (no LDS round trip, unlike __shfl's ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141; // lane i <- lane 7-i within each 8-lane half-row
constexpr int DPP_BCAST1 = 0x55;       // quad_perm [1,1,1,1]
constexpr int DPP_BCAST2 = 0xAA;       // quad_perm [2,2,2,2]
constexpr int DPP_BCAST3 = 0xFF;       // quad_perm [3,3,3,3]

// Gate nonlinearities on v_exp_f32 / v_rcp_f32 (~1 ulp each; the recurrence's fp32 rounding,
// not these, dominates its error against the oracle).
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float tanh_fast(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * 2.8853900817779268f));
}

// Thread layout (8H threads): thread = (hidden unit u = tid / 8, k-slice ks = tid % 8).  The
// thread keeps the four gate rows (i, f, g, o) of unit u restricted to its slice
// k in [ks*H/8, (ks+1)*H/8) in VGPRs, reads only that slice of h from LDS (H/8 floats —
// the LDS read traffic per step is 1/4 of a two-threads-per-row layout, which was LDS-bandwidth
// bound), and the 8 slices of a unit are adjacent lanes: three xor-shuffle adds give every lane
// of the group the four pre-activations.  Lanes 0..3 of the group each apply one gate's
// activation, lane 0 gathers them and updates the cell — no LDS round trip between the matvec
// and the cell.  h goes to an LDS history ring, flushed to `out` every CH steps with coalesced
// workgroup stores; the step barrier waits for LDS only.  Packed FMAs (v_pk_fma_f32).
template <int H, int DBG = 0>
__global__ __launch_bounds__(8 * H) void lstm_recurrent_kernel(
    const float* __restrict__ gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
    const float* __restrict__ whh, int T, float* __restrict__ out, int64_t o_ws, int64_t o_seq,
    int64_t o_t) {
  constexpr int G = 4 * H;   // gate rows
  constexpr int KW = H / 8;  // k-slice width
  static_assert(KW % 2 == 0, "H >= 16");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int u = tid >> 3;
  const int ks = tid & 7;
  const int ws = blockIdx.y;
  const int seq = blockIdx.x;
  constexpr int CH = 32;
  __shared__ __attribute__((aligned(16))) float hist[2 * CH][H];

  // w[gate][j]: W_hh[ws][gate*H + u][ks*KW + j], packed in pairs
  f32x2l w[4][KW / 2];
#pragma unroll
  for (int gt = 0; gt < 4; ++gt) {
    const float* wrow = whh + ((int64_t)ws * G + gt * H + u) * H + ks * KW;
#pragma unroll
    for (int j = 0; j < KW; j += 2) w[gt][j / 2] = *reinterpret_cast<const f32x2l*>(wrow + j);
  }
  if (tid < H) hist[2 * CH - 1][tid] = 0.f;  // h(-1) = 0
  float cstate = 0.f;  // meaningful in lane ks == 0 of each unit group
  // gx of this unit: lane ks < 4 fetches gate ks's projected input
  const float* gp = gx + ws * gx_ws + seq * gx_seq + (ks & 3) * H + u;
  float* op = out + ws * o_ws + seq * o_seq;
  float gnext = DBG == 1 ? 0.1f : gp[0];
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const float gcur = gnext;
    if (DBG != 1 && t + 1 < T) gnext = gp[(int64_t)(t + 1) * gx_t];
    const float* hp = hist[(t + 2 * CH - 1) % (2 * CH)] + ks * KW;
    f32x2l acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
    if constexpr (KW % 4 == 0) {
#pragma unroll
      for (int j = 0; j < KW; j += 4) {
        const f32x4 hv = *reinterpret_cast<const f32x4*>(hp + j);
        const f32x2l h01 = {hv[0], hv[1]}, h23 = {hv[2], hv[3]};
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) {
          acc[gt] = __builtin_elementwise_fma(w[gt][j / 2], h01, acc[gt]);
          acc[gt] = __builtin_elementwise_fma(w[gt][j / 2 + 1], h23, acc[gt]);
        }
      }
    } else {  // H = 16: 2-wide slices
      const f32x2l h01 = *reinterpret_cast<const f32x2l*>(hp);
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) acc[gt] = __builtin_elementwise_fma(w[gt][0], h01, acc[gt]);
    }
    float pre[4];
#pragma unroll
    for (int gt = 0; gt < 4; ++gt) {  // 8-lane group sum: xor 1, xor 2, half-row mirror
      float v = acc[gt][0] + acc[gt][1];
      v += dpp<DPP_XOR1>(v);
      v += dpp<DPP_XOR2>(v);
      v += dpp<DPP_HALF_MIRROR>(v);
      pre[gt] = v;
    }
    // lane ks (< 4) of the group: activation of gate ks (i, f, g, o = sig, sig, tanh, sig)
    const int gsel = ks & 3;
    const float pg = (gsel == 0 ? pre[0] : gsel == 1 ? pre[1] : gsel == 2 ? pre[2] : pre[3]) + gcur;
    const float act = gsel == 2 ? tanh_fast(pg) : sigm_fast(pg);
    const float fg = dpp<DPP_BCAST1>(act);
    const float gg = dpp<DPP_BCAST2>(act);
    const float og = dpp<DPP_BCAST3>(act);
    if (ks == 0) {
      cstate = fg * cstate + act * gg;
      hist[t % (2 * CH)][u] = og * tanh_fast(cstate);
    }
    // Only LDS is exchanged between waves: wait for LDS alone (__syncthreads() would also be
    // a release fence draining vmcnt, i.e. the prefetched gx load, on every step).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if ((t + 1) % CH == 0 || t == T - 1) {  // uniform: flush steps t0 .. t
      const int t0 = t - (t % CH);
      const int n = (t - t0 + 1) * H;
      for (int i = tid; i < n; i += 8 * H) {
        const int r = t0 + i / H, c = i % H;
        op[(int64_t)r * o_t + c] = hist[r % (2 * CH)][c];
      }
    }
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
      if (getenv("CLSKD_LSTM_DEBUG") && getenv("CLSKD_LSTM_DEBUG")[0] == '1')  // timing experiment
        hipLaunchKernelGGL((lstm_recurrent_kernel<128, 1>), grid, dim3(1024), 0, st, gx, gx_ws, gx_seq,
                           gx_t, whh, T, out, o_ws, o_seq, o_t);
      else
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
