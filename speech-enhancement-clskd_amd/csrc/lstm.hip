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

// Thread layout (NKS*H threads): thread = (hidden unit u = tid / NKS, k-slice ks = tid % NKS).
// The thread keeps the four gate rows (i, f, g, o) of unit u restricted to its slice
// k in [ks*KW, (ks+1)*KW), KW = H/NKS, in VGPRs and reads that slice of h from LDS; the NKS
// slices of a unit are adjacent lanes, reduced with log2(NKS) DPP adds.  Few, fat threads: the
// per-step VALU work besides the FMAs (reductions, gate selects, activations) is paid once per
// thread, so NKS = 2 (H = 128: 4 waves, one per SIMD, 256 weights per lane) issues ~2x fewer
// instructions per SIMD per step than an 8-slice layout.  Gates: NKS >= 4 -> lane ks < 4 applies
// gate ks; NKS = 2 -> lane 0 applies i and g, lane 1 f and o.  Lane 0 of the group updates the
// cell.  h goes to an LDS history ring, flushed to `out` every CH steps with coalesced
// workgroup stores; the step barrier waits for LDS only.  The projected inputs are prefetched
// two steps ahead (named registers, loop unrolled by two).  Packed FMAs (v_pk_fma_f32).
template <int H, int NKS, int DBG = 0>
__global__ __launch_bounds__(NKS * H) void lstm_recurrent_kernel(
    const float* __restrict__ gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
    const float* __restrict__ whh, int T, float* __restrict__ out, int64_t o_ws, int64_t o_seq,
    int64_t o_t, int prio) {
  // the serial chain shares its CU with the concurrent streams' GEMMs: issue priority keeps its
  // per-step latency close to the isolated one (CLSKD_LSTM_PRIO)
  if (prio) __builtin_amdgcn_s_setprio(3);
  constexpr int G = 4 * H;     // gate rows
  constexpr int KW = H / NKS;  // k-slice width
  constexpr int NT = NKS * H;  // threads
  static_assert(NKS == 2 || NKS == 4 || NKS == 8, "k-slices");
  static_assert(KW % 4 == 0, "k-slice of whole float4s");
  const int tid = threadIdx.x;
  const int u = tid / NKS;
  const int ks = tid % NKS;
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
  // this lane's gates: NKS >= 4 -> gate ks & 3 (lanes >= 4 duplicate); NKS = 2 -> gates ks, ks+2
  const int ga = NKS >= 4 ? (ks & 3) : ks;
  const float* gp = gx + ws * gx_ws + seq * gx_seq + u;
  float* op = out + ws * o_ws + seq * o_seq;
  auto load_g = [&](int t, float& g0, float& g1) {
    const float* q = gp + (int64_t)min(t, T - 1) * gx_t;
    g0 = DBG == 1 ? 0.1f : q[ga * H];
    if constexpr (NKS == 2) g1 = DBG == 1 ? 0.1f : q[(ga + 2) * H];
  };
  float ga0 = 0.f, ga1 = 0.f, gb0 = 0.f, gb1 = 0.f;
  load_g(0, ga0, ga1);
  load_g(1, gb0, gb1);
  __syncthreads();

  auto step = [&](int t, float g0, float g1) {
    const float* hp = hist[(t + 2 * CH - 1) % (2 * CH)] + ks * KW;
    f32x4 hv[KW / 4];
#pragma unroll
    for (int j = 0; j < KW / 4; ++j) hv[j] = reinterpret_cast<const f32x4*>(hp)[j];
    // every h read issued before the first FMA: the compiler split the 8 reads of H = 128 into
    // three dependent groups (one register quad reused); the memory clobber keeps all reads
    // above the pins, and the pins make each value live at once (FMAs start as they arrive)
#pragma unroll
    for (int j = 0; j < KW / 4; ++j) asm volatile("" : "+v"(hv[j]) : : "memory");
    f32x2l acc[4][2] = {};
#pragma unroll
    for (int j = 0; j < KW / 4; ++j) {
      const f32x2l h01 = {hv[j][0], hv[j][1]}, h23 = {hv[j][2], hv[j][3]};
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) {
        acc[gt][j & 1] = __builtin_elementwise_fma(w[gt][2 * j], h01, acc[gt][j & 1]);
        acc[gt][j & 1] = __builtin_elementwise_fma(w[gt][2 * j + 1], h23, acc[gt][j & 1]);
      }
    }
    float pre[4];
#pragma unroll
    for (int gt = 0; gt < 4; ++gt) {  // NKS-lane group sum
      const f32x2l a2 = acc[gt][0] + acc[gt][1];
      float v = a2[0] + a2[1];
      v += dpp<DPP_XOR1>(v);
      if constexpr (NKS >= 4) v += dpp<DPP_XOR2>(v);
      if constexpr (NKS == 8) v += dpp<DPP_HALF_MIRROR>(v);
      pre[gt] = v;
    }
    float ig, fg, gg, og;
    if constexpr (NKS >= 4) {
      // lane ks (< 4): activation of gate ks (i, f, g, o = sig, sig, tanh, sig), branch-free
      const float p01 = (ga & 1) ? pre[1] : pre[0];
      const float p23 = (ga & 1) ? pre[3] : pre[2];
      const float pg = ((ga & 2) ? p23 : p01) + g0;
      const float k = ga == 2 ? 2.f : 1.f;
      const float act = fmaf(k, sigm_fast(k * pg), ga == 2 ? -1.f : 0.f);
      ig = act;
      fg = dpp<DPP_BCAST1>(act);
      gg = dpp<DPP_BCAST2>(act);
      og = dpp<DPP_BCAST3>(act);
    } else {
      // lane 0: i (sig) and g (tanh); lane 1: f (sig) and o (sig)
      const float pa = (ks ? pre[1] : pre[0]) + g0;
      const float pb = (ks ? pre[3] : pre[2]) + g1;
      const float a0 = sigm_fast(pa);
      const float kb = ks ? 1.f : 2.f;
      const float a1 = fmaf(kb, sigm_fast(kb * pb), ks ? 0.f : -1.f);
      ig = a0;
      gg = a1;
      fg = dpp<DPP_BCAST1>(a0);  // quad_perm [1,1,1,1]: lane 0 of the pair reads lane 1
      og = dpp<DPP_BCAST1>(a1);
      if constexpr (true) {      // pairs (2,3) of a quad take lane 3
        const float fg3 = dpp<DPP_BCAST3>(a0), og3 = dpp<DPP_BCAST3>(a1);
        const bool hi = (tid & 2) != 0;
        fg = hi ? fg3 : fg;
        og = hi ? og3 : og;
      }
    }
    if (ks == 0) {
      cstate = fg * cstate + ig * gg;
      hist[t % (2 * CH)][u] = og * tanh_fast(cstate);
    }
    // Only LDS is exchanged between waves: wait for LDS alone (__syncthreads() would also be
    // a release fence draining vmcnt, i.e. the prefetched gx loads, on every step).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if ((t + 1) % CH == 0 || t == T - 1) {  // uniform: flush steps t0 .. t
      const int tf0 = t - (t % CH);
      const int n = (t - tf0 + 1) * H;
      for (int k = tid; k < n; k += NT) {
        const int r = tf0 + k / H, c = k % H;
        op[(int64_t)r * o_t + c] = hist[r % (2 * CH)][c];
      }
    }
  };

  for (int t = 0; t < T; t += 2) {
    step(t, ga0, ga1);
    load_g(t + 2, ga0, ga1);
    if (t + 1 < T) step(t + 1, gb0, gb1);
    load_g(t + 3, gb0, gb1);
  }
}


// Single-wave recurrence for small H (H * S = 64 lanes: S = 64 / H k-slices per unit; H = 32:
// S = 2, H = 16: S = 4).  The student's H = 32 layers sit on the step's critical chain, where
// the 8-wave layout above pays an s_barrier and a cross-wave LDS round trip every step: here
// one wave holds the whole recurrence, h is exchanged through a double-buffered LDS row that
// the same wave writes and then reads (LDS operations of one wave complete in order: no
// barrier), the S slices of a unit reduce with log2(S) DPP adds, lane s < 4 of a unit applies
// gate(s) as in the k-sliced kernel, lane 0 keeps the cell, and h_t goes straight to `out`
// (one 4*H-byte store per step).  Inputs prefetched two steps ahead.
// pre (optional, may alias gx): the gate pre-activations gx + W_hh h_{t-1} of every step, in
// gx's layout — what the backward's gate derivatives need (clskd_lstm_bwd `pre`); each lane
// stores the pre-activations it formed, at the addresses its gate inputs came from (two steps
// after they were read, so writing over gx in place is safe).
template <int H>
__global__ __launch_bounds__(64) void lstm_wave_kernel(
    const float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
    const float* __restrict__ whh, int T, float* __restrict__ out, int64_t o_ws, int64_t o_seq,
    int64_t o_t, int prio, float* pre, float* __restrict__ cout = nullptr) {
  if (prio) __builtin_amdgcn_s_setprio(3);
  constexpr int S = 64 / H;   // k-slices per unit
  constexpr int KW = H / S;   // k-slice width
  constexpr int G = 4 * H;
  static_assert((S == 2 || S == 4) && KW % 4 == 0, "single-wave layout");
  const int lane = threadIdx.x;
  const int u = lane / S, ks = lane % S;
  const int ws = blockIdx.y, seq = blockIdx.x;
  __shared__ __attribute__((aligned(16))) float hb[2][H];
  f32x2l w[4][KW / 2];
#pragma unroll
  for (int gt = 0; gt < 4; ++gt) {
    const float* wrow = whh + ((int64_t)ws * G + gt * H + u) * H + ks * KW;
#pragma unroll
    for (int j = 0; j < KW; j += 2) w[gt][j / 2] = *reinterpret_cast<const f32x2l*>(wrow + j);
  }
  if (lane < H) hb[1][lane] = 0.f;  // h(-1) = 0
  float cstate = 0.f;
  // this lane's gates: S = 4 -> gate ks; S = 2 -> gates ks, ks + 2
  const float* gp = gx + ws * gx_ws + seq * gx_seq + u;
  float* pp = pre ? pre + ws * gx_ws + seq * gx_seq + u : nullptr;
  float* op = out + ws * o_ws + seq * o_seq + u;
  // taped forward: the cell states c_t too, [ws][seq][T][H] (the backward's cell scan input)
  float* cq = cout ? cout + ((int64_t)ws * gridDim.x + seq) * (int64_t)T * H + u : nullptr;
  auto load_g = [&](int t, float& g0, float& g1) {
    const float* q = gp + (int64_t)min(t, T - 1) * gx_t;
    g0 = q[ks * H];
    if constexpr (S == 2) g1 = q[(ks + 2) * H];
  };
  float ga0 = 0.f, ga1 = 0.f, gb0 = 0.f, gb1 = 0.f;
  load_g(0, ga0, ga1);
  load_g(1, gb0, gb1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  auto step = [&](int t, float g0, float g1) {
    const float* hp = hb[(t + 1) & 1] + ks * KW;  // h(t-1)
    f32x4 hv[KW / 4];
#pragma unroll
    for (int j = 0; j < KW / 4; ++j) hv[j] = reinterpret_cast<const f32x4*>(hp)[j];
    f32x2l acc[4][2] = {};
#pragma unroll
    for (int j = 0; j < KW / 4; ++j) {
      const f32x2l h01 = {hv[j][0], hv[j][1]}, h23 = {hv[j][2], hv[j][3]};
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) {
        acc[gt][j & 1] = __builtin_elementwise_fma(w[gt][2 * j], h01, acc[gt][j & 1]);
        acc[gt][j & 1] = __builtin_elementwise_fma(w[gt][2 * j + 1], h23, acc[gt][j & 1]);
      }
    }
    float pre[4];
#pragma unroll
    for (int gt = 0; gt < 4; ++gt) {
      const f32x2l a2 = acc[gt][0] + acc[gt][1];
      float v = a2[0] + a2[1];
      v += dpp<DPP_XOR1>(v);
      if constexpr (S == 4) v += dpp<DPP_XOR2>(v);
      pre[gt] = v;
    }
    float ig, fg, gg, og;
    if constexpr (S == 4) {
      const float p01 = (ks & 1) ? pre[1] : pre[0];
      const float p23 = (ks & 1) ? pre[3] : pre[2];
      const float pg = ((ks & 2) ? p23 : p01) + g0;
      if (pp) pp[(int64_t)t * gx_t + ks * H] = pg;
      const float k = ks == 2 ? 2.f : 1.f;
      const float act = fmaf(k, sigm_fast(k * pg), ks == 2 ? -1.f : 0.f);
      ig = act;
      fg = dpp<DPP_BCAST1>(act);
      gg = dpp<DPP_BCAST2>(act);
      og = dpp<DPP_BCAST3>(act);
    } else {
      // lane 0: i (sig) and g (tanh); lane 1: f (sig) and o (sig)
      const float pa = (ks ? pre[1] : pre[0]) + g0;
      const float pb = (ks ? pre[3] : pre[2]) + g1;
      if (pp) {
        pp[(int64_t)t * gx_t + ks * H] = pa;
        pp[(int64_t)t * gx_t + (ks + 2) * H] = pb;
      }
      const float a0 = sigm_fast(pa);
      const float kb = ks ? 1.f : 2.f;
      const float a1 = fmaf(kb, sigm_fast(kb * pb), ks ? 0.f : -1.f);
      ig = a0;
      gg = a1;
      // lane 0 of each pair reads lane 1: quad_perm [1,1,3,3]
      fg = dpp<0xF5>(a0);
      og = dpp<0xF5>(a1);
    }
    if (ks == 0) {
      cstate = fg * cstate + ig * gg;
      const float hn = og * tanh_fast(cstate);
      hb[t & 1][u] = hn;
      op[(int64_t)t * o_t] = hn;
      if (cq) cq[(int64_t)t * H] = cstate;
    }
    // one wave: its LDS write completes before its next read is served (in-order LDS queue);
    // the wait + clobber keep the compiler from moving the next step's reads above the write
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  for (int t = 0; t < T; t += 2) {
    step(t, ga0, ga1);
    load_g(t + 2, ga0, ga1);
    if (t + 1 < T) step(t + 1, gb0, gb1);
    load_g(t + 3, gb0, gb1);
  }
}

// ------------------------------------------------------------------------------------------
// Backward of the recurrence (BPTT) for one (weight set, sequence) per workgroup.
// Inputs: pre[ws][seq][t][4H] = the gate PRE-activations of the forward (x W_ih^T + b + h_{t-1}
// W_hh^T — the host rebuilds them with one conv-engine GEMM over the saved h history, so the
// forward kernel stores nothing extra), dh[ws][seq][t][H] = dL/dh_t from the layer's outputs.
// Phase 1 (lanes ks == 0, one unit each): the cell scan c_t = f c_{t-1} + i g into cbuf.
// Phase 2 (t = T-1 .. 0): lane ks == 0 of unit u forms dh = dh_in + (W_hh^T da_{t+1})_u and the
// gate gradients da (i, f, g, o pre-activation) of unit u, writes them to dgates and LDS; after
// one barrier every thread (u, ks) multiplies its slice of W_hh's column u with da and the NKS
// slices reduce by lane shuffles into (W_hh^T da_t)_u for step t-1.  da is double-buffered in
// LDS, so one barrier per step suffices.
// ------------------------------------------------------------------------------------------
template <int H, int NKS>
__global__ __launch_bounds__(NKS * H) void lstm_bwd_kernel(
    const float* __restrict__ pre, int64_t p_ws, int64_t p_seq, int64_t p_t,
    const float* __restrict__ dh, int64_t d_ws, int64_t d_seq, int64_t d_t,
    const float* __restrict__ whh, int T, float* __restrict__ cbuf,
    float* __restrict__ dg, int64_t g_ws, int64_t g_seq, int64_t g_t) {
  constexpr int G = 4 * H;
  constexpr int GW = G / NKS;  // gate rows per k-slice
  const int tid = threadIdx.x;
  const int u = tid / NKS;
  const int ks = tid % NKS;
  const int ws = blockIdx.y;
  const int seq = blockIdx.x;
  static_assert(NKS == 8 && GW % 4 == 0, "lstm_bwd: 8 k-slices of whole float4s");
  __shared__ __attribute__((aligned(16))) float das[2][G];
  // column u of W_hh restricted to gate rows [ks*GW, (ks+1)*GW)
  float wc[GW];
#pragma unroll
  for (int j = 0; j < GW; ++j) wc[j] = whh[((int64_t)ws * G + ks * GW + j) * H + u];
  const float* pp = pre + ws * p_ws + seq * p_seq + u;
  const float* dp = dh + ws * d_ws + seq * d_seq + u;
  float* cp = cbuf + ((int64_t)ws * gridDim.x + seq) * (int64_t)T * H + u;
  float* gp = dg + ws * g_ws + seq * g_seq + u;
  auto acts = [&](int t, float& ig, float& fg, float& gg, float& og) {
    const float* q = pp + (int64_t)t * p_t;
    ig = sigm_fast(q[0]);
    fg = sigm_fast(q[H]);
    gg = fmaf(2.f, sigm_fast(2.f * q[2 * H]), -1.f);
    og = sigm_fast(q[3 * H]);
  };
  if (ks == 0) {
    float c = 0.f;
#pragma unroll 4
    for (int t = 0; t < T; ++t) {
      float ig, fg, gg, og;
      acts(t, ig, fg, gg, og);
      c = fg * c + ig * gg;
      cp[(int64_t)t * H] = c;
    }
  }
  // phase 1 wrote cbuf from lanes ks == 0 and phase 2 reads it from the same lanes: no barrier.
  // Phase 2 keeps every global load off the serial chain: step t-1's operands (gate
  // pre-activations, c_{t-1}, c_{t-2}, dh) are loaded right after step t's gate gradients, so
  // they are in flight during the barrier and the W_hh^T reduction.
  float dc = 0.f, dhr = 0.f;
  float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f, cc = 0.f, cpv = 0.f, dhin = 0.f;
  auto fetch = [&](int t) {
    const float* q = pp + (int64_t)t * p_t;
    q0 = q[0];
    q1 = q[H];
    q2 = q[2 * H];
    q3 = q[3 * H];
    cc = cp[(int64_t)t * H];
    cpv = t > 0 ? cp[(int64_t)(t - 1) * H] : 0.f;
    dhin = dp[(int64_t)t * d_t];
  };
  if (ks == 0) fetch(T - 1);
  for (int t = T - 1; t >= 0; --t) {
    const int buf = t & 1;
    if (ks == 0) {
      const float ig = sigm_fast(q0), fg = sigm_fast(q1);
      const float gg = fmaf(2.f, sigm_fast(2.f * q2), -1.f), og = sigm_fast(q3);
      const float ct = cc, cprev = cpv;
      const float tc = tanh_fast(ct);
      const float dht = dhin + dhr;
      dc = fmaf(dht * og, 1.f - tc * tc, dc);
      const float a_i = dc * gg * ig * (1.f - ig);
      const float a_f = dc * cprev * fg * (1.f - fg);
      const float a_g = dc * ig * (1.f - gg * gg);
      const float a_o = dht * tc * og * (1.f - og);
      dc *= fg;
      das[buf][u] = a_i;
      das[buf][H + u] = a_f;
      das[buf][2 * H + u] = a_g;
      das[buf][3 * H + u] = a_o;
      float* o = gp + (int64_t)t * g_t;
      o[0] = a_i;
      o[H] = a_f;
      o[2 * H] = a_g;
      o[3 * H] = a_o;
      if (t > 0) fetch(t - 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS-only barrier (loads stay in flight)
    __builtin_amdgcn_s_barrier();
    float s0 = 0.f, s1 = 0.f;
    const f32x4* dv = reinterpret_cast<const f32x4*>(&das[buf][ks * GW]);
#pragma unroll
    for (int j = 0; j < GW / 4; ++j) {  // ds_read_b128: 4 LDS reads per 16 gate rows
      const f32x4 v = dv[j];
      s0 = fmaf(wc[4 * j], v[0], s0);
      s1 = fmaf(wc[4 * j + 1], v[1], s1);
      s0 = fmaf(wc[4 * j + 2], v[2], s0);
      s1 = fmaf(wc[4 * j + 3], v[3], s1);
    }
    float s = s0 + s1;
    // NKS = 8 slices of a unit are 8 adjacent lanes: DPP xor1, xor2, half-row mirror
    s += dpp<DPP_XOR1>(s);
    s += dpp<DPP_XOR2>(s);
    s += dpp<DPP_HALF_MIRROR>(s);
    dhr = s;
  }
}

// ------------------------------------------------------------------------------------------
// The same BPTT for H = 16 / 32 in ONE wave per (weight set, sequence): lane (u, ks) of the
// S = 64 / H lanes of unit u.  Every lane of a unit forms the unit's gate gradients (redundant,
// no divergence) and writes its share of them (S = 2: {i, f} / {g, o}; S = 4: one gate) to
// dgates and LDS; after a wave-local LDS wait (no workgroup barrier: one wave, in-order LDS) each
// lane multiplies its G / S gate rows of W_hh's column u with da and the S lanes combine by DPP
// into (W_hh^T da_t)_u.  A step's operands (4 pre-activations, c_t, c_{t-1}, dh_in) are fetched
// four steps ahead into a register ring, so the serial chain waits on no global load.  The
// 4-wave kernel above spent ~820 ns per step (its barrier and the 8-lane reduction); this one is
// bound by the chain's VALU / LDS latency (tools/lstm_micro.py).  PIN (round 6,
// CLSKD_LSTM_BWD_PIN): the lane's GW / 4 gate-gradient reads are issued back to back and waited
// once — the compiler interleaved each ds_read_b128 with the FMAs of the previous one, a chain of
// 16 LDS round trips per step at H = 32.
// ------------------------------------------------------------------------------------------
template <int H, bool PIN>
__global__ __launch_bounds__(64) void lstm_bwd_wave_kernel(
    const float* __restrict__ pre, int64_t p_ws, int64_t p_seq, int64_t p_t,
    const float* __restrict__ dh, int64_t d_ws, int64_t d_seq, int64_t d_t,
    const float* __restrict__ whh, int T, float* __restrict__ cbuf,
    float* __restrict__ dg, int64_t g_ws, int64_t g_seq, int64_t g_t, int c_ready) {
  constexpr int G = 4 * H;
  constexpr int S = 64 / H;  // lanes per unit
  constexpr int GW = G / S;  // gate rows per lane in the W_hh^T reduction
  static_assert((S == 2 || S == 4) && GW % 4 == 0, "lstm_bwd_wave: H = 16 or 32");
  const int lane = threadIdx.x;
  const int u = lane / S, ks = lane % S;
  const int ws = blockIdx.y, seq = blockIdx.x;
  __shared__ __attribute__((aligned(16))) float das[2][G];
  f32x2l wc[GW / 2];  // packed pairs: the reduction runs as v_pk_fma_f32
#pragma unroll
  for (int j = 0; j < GW; ++j) wc[j / 2][j % 2] = whh[((int64_t)ws * G + ks * GW + j) * H + u];
  const float* pp = pre + ws * p_ws + seq * p_seq + u;
  const float* dp = dh + ws * d_ws + seq * d_seq + u;
  float* cp = cbuf + ((int64_t)ws * gridDim.x + seq) * (int64_t)T * H + u;
  float* gp = dg + ws * g_ws + seq * g_seq + u;
  // phase 1: the cell scan, by every lane of the unit (identical values to the same address;
  // each lane reads back only what it wrote itself) — unless the taped forward stored the cell
  // states already (c_ready: lstm_wave_kernel's cout; the serial scan is ~half of this kernel)
  if (!c_ready) {
    float c = 0.f;
#pragma unroll 4
    for (int t = 0; t < T; ++t) {
      const float* q = pp + (int64_t)t * p_t;
      const float ig = sigm_fast(q[0]), fg = sigm_fast(q[H]);
      const float gg = fmaf(2.f, sigm_fast(2.f * q[2 * H]), -1.f);
      c = fg * c + ig * gg;
      cp[(int64_t)t * H] = c;
    }
  }
  struct Op {
    float q0, q1, q2, q3, cc, cpv, dhin;
  };
  auto fetch = [&](int t, Op& o) {
    if (t < 0) return;
    const float* q = pp + (int64_t)t * p_t;
    o.q0 = q[0];
    o.q1 = q[H];
    o.q2 = q[2 * H];
    o.q3 = q[3 * H];
    o.cc = cp[(int64_t)t * H];
    o.cpv = t > 0 ? cp[(int64_t)(t - 1) * H] : 0.f;
    o.dhin = dp[(int64_t)t * d_t];
  };
  float dc = 0.f, dhr = 0.f;
  auto step = [&](int t, const Op& o) {
    const int buf = t & 1;
    const float ig = sigm_fast(o.q0), fg = sigm_fast(o.q1);
    const float gg = fmaf(2.f, sigm_fast(2.f * o.q2), -1.f), og = sigm_fast(o.q3);
    const float tc = tanh_fast(o.cc);
    const float dht = o.dhin + dhr;
    dc = fmaf(dht * og, 1.f - tc * tc, dc);
    const float a_i = dc * gg * ig * (1.f - ig);
    const float a_f = dc * o.cpv * fg * (1.f - fg);
    const float a_g = dc * ig * (1.f - gg * gg);
    const float a_o = dht * tc * og * (1.f - og);
    dc *= fg;
    float* go = gp + (int64_t)t * g_t;
    if constexpr (S == 2) {  // lane 0 of the unit: gates i, f; lane 1: g, o
      const float v0 = ks ? a_g : a_i, v1 = ks ? a_o : a_f;
      das[buf][(2 * ks) * H + u] = v0;
      das[buf][(2 * ks + 1) * H + u] = v1;
      go[(2 * ks) * H] = v0;
      go[(2 * ks + 1) * H] = v1;
    } else {
      const float v = ks == 0 ? a_i : ks == 1 ? a_f : ks == 2 ? a_g : a_o;
      das[buf][ks * H + u] = v;
      go[ks * H] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: da of step t written
    f32x2l a0 = {0.f, 0.f}, a1 = {0.f, 0.f};  // four independent chains, two per packed FMA
    const f32x4* dv = reinterpret_cast<const f32x4*>(&das[buf][ks * GW]);
    if constexpr (PIN) {
      f32x4 v[GW / 4];
#pragma unroll
      for (int j = 0; j < GW / 4; ++j) v[j] = dv[j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read in flight, one wait
#pragma unroll
      for (int j = 0; j < GW / 4; ++j) {
        const f32x2l v01 = {v[j][0], v[j][1]}, v23 = {v[j][2], v[j][3]};
        a0 = wc[2 * j] * v01 + a0;
        a1 = wc[2 * j + 1] * v23 + a1;
      }
    } else {
#pragma unroll
      for (int j = 0; j < GW / 4; ++j) {
        const f32x4 v = dv[j];
        const f32x2l v01 = {v[0], v[1]}, v23 = {v[2], v[3]};
        a0 = wc[2 * j] * v01 + a0;
        a1 = wc[2 * j + 1] * v23 + a1;
      }
    }
    const f32x2l a = a0 + a1;
    float s = a[0] + a[1];
    s += dpp<DPP_XOR1>(s);
    if constexpr (S == 4) s += dpp<DPP_XOR2>(s);
    dhr = s;
  };
  Op o0{}, o1{}, o2{}, o3{};
  fetch(T - 1, o0);
  fetch(T - 2, o1);
  fetch(T - 3, o2);
  fetch(T - 4, o3);
  for (int t = T - 1; t >= 0; t -= 4) {
    step(t, o0);
    fetch(t - 4, o0);
    if (t - 1 < 0) break;
    step(t - 1, o1);
    fetch(t - 5, o1);
    if (t - 2 < 0) break;
    step(t - 2, o2);
    fetch(t - 6, o2);
    if (t - 3 < 0) break;
    step(t - 3, o3);
    fetch(t - 7, o3);
  }
}

// ------------------------------------------------------------------------------------------
// One recurrence step with carried state (streaming inference, config C5): for every (weight
// set, sequence), gates = gx + W_hh h, c = f c + i g, h = o tanh(c), with h and c updated in
// place (h read into LDS before any write).  Same activation functions as the offline
// recurrence, so a stream of steps reproduces lstm_recurrent_kernel's sequence.
// One workgroup per (ws, seq); thread g < 4H forms gate row g.
// ------------------------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(4 * H) void lstm_cell_kernel(const float* __restrict__ gx, int64_t gx_ws,
                                                         int64_t gx_seq, const float* __restrict__ whh,
                                                         float* __restrict__ h, float* __restrict__ c,
                                                         int64_t s_ws, int64_t s_seq,
                                                         float* __restrict__ out, int64_t o_ws,
                                                         int64_t o_seq) {
  constexpr int G = 4 * H;
  const int g = threadIdx.x;
  const int ws = blockIdx.y, seq = blockIdx.x;
  __shared__ float hs[H];
  __shared__ float act[G];
  float* hp = h + ws * s_ws + seq * s_seq;
  float* cp = c + ws * s_ws + seq * s_seq;
  if (g < H) hs[g] = hp[g];
  __syncthreads();
  const float* w = whh + ((int64_t)ws * G + g) * H;
  float a = gx[ws * gx_ws + seq * gx_seq + g];
#pragma unroll 8
  for (int j = 0; j < H; ++j) a = fmaf(w[j], hs[j], a);
  const int gate = g / H;
  act[g] = gate == 2 ? fmaf(2.f, sigm_fast(2.f * a), -1.f) : sigm_fast(a);
  __syncthreads();
  if (g < H) {
    const float cn = act[H + g] * cp[g] + act[g] * act[2 * H + g];
    const float hn = act[3 * H + g] * tanh_fast(cn);
    cp[g] = cn;
    hp[g] = hn;
    out[ws * o_ws + seq * o_seq + g] = hn;
  }
}
}  // namespace clskd

using namespace clskd;

extern "C" int clskd_lstm_pre_capable(int32_t H) {
  return H == 32 && knob(KNOB_LSTM_NKS32) == 1 && knob(KNOB_LSTM_PRE) != 0 ? 1 : 0;
}

extern "C" int clskd_lstm_recurrent(const float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
                                    const float* whh, int32_t nws, int32_t nseq, int32_t T,
                                    int32_t H, float* out, int64_t o_ws, int64_t o_seq,
                                    int64_t o_t, void* stream) {
  CLSKD_CHECK_ARG(gx && whh && out, "lstm: null pointer");
  CLSKD_CHECK_SHAPE(nws >= 1 && nseq >= 1 && T >= 1, "lstm: empty shape");
  CLSKD_CHECK_ARG(((uintptr_t)whh & 15) == 0, "lstm: whh must be 16-byte aligned");
  if (skip_kernel(SKIP_LSTM)) return CLSKD_OK;
  dim3 grid(nseq, nws);
  hipStream_t st = as_stream(stream);
  // k-slices per unit (measured on MI355X, tools/lstm_micro.py): H = 128 -> 4 (662 ns/step vs
  // 772 with 8 — twice the reduction work — and 953 with 2, whose 256 weights per lane spill
  // to AGPRs); H = 32 -> 8 (281 ns/step vs 297 / 312 with 4 / 2: a latency-bound chain, more
  // waves hide more of it).  A/B knobs CLSKD_LSTM_NKS (H=128) and CLSKD_LSTM_NKS32 (H=32).
  const int nks128 = [] {
    const int v = knob(KNOB_LSTM_NKS);
    return (v == 2 || v == 8) ? v : 4;
  }();
  // H = 32: CLSKD_LSTM_NKS32 = 2 | 4 | 8 selects the k-sliced multi-wave kernel, 1 (default)
  // the single-wave kernel (lstm_wave_kernel: 245 ns/step against 281 for the 8-slice kernel)
  const int nks32 = knob(KNOB_LSTM_NKS32);
  const int prio = knob(KNOB_LSTM_PRIO) == 1 ? 1 : 0;
  {
    const int rc = experiment_guard("CLSKD_LSTM32_TDIV", H == 32 ? knob(KNOB_LSTM32_TDIV) : 0);
    if (rc != CLSKD_OK) return rc;
    const int rc2 = experiment_guard("CLSKD_LSTM128_TDIV", H == 128 ? knob(KNOB_LSTM128_TDIV) : 0);
    if (rc2 != CLSKD_OK) return rc2;
  }
#define LSTM_LAUNCH(H_, NKS_) \
  hipLaunchKernelGGL((lstm_recurrent_kernel<H_, NKS_>), grid, dim3(NKS_ * H_), 0, st, gx, gx_ws, \
                     gx_seq, gx_t, whh, T, out, o_ws, o_seq, o_t, prio)
  switch (H) {
    case 16:
      LSTM_LAUNCH(16, 4);
      break;
    case 32:
#ifdef CLSKD_EXPERIMENTS
      if (const int td = knob(KNOB_LSTM32_TDIV)) T = max(1, T / max(1, td));  // timing only
#endif
      if (nks32 == 4) LSTM_LAUNCH(32, 4);
      else if (nks32 == 2) LSTM_LAUNCH(32, 2);
      else if (nks32 == 8) LSTM_LAUNCH(32, 8);
      else hipLaunchKernelGGL(lstm_wave_kernel<32>, grid, dim3(64), 0, st, gx, gx_ws, gx_seq, gx_t,
                              whh, T, out, o_ws, o_seq, o_t, prio, (float*)nullptr);
      break;
    case 64:
      LSTM_LAUNCH(64, 4);
      break;
    case 128:
#ifdef CLSKD_EXPERIMENTS
      // timing experiment only (wrong results): CLSKD_LSTM128_TDIV = d runs T / d steps
      if (const int td = knob(KNOB_LSTM128_TDIV)) T = max(1, T / max(1, td));
#endif
      if (nks128 == 8) LSTM_LAUNCH(128, 8);
      else if (nks128 == 4) LSTM_LAUNCH(128, 4);
      else LSTM_LAUNCH(128, 2);
      break;
    default:
      set_error("lstm: hidden size %d not built (16, 32, 64, 128)", H);
      return CLSKD_E_SHAPE;
  }
#undef LSTM_LAUNCH
  CLSKD_LAUNCH_CHECK("lstm_recurrent");
  return CLSKD_OK;
}

extern "C" int clskd_lstm_recurrent_pre(float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
                                        const float* whh, int32_t nws, int32_t nseq, int32_t T,
                                        int32_t H, float* out, int64_t o_ws, int64_t o_seq,
                                        int64_t o_t, float* cbuf, void* stream) {
  CLSKD_CHECK_ARG(gx && whh && out, "lstm_pre: null pointer");
  CLSKD_CHECK_SHAPE(nws >= 1 && nseq >= 1 && T >= 1, "lstm_pre: empty shape");
  CLSKD_CHECK_ARG(((uintptr_t)whh & 15) == 0, "lstm_pre: whh must be 16-byte aligned");
  CLSKD_CHECK_SHAPE(clskd_lstm_pre_capable(H), "lstm_pre: H=%d runs on a kernel without the "
                    "pre-activation output (clskd_lstm_pre_capable)", H);
  if (skip_kernel(SKIP_LSTM_PRE)) return CLSKD_OK;
  hipLaunchKernelGGL(lstm_wave_kernel<32>, dim3(nseq, nws), dim3(64), 0, as_stream(stream), gx,
                     gx_ws, gx_seq, gx_t, whh, T, out, o_ws, o_seq, o_t,
                     knob(KNOB_LSTM_PRIO) == 1 ? 1 : 0, gx, cbuf);
  CLSKD_LAUNCH_CHECK("lstm_recurrent_pre");
  return CLSKD_OK;
}

extern "C" int clskd_lstm_bwd(const float* pre, int64_t p_ws, int64_t p_seq, int64_t p_t,
                              const float* dh, int64_t d_ws, int64_t d_seq, int64_t d_t,
                              const float* whh, int32_t nws, int32_t nseq, int32_t T, int32_t H,
                              float* cbuf, int32_t c_ready, float* dgates, int64_t g_ws,
                              int64_t g_seq, int64_t g_t, void* stream) {
  CLSKD_CHECK_ARG(pre && dh && whh && cbuf && dgates, "lstm_bwd: null pointer");
  CLSKD_CHECK_SHAPE(nws >= 1 && nseq >= 1 && T >= 1, "lstm_bwd: empty shape");
  if (skip_kernel(SKIP_LSTM_BWD)) return CLSKD_OK;
  dim3 grid(nseq, nws);
  hipStream_t st = as_stream(stream);
#define LSTM_BWD(H_, NKS_)                                                                     \
  hipLaunchKernelGGL((lstm_bwd_kernel<H_, NKS_>), grid, dim3(NKS_ * H_), 0, st, pre, p_ws, p_seq, \
                     p_t, dh, d_ws, d_seq, d_t, whh, T, cbuf, dgates, g_ws, g_seq, g_t)
  // H = 16 / 32: the single-wave kernel unless CLSKD_LSTM_BWD_WAVE=0 (A/B)
  const bool wave = knob(KNOB_LSTM_BWD_WAVE) != 0;
  if (wave && (H == 16 || H == 32)) {
    const bool pin = knob(KNOB_LSTM_BWD_PIN) != 0;
#define LSTM_BWD_WAVE(H_, PIN_)                                                                   \
  hipLaunchKernelGGL((lstm_bwd_wave_kernel<H_, PIN_>), grid, dim3(64), 0, st, pre, p_ws, p_seq,   \
                     p_t, dh, d_ws, d_seq, d_t, whh, T, cbuf, dgates, g_ws, g_seq, g_t, c_ready)
    if (H == 16) {
      if (pin) LSTM_BWD_WAVE(16, true); else LSTM_BWD_WAVE(16, false);
    } else {
      if (pin) LSTM_BWD_WAVE(32, true); else LSTM_BWD_WAVE(32, false);
    }
#undef LSTM_BWD_WAVE
    CLSKD_LAUNCH_CHECK("lstm_bwd");
    return CLSKD_OK;
  }
  switch (H) {
    case 16: LSTM_BWD(16, 8); break;
    case 32: LSTM_BWD(32, 8); break;
    case 64: LSTM_BWD(64, 8); break;
    case 128: LSTM_BWD(128, 8); break;
    default:
      set_error("lstm_bwd: hidden size %d not built (16, 32, 64, 128)", H);
      return CLSKD_E_SHAPE;
  }
#undef LSTM_BWD
  CLSKD_LAUNCH_CHECK("lstm_bwd");
  return CLSKD_OK;
}

extern "C" int clskd_lstm_cell(const float* gx, int64_t gx_ws, int64_t gx_seq, const float* whh,
                               int32_t nws, int32_t nseq, int32_t H, float* h, float* c,
                               int64_t s_ws, int64_t s_seq, float* out, int64_t o_ws, int64_t o_seq,
                               void* stream) {
  CLSKD_CHECK_ARG(gx && whh && h && c && out, "lstm_cell: null pointer");
  CLSKD_CHECK_SHAPE(nws >= 1 && nseq >= 1, "lstm_cell: empty shape");
  dim3 grid(nseq, nws);
  hipStream_t st = as_stream(stream);
  switch (H) {
    case 16: hipLaunchKernelGGL(lstm_cell_kernel<16>, grid, dim3(64), 0, st, gx, gx_ws, gx_seq, whh, h, c, s_ws, s_seq, out, o_ws, o_seq); break;
    case 32: hipLaunchKernelGGL(lstm_cell_kernel<32>, grid, dim3(128), 0, st, gx, gx_ws, gx_seq, whh, h, c, s_ws, s_seq, out, o_ws, o_seq); break;
    case 64: hipLaunchKernelGGL(lstm_cell_kernel<64>, grid, dim3(256), 0, st, gx, gx_ws, gx_seq, whh, h, c, s_ws, s_seq, out, o_ws, o_seq); break;
    case 128: hipLaunchKernelGGL(lstm_cell_kernel<128>, grid, dim3(512), 0, st, gx, gx_ws, gx_seq, whh, h, c, s_ws, s_seq, out, o_ws, o_seq); break;
    default:
      set_error("lstm_cell: hidden size %d not built (16, 32, 64, 128)", H);
      return CLSKD_E_SHAPE;
  }
  CLSKD_LAUNCH_CHECK("lstm_cell");
  return CLSKD_OK;
}
