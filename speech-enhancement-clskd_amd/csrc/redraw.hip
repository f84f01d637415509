// Per-step re-draw of the ReviewKD ABF weights (framework.py:194-195: the reference rebuilds its
// ABF modules every step, so conv1/conv2 are kaiming_uniform(a=1) and att_conv carries the
// default Conv2d init).  One launch draws every weight of a ReviewKD module with a counter-based
// Philox4x32-10 generator and writes it twice: into the nn.Module parameter (its own layout) and
// into the packed MFMA operand [N][Kp] (k = tap*Cin + c) in that operand's storage type — the
// ~200 small torch ops of init + pack + cast become one kernel.  The draw counter lives in device
// memory and the last workgroup advances it, so a captured hipGraph re-draws on every replay.
#include "common.h"

namespace clskd {

struct DrawJobsArg {
  clskd_draw_job j[CLSKD_DRAW_MAX_JOBS];
  int32_t first_block[CLSKD_DRAW_MAX_JOBS];
  int32_t n;
};

constexpr int DRAW_THREADS = 256;
constexpr int DRAW_PER_BLOCK = DRAW_THREADS * 4;  // one Philox call -> 4 uniforms per thread

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ __launch_bounds__(DRAW_THREADS) void uniform_redraw_kernel(const DrawJobsArg a,
                                                                      uint64_t seed,
                                                                      unsigned long long* state) {
  int q = 0;
  for (int k = 1; k < a.n; ++k)
    if ((int)blockIdx.x >= a.first_block[k]) q = k;
  const clskd_draw_job& j = a.j[q];
  const unsigned long long draw = __atomic_load_n(&state[0], __ATOMIC_RELAXED);
  const int64_t e0 = ((int64_t)(blockIdx.x - a.first_block[q]) * DRAW_THREADS + threadIdx.x) * 4;
  const uint4 r = philox4x32_10(
      make_uint4((uint32_t)e0, (uint32_t)(e0 >> 32) ^ ((uint32_t)j.stream_id << 16),
                 (uint32_t)draw, (uint32_t)(draw >> 32)),
      make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const uint32_t rv[4] = {r.x, r.y, r.z, r.w};
  const int ctap = j.Cin * j.ntap;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t e = e0 + i;
    if (e >= j.numel) break;
    // 24-bit uniform in [0, 1), then a + (b - a) * u like torch's uniform_
    const float u = (float)(rv[i] >> 8) * (1.0f / 16777216.0f);
    const float v = -j.bound + (2.0f * j.bound) * u;
    j.param[e] = v;
    if (j.packed) {
      const int64_t n = e / ctap;
      const int rem = (int)(e - n * ctap);
      const int c = rem / j.ntap, tap = rem - c * j.ntap;  // param layout [N][Cin][ntap]
      const int64_t o = n * j.Kp + (int64_t)tap * j.Cin + c;
      if (j.packed_dtype == CLSKD_BF16)
        reinterpret_cast<__bf16*>(j.packed)[o] = (__bf16)v;
      else
        reinterpret_cast<float*>(j.packed)[o] = v;
    }
  }
  // The last workgroup to arrive advances the draw counter.  Every block's read of state[0]
  // has returned before its ticket (its stores consumed the value), so no fence is needed —
  // and none is wanted: an agent-scope fence on gfx950 writes back and invalidates the XCD's
  // whole L2 (buffer_wbl2 / buffer_inv sc1), evicting the concurrent streams' working sets.
  // The next launch sees the new counter across the kernel boundary.
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = atomicAdd(&state[1], 1ull);
    if (t == gridDim.x - 1) {
      state[0] = draw + 1;
      state[1] = 0;
    }
  }
}

}  // namespace clskd

using namespace clskd;

extern "C" int clskd_uniform_redraw(const clskd_draw_job* jobs, int32_t njobs, uint64_t seed,
                                    uint64_t* state, void* stream) {
  CLSKD_CHECK_ARG(jobs && state, "uniform_redraw: null pointer");
  CLSKD_CHECK_SHAPE(njobs >= 1 && njobs <= CLSKD_DRAW_MAX_JOBS, "uniform_redraw: %d jobs (1..%d)",
                    njobs, CLSKD_DRAW_MAX_JOBS);
  DrawJobsArg a;
  a.n = njobs;
  int64_t blocks = 0;
  for (int k = 0; k < CLSKD_DRAW_MAX_JOBS; ++k) {
    const clskd_draw_job& j = jobs[k < njobs ? k : 0];
    a.j[k] = j;
    if (k >= njobs) {
      a.first_block[k] = INT32_MAX;
      continue;
    }
    CLSKD_CHECK_ARG(j.param, "uniform_redraw: job %d has a null parameter", k);
    CLSKD_CHECK_SHAPE(j.numel >= 1 && j.Cin >= 1 && j.ntap >= 1 && j.numel % ((int64_t)j.Cin * j.ntap) == 0,
                      "uniform_redraw: job %d shape (numel %lld, Cin %d, ntap %d)", k,
                      (long long)j.numel, j.Cin, j.ntap);
    CLSKD_CHECK_SHAPE(!j.packed || j.Kp >= j.Cin * j.ntap, "uniform_redraw: job %d Kp %d < K", k,
                      j.Kp);
    CLSKD_CHECK_ARG(!j.packed || j.packed_dtype == CLSKD_F32 || j.packed_dtype == CLSKD_BF16,
                    "uniform_redraw: job %d packed dtype", k);
    CLSKD_CHECK_ARG(j.bound >= 0.f, "uniform_redraw: job %d bound", k);
    a.first_block[k] = (int32_t)blocks;
    blocks += (j.numel + DRAW_PER_BLOCK - 1) / DRAW_PER_BLOCK;
  }
  CLSKD_CHECK_SHAPE(blocks < INT32_MAX, "uniform_redraw: too many elements");
  hipLaunchKernelGGL(uniform_redraw_kernel, dim3((unsigned)blocks), dim3(DRAW_THREADS), 0,
                     as_stream(stream), a, seed, reinterpret_cast<unsigned long long*>(state));
  CLSKD_LAUNCH_CHECK("uniform_redraw");
  return CLSKD_OK;
}
