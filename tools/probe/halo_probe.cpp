// Phase timing of the halo kernel (workgroup 0, thread 0, s_memrealtime @ 100 MHz) on the
// ReviewKD 3x3 shape (B=16, F=64, T=643, 64 -> 64 channels).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
__device__ unsigned long long g_trace[64];
#define HALO_TRACE(i)                                                         \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_trace[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#include "../../speech-enhancement-clskd_amd/csrc/conv_halo.hip"
#include "../../speech-enhancement-clskd_amd/csrc/capi.cpp"

int main() {
  const int B = 16, F = 64, T = 643, C = 64, N = 64;
  const int K = 9 * C, Kp = 576;
  __bf16 *x, *w, *out;
  float* bias;
  (void)hipMalloc(&x, (size_t)B * F * T * C * 2);
  (void)hipMalloc(&w, (size_t)N * Kp * 2);
  (void)hipMalloc(&out, (size_t)B * F * T * N * 2);
  (void)hipMalloc(&bias, N * 4);
  (void)hipMemset(x, 0, (size_t)B * F * T * C * 2);
  (void)hipMemset(w, 0, (size_t)N * Kp * 2);
  (void)hipMemset(bias, 0, N * 4);
  clskd_conv_desc d;
  memset(&d, 0, sizeof d);
  d.B = B; d.Fo = F; d.To = T; d.N = N; d.K = Kp; d.stride_f = 1; d.stride_t = 1; d.nseg = 1;
  d.seg[0].ptr = (const float*)x; d.seg[0].sB = (int64_t)F * T * C; d.seg[0].sF = (int64_t)T * C;
  d.seg[0].sT = C; d.seg[0].F = F; d.seg[0].T = T;
  for (int s = 1; s < 4; ++s) d.seg[s] = d.seg[0];
  d.weight = w; d.bias = bias; d.out = out;
  d.oB = (int64_t)F * T * N; d.oF = (int64_t)T * N; d.oT = N; d.oNhi = 0; d.oNlo = 1; d.nlo = 1 << 30;
  d.of_mul = 1; d.of_add = 0; d.compute = CLSKD_BF16; d.in_dtype = CLSKD_BF16; d.out_dtype = CLSKD_BF16;
  d.ntaps = 9; d.ctot = C; d.seg_c[0] = C;
  for (int t = 0; t < 9; ++t) { d.tap_df[t] = t / 3 - 1; d.tap_dt[t] = t % 3 - 1; }
  bool launched = false;
  for (int rep = 0; rep < 3; ++rep) clskd::launch_conv_halo(d, 0, &launched);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  clskd::launch_conv_halo(d, 0, &launched);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long tr[64];
  (void)hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_trace), sizeof tr);
  printf("launched %d, kernel %.1f us; block 0 phases (us since start):\n", (int)launched, ms * 1e3);
  printf("  prologue done %.2f\n", (tr[1] - tr[0]) / 100.0);
  for (int i = 2; i < 14; ++i) if (tr[i]) printf("  tile %d done %.2f\n", i - 2, (tr[i] - tr[0]) / 100.0);
  printf("  end %.2f\n", (tr[40] - tr[0]) / 100.0);
  return 0;
}
