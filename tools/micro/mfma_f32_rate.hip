// Microbenchmark (diagnostic): issue rate of v_mfma_f32_32x32x2_f32 on one SIMD with 1 or 2
// waves, 1/2/4 accumulator chains, with and without an LDS fragment read per 8 MFMAs.
// hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f32_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CH, int LDS>
__global__ void k(float* out, long long* cyc, int iters) {
  __shared__ f32x4 sh[1024];
  const int lane = threadIdx.x & 63;
  sh[threadIdx.x % 1024] = f32x4{1.f, 2.f, 3.f, 4.f};
  __syncthreads();
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x16{};
  f32x4 a = sh[lane], b = sh[lane + 64];
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    f32x4 a2 = a, b2 = b;
    if (LDS) {
      a2 = sh[(lane + i) & 1023];
      b2 = sh[(lane + 64 + i) & 1023];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j % CH] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j & 3], b[j & 3], acc[j % CH], 0, 0, 0);
    a = a2;
    b = b2;
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int c = 0; c < CH; ++c) s += acc[c][lane & 15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int CH, int LDS>
void run(int waves_per_simd) {
  float* out;
  long long* cyc;
  const int threads = 256 * waves_per_simd;
  hipMalloc(&out, 4096 * sizeof(float) * 4);
  hipMalloc(&cyc, 16 * 16 * sizeof(long long));
  const int iters = 2000;
  hipLaunchKernelGGL((k<CH, LDS>), dim3(1), dim3(threads), 0, 0, out, cyc, iters);
  hipLaunchKernelGGL((k<CH, LDS>), dim3(1), dim3(threads), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long h[16];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int w = 0; w < threads / 64; ++w) mx = h[w] > mx ? h[w] : mx;
  printf("chains %d lds %d waves/SIMD %d: %.1f clock64 ticks per MFMA per SIMD (max over waves)\n",
         CH, LDS, waves_per_simd, mx / (iters * 8.0 * waves_per_simd));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<1, 0>(1); run<2, 0>(1); run<4, 0>(1);
  run<1, 0>(2); run<2, 0>(2); run<4, 0>(2);
  run<2, 1>(1); run<4, 1>(1); run<2, 1>(2); run<4, 1>(2);
  return 0;
}
