// Microbenchmark (diagnostic): the fp32 halo kernel's inner loop alone — 8 waves (2 per SIMD),
// per tap one A + two B ds_read_b128 issued a tap ahead and 8 v_mfma_f32_32x32x2_f32 on two
// accumulators, one s_barrier per 10 taps — to separate the MFMA/LDS loop from DMA, epilogue
// and tile bookkeeping.  Reports clock64 ticks per MFMA per SIMD.
// hipcc --offload-arch=gfx950 -O3 tools/micro/halo32_loop.hip -o tools/micro/halo32_loop
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int BAR>
__global__ __launch_bounds__(512) void k(float* out, long long* cyc, int chunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  for (int i = tid; i < 128 * 1024 / 16; i += 512) reinterpret_cast<f32x4*>(sm)[i] = f32x4{1.f, 0.5f, 0.25f, 2.f};
  __syncthreads();
  const unsigned char* hb = sm;
  const unsigned char* wl = sm + 48 * 1024;
  f32x16 acc0{}, acc1{};
  const int prow0 = wave * 2 * 33 + l32;
  const long long t0 = clock64();
  for (int c = 0; c < chunks; ++c) {
    if (BAR) __syncthreads();
    f32x4 af[2], bw[2][2];
    auto load = [&](int t, int sl) {
      const int p = prow0 + (t >> 1) * 33 + (t & 1);
      const int kq = t * 8 + (c & 7) + h;
      af[sl] = *reinterpret_cast<const f32x4*>(hb + p * 32 + ((h ^ ((p >> 3) & 1)) << 4));
      bw[sl][0] = *reinterpret_cast<const f32x4*>(wl + (kq * 64 + l32) * 16);
      bw[sl][1] = *reinterpret_cast<const f32x4*>(wl + (kq * 64 + 32 + l32) * 16);
    };
    load(0, 0);
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      if (t + 1 < 10) load(t + 1, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(af[t & 1][j], bw[t & 1][0][j], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(af[t & 1][j], bw[t & 1][1][j], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 512 + tid] = acc0[lane & 15] + acc1[lane & 7];
  if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int BAR>
void run(int grid) {
  float* out;
  long long* cyc;
  hipMalloc(&out, grid * 512 * sizeof(float));
  hipMalloc(&cyc, grid * 8 * sizeof(long long));
  const int chunks = 200;
  hipFuncSetAttribute((const void*)k<BAR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k<BAR>, dim3(grid), dim3(512), 128 * 1024, 0, out, cyc, chunks);
  hipDeviceSynchronize();
  long long h[8];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int w = 0; w < 8; ++w) mx = h[w] > mx ? h[w] : mx;
  printf("barrier %d grid %d: %.1f ticks per MFMA per SIMD\n", BAR, grid, mx / (chunks * 80.0 * 2));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0>(1); run<1>(1); run<0>(256); run<1>(256);
  return 0;
}
