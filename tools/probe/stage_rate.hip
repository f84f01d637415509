// Probe: operand-staging throughput into LDS on gfx950, L2-resident source (2 MiB buffer).
// Each workgroup streams `tiles` tiles of TILE_KB KiB from the buffer into a 3-stage LDS ring
// with no compute, by (a) LDS-DMA global_load_lds_dwordx4 with counted vmcnt, or (b)
// global_load_dwordx4 into VGPRs + ds_write_b128.  Prints GB/s chip-wide and per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep) : "v"(gsrc), "s"(lds_base) : "memory");
}

template <int NW, int TILE_KB, int MODE>
__global__ __launch_bounds__(NW * 64) void stage_kernel(const uint4* __restrict__ src, size_t n16,
                                                         int tiles, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int PER_WAVE = TILE_KB * 1024 / 1024 / NW;  // 1-KiB wave instructions per wave
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  size_t base = ((size_t)blockIdx.x * 7919) % (n16 - 64 * 1024);
  unsigned acc = 0;
  for (int t = 0; t < tiles; ++t) {
    const int st = t % 3;
    auto addr = [&](int i) -> size_t {
      if (MODE >= 2) {  // gathered: 8 rows x 128 B per wave instruction (the im2col pattern)
        const unsigned row = (unsigned)(t * NW + wave) * 131u + (unsigned)i * 977u + (unsigned)(lane >> 3) * 7919u;
        return ((size_t)(row % (n16 / 8)) * 8 + (lane & 7)) % n16;
      }
      return (base + ((size_t)(t * NW + wave) * PER_WAVE + i) * 64 + lane) % n16;
    };
    if (MODE == 0 || MODE == 2) {
#pragma unroll
      for (int i = 0; i < PER_WAVE; ++i) {
        const size_t e = addr(i);
        glds16((const void*)(uint64_t)(uintptr_t)(src + e), lds0 + st * TILE_KB * 1024 + (wave * PER_WAVE + i) * 1024);
      }
      if (t >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_WAVE) : "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      uint4 v[PER_WAVE];
#pragma unroll
      for (int i = 0; i < PER_WAVE; ++i) {
        const size_t e = addr(i);
        v[i] = src[e];
      }
#pragma unroll
      for (int i = 0; i < PER_WAVE; ++i)
        *reinterpret_cast<uint4*>(smem + st * TILE_KB * 1024 + (wave * PER_WAVE + i) * 1024 + lane * 16) = v[i];
      __syncthreads();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  acc += reinterpret_cast<unsigned*>(smem)[threadIdx.x];
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int NW, int TILE_KB, int MODE>
static void run(const uint4* src, size_t n16, unsigned* sink, int blocks, int tiles) {
  auto k = stage_kernel<NW, TILE_KB, MODE>;
  const size_t lds = 3 * TILE_KB * 1024;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(NW * 64), lds, 0, src, n16, tiles, sink);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(NW * 64), lds, 0, src, n16, tiles, sink);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double bytes = 5.0 * blocks * (double)tiles * TILE_KB * 1024;
  printf("mode %-10s waves %2d tile %2d KiB blocks %4d: %7.2f TB/s chip, %6.1f GB/s per CU\n",
         MODE == 0 ? "DMA-contig" : MODE == 1 ? "vgpr-contig" : MODE == 2 ? "DMA-gather" : "vgpr-gather", NW, TILE_KB, blocks, bytes / (ms * 1e-3) / 1e12,
         bytes / (ms * 1e-3) / 1e9 / 256);
}

int main() {
  const size_t bytes = 2u << 20;
  const size_t n16 = bytes / 16;
  uint4* src;
  unsigned* sink;
  (void)hipMalloc(&src, bytes);
  (void)hipMalloc(&sink, 64);
  (void)hipMemset(src, 1, bytes);
  const int tiles = 200;
  run<8, 48, 0>(src, n16, sink, 256, tiles);
  run<8, 48, 1>(src, n16, sink, 256, tiles);
  run<4, 48, 0>(src, n16, sink, 256, tiles);
  run<4, 48, 1>(src, n16, sink, 256, tiles);
  run<16, 48, 0>(src, n16, sink, 256, tiles);
  run<16, 48, 1>(src, n16, sink, 256, tiles);
  run<8, 48, 2>(src, n16, sink, 256, tiles);
  run<8, 48, 3>(src, n16, sink, 256, tiles);
  run<16, 48, 2>(src, n16, sink, 256, tiles);
  run<16, 48, 3>(src, n16, sink, 256, tiles);
  run<8, 16, 0>(src, n16, sink, 512, tiles);
  run<8, 16, 1>(src, n16, sink, 512, tiles);
  run<8, 32, 0>(src, n16, sink, 512, tiles);
  run<8, 32, 1>(src, n16, sink, 512, tiles);
  return 0;
}
