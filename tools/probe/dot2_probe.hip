// Probe: semantics of __builtin_amdgcn_fdot2_f32_bf16 (v_dot2c_f32_bf16) on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
__global__ void k(const uint32_t* a, const uint32_t* w, float* out) {
  const int i = threadIdx.x;
  float acc = 0.5f;
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[i]),
                                        __builtin_bit_cast(bf16x2, ((cu32p)w)[0]), acc, false);
  out[i] = acc;
  out[64 + i] = (float)__builtin_bit_cast(bf16x2, a[i])[0];
  out[128 + i] = (float)__builtin_bit_cast(bf16x2, a[i])[1];
}
static uint16_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
int main() {
  uint32_t ha[64], hw[1];
  for (int i = 0; i < 64; ++i) ha[i] = bf(1.0f + i) | ((uint32_t)bf(-2.0f) << 16);
  hw[0] = bf(3.0f) | ((uint32_t)bf(0.25f) << 16);
  uint32_t *da, *dw; float* dout;
  hipMalloc(&da, sizeof ha); hipMalloc(&dw, 4); hipMalloc(&dout, 192 * 4);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(dw, hw, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, da, dw, dout);
  float h[192];
  hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i)
    printf("i=%d a=(%g,%g) w=(3,0.25) dot2+0.5=%g expected %g\n", i, h[64 + i], h[128 + i], h[i],
           (1.0f + i) * 3.0f + (-2.0f) * 0.25f + 0.5f);
  return 0;
}
