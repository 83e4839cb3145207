// Probe: semantics of gfx950's v_cvt_scalef32_pk_f32_fp8 (scaled fp8 -> f32) for a non-power-of-two
// scale -- is the scale multiplied in full, or only its exponent (E8M0-style)?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* in, const float* sc, float* out) {
  const int i = threadIdx.x;
  f2 a = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(in[i], sc[i], false);
  f2 b = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(in[i], sc[i], true);
  f2 c = __builtin_amdgcn_cvt_pk_f32_fp8(in[i], false);
  out[6 * i] = a.x; out[6 * i + 1] = a.y; out[6 * i + 2] = b.x; out[6 * i + 3] = b.y;
  out[6 * i + 4] = c.x; out[6 * i + 5] = c.y;
}
int main() {
  const int n = 4;
  unsigned hin[n] = {0x40384038u, 0x38403840u, 0x7e017e01u, 0x01020304u};  // fp8 e4m3 bytes
  float hsc[n] = {1.0f, 3.0f, 0.375f, 1.5f};
  unsigned* din; float *dsc, *dout;
  (void)hipMalloc(&din, sizeof(hin)); (void)hipMalloc(&dsc, sizeof(hsc)); (void)hipMalloc(&dout, 6 * n * sizeof(float));
  (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
  (void)hipMemcpy(dsc, hsc, sizeof(hsc), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(n), 0, 0, din, dsc, dout);
  float h[6 * n];
  if (hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
  for (int i = 0; i < n; ++i)
    printf("in=%08x scale=%g  scaled: %g %g %g %g   plain: %g %g\n", hin[i], hsc[i], h[6 * i], h[6 * i + 1],
           h[6 * i + 2], h[6 * i + 3], h[6 * i + 4], h[6 * i + 5]);
  return 0;
}
