// Probe of the two gfx950 primitives an MFMA fp8 forward needs (run on the GPU box; prints PASS/FAIL):
//  1. ds_read_b64_tr_b8 (__builtin_amdgcn_ds_read_tr8_b64_v2i32): per 16-lane group, lane 2q+p supplies the
//     address of row q (q = 0..7), bytes 8p..8p+7 of an 8-row x 16-byte block; expected: lane i of the group
//     receives column i of the 8 rows, row j in byte j.
//  2. v_mfma_f32_16x16x32_bf8_fp8: A (e5m2) lane l holds A[m = l & 15][k = 8 (l >> 4) + j] in byte j, B (e4m3)
//     lane l holds B[k = 8 (l >> 4) + j][n = l & 15]; D: col = l & 15, row = 4 (l >> 4) + i.
// Exact small-integer data, asymmetric operands (cdna_hip_programming.md §3).
//   hipcc --offload-arch=gfx950 -O2 -o mfma_fp8_probe mfma_fp8_probe.hip && ./mfma_fp8_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void tr8_probe(uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 128];
  const int l = threadIdx.x;
  for (int k = l; k < 512; k += 64) lds[k] = (uint8_t)(k * 7 + 3);
  __syncthreads();
  const int g = l >> 4, i = l & 15;
  const int addr = 128 * g + (i >> 1) * 16 + (i & 1) * 8;
  typedef __attribute__((__vector_size__(2 * sizeof(int)))) int i32x2;
  auto p = reinterpret_cast<__attribute__((address_space(3))) i32x2*>(
      reinterpret_cast<__attribute__((address_space(3))) uint8_t*>((__attribute__((address_space(3))) uint8_t*)lds) + addr);
  const i32x2 r = __builtin_amdgcn_ds_read_tr8_b64_v2i32(p);
  reinterpret_cast<int*>(out)[2 * l] = r[0];
  reinterpret_cast<int*>(out)[2 * l + 1] = r[1];
}

__global__ void mfma_probe(const uint8_t* A, const uint8_t* B, float* D) {
  // A: [16][32] e5m2 bytes row-major; B: [32][16] e4m3 bytes row-major
  const int l = threadIdx.x;
  long a = 0, b = 0;
  for (int j = 0; j < 8; ++j) {
    a |= (long)A[(l & 15) * 32 + 8 * (l >> 4) + j] << (8 * j);
    b |= (long)B[(8 * (l >> 4) + j) * 16 + (l & 15)] << (8 * j);
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[l * 4 + i] = c[i];
}

static uint8_t enc(int v, int ebits, int mbits) {  // small integers (|v| <= 8) -> OCP fp8 (normal)
  if (v == 0) return 0;
  const int s = v < 0;
  int a = s ? -v : v;
  int e = 0;
  while ((1 << (e + 1)) <= a) ++e;
  const int bias = (1 << (ebits - 1)) - 1;
  const int mant = ((a << mbits) >> e) & ((1 << mbits) - 1);
  return (uint8_t)((s << 7) | ((e + bias) << mbits) | mant);
}

int main() {
  uint8_t* d;
  hipMalloc(&d, 512);
  hipLaunchKernelGGL(tr8_probe, dim3(1), dim3(64), 0, 0, d);
  std::vector<uint8_t> h(512);
  hipMemcpy(h.data(), d, 512, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    for (int j = 0; j < 8; ++j) {
      const uint8_t want = (uint8_t)((128 * g + 16 * j + i) * 7 + 3);
      if (h[8 * l + j] != want) ++bad;
    }
  }
  printf("tr8: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  if (bad) {
    for (int l = 0; l < 4; ++l) {
      printf("lane %d:", l);
      for (int j = 0; j < 8; ++j) printf(" %3d", (int)((uint8_t)(h[8 * l + j] - 3) * 183 % 256));  // (x*7 inverse mod 256 = 183)
      printf("\n");
    }
  }
  // MFMA
  std::vector<int> Ai(16 * 32), Bi(32 * 16);
  std::vector<uint8_t> A(16 * 32), B(32 * 16);
  for (int m = 0; m < 16; ++m)
    for (int k = 0; k < 32; ++k) { Ai[m * 32 + k] = ((m * 5 + k * 3) % 9) - 4; A[m * 32 + k] = enc(Ai[m * 32 + k], 5, 2); }
  for (int k = 0; k < 32; ++k)
    for (int n = 0; n < 16; ++n) { Bi[k * 16 + n] = ((k * 7 + n * 2 + 1) % 7) - 3; B[k * 16 + n] = enc(Bi[k * 16 + n], 4, 3); }
  uint8_t *dA, *dB;
  float* dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  std::vector<float> D(256);
  hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
  int badm = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * (l >> 4) + i, col = l & 15;
      int want = 0;
      for (int k = 0; k < 32; ++k) want += Ai[row * 32 + k] * Bi[k * 16 + col];
      if (D[l * 4 + i] != (float)want) ++badm;
    }
  printf("mfma bf8 x fp8 16x16x32: %s (%d mismatches)\n", badm ? "FAIL" : "PASS", badm);
  return bad || badm;
}
