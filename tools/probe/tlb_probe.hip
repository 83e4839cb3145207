// Does the allocation path change the random-row gather rate over a 32 GB table (UTCL1 misses were
// ~50% in the k64 forward)?  hipMalloc vs hipExtMallocWithFlags(hipDeviceMallocContiguous), 5.1M
// uniformly random 256-B rows (the forward's occurrence count), read-only, 8 rows in flight per group.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/tlb_probe.hip -o tools/probe/tlb_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

template <int UNR>
__global__ __launch_bounds__(256) void gather_ro(const float4* __restrict__ tab, const int* __restrict__ idx, int n,
                                                 float* out) {
  const int lane = threadIdx.x & 63, g = lane / 16, t = lane % 16;
  const int groups = gridDim.x * 4 * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = ((blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + g) * UNR; base < n; base += groups * UNR) {
    float4 r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = base + u;
      const long long row = idx[i < n ? i : base];
      r[u] = tab[row * 16 + t];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc.x += r[u].x; acc.y += r[u].y; acc.z += r[u].z; acc.w += r[u].w;
    }
  }
  if (acc.x + acc.y + acc.z + acc.w == 1.2345f) out[0] = acc.x;
}

static float time_us(const float4* tab, const int* d, int n, float* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(gather_ro<8>, dim3(4096), dim3(256), 0, 0, tab, d, n, out);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(gather_ro<8>, dim3(4096), dim3(256), 0, 0, tab, d, n, out);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / 20;
}

int main() {
  const long long V = 125000000LL;
  const int n = 5111808;
  const size_t bytes = (size_t)V * 256;
  float4 *t0 = nullptr, *t1 = nullptr;
  CK(hipMalloc(&t0, bytes));
  CK(hipMemset(t0, 0, bytes));
  const hipError_t ec = hipExtMallocWithFlags(reinterpret_cast<void**>(&t1), bytes, hipDeviceMallocContiguous);
  if (ec != hipSuccess) {
    printf("hipDeviceMallocContiguous of %.1f GB: %s\n", bytes / 1e9, hipGetErrorString(ec));
    t1 = nullptr;
  } else {
    CK(hipMemset(t1, 0, bytes));
  }
  std::mt19937_64 rng(7);
  std::vector<int> h(n);
  for (auto& x : h) x = (int)(rng() % (unsigned long long)V);
  int* d;
  float* out;
  CK(hipMalloc(&d, (size_t)n * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemcpy(d, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  for (int round = 0; round < 3; ++round) {
    const float a = time_us(t0, d, n, out);
    printf("hipMalloc            : %7.1f us (%.2f TB/s of rows)\n", a, n * 256.0 / a / 1e6);
    if (t1) {
      const float b = time_us(t1, d, n, out);
      printf("contiguous allocation: %7.1f us (%.2f TB/s of rows)\n", b, n * 256.0 / b / 1e6);
    }
  }
  return 0;
}
