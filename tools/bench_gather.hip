// Random-row gather roofline on MI355X: how fast can the memory system deliver uniformly random
// 256-B rows (k=64 fp32 table rows) of a table far larger than the Infinity Cache, read-only and
// read-modify-write, with many rows in flight per lane group.  The anchor for the step's two big
// kernels: the forward reads the batch's cold rows once per occurrence, the chunk backward
// read-modify-writes each distinct row (v + Adagrad slot).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench_gather.hip -o /tmp/bench_gather
//   /tmp/bench_gather [table_rows=125000000] [n_rows=378000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int LPR = 16;  // 16 lanes x 16 B = one 256-B row
constexpr int G = 64 / LPR;

// read-only: UNR rows in flight per lane group, summed into a per-thread accumulator
template <int UNR>
__global__ __launch_bounds__(256) void gather_ro(const float4* __restrict__ tab, const int* __restrict__ idx, int n,
                                                 float* out) {
  const int lane = threadIdx.x & 63, g = lane / LPR, t = lane % LPR;
  const int groups = gridDim.x * 4 * G;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = ((blockIdx.x * 4 + (threadIdx.x >> 6)) * G + g) * UNR; base < n; base += groups * UNR) {
    float4 r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = base + u;
      const long long row = idx[i < n ? i : base];
      r[u] = tab[row * LPR + t];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc.x += r[u].x; acc.y += r[u].y; acc.z += r[u].z; acc.w += r[u].w;
    }
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;  // keep the loads
}

// read-modify-write of two arrays (v and its Adagrad slot), UNR rows in flight
template <int UNR>
__global__ __launch_bounds__(256) void rmw2(float4* __restrict__ v, float4* __restrict__ s, const int* __restrict__ idx,
                                            int n) {
  const int lane = threadIdx.x & 63, g = lane / LPR, t = lane % LPR;
  const int groups = gridDim.x * 4 * G;
  for (int base = ((blockIdx.x * 4 + (threadIdx.x >> 6)) * G + g) * UNR; base < n; base += groups * UNR) {
    float4 a[UNR], b[UNR];
    long long rows[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = base + u;
      rows[u] = idx[i < n ? i : base];
      a[u] = v[rows[u] * LPR + t];
      b[u] = s[rows[u] * LPR + t];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (base + u >= n) continue;
      b[u].x += 1e-6f; b[u].y += 1e-6f; b[u].z += 1e-6f; b[u].w += 1e-6f;
      a[u].x -= 1e-6f * b[u].x; a[u].y -= 1e-6f * b[u].y; a[u].z -= 1e-6f * b[u].z; a[u].w -= 1e-6f * b[u].w;
      v[rows[u] * LPR + t] = a[u];
      s[rows[u] * LPR + t] = b[u];
    }
  }
}

template <class F>
float time_us(F f, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  const long long V = argc > 1 ? atoll(argv[1]) : 125000000LL;
  const int n = argc > 2 ? atoi(argv[2]) : 378000;
  float4 *v, *s;
  CK(hipMalloc(&v, V * 256));
  CK(hipMalloc(&s, V * 256));
  CK(hipMemset(v, 0, V * 256));
  CK(hipMemset(s, 0, V * 256));
  std::mt19937_64 rng(7);
  std::vector<int> h(n);
  for (auto& x : h) x = (int)(rng() % (unsigned long long)V);
  std::vector<int> hs(h);
  std::sort(hs.begin(), hs.end());
  int *d, *ds;
  float* out;
  CK(hipMalloc(&d, n * 4));
  CK(hipMalloc(&ds, n * 4));
  CK(hipMalloc(&out, 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), n * 4, hipMemcpyHostToDevice));
  const double gb = (double)n * 256 / 1e9;
  printf("table %lld rows x 256 B (%.1f GB each array), %d uniformly random rows\n", V, V * 256 / 1e9, n);
  for (int grid : {1024, 2048, 4096, 8192}) {
    const float t1 = time_us([&] { hipLaunchKernelGGL(gather_ro<1>, dim3(grid), dim3(256), 0, 0, v, d, n, out); }, 20);
    const float t4 = time_us([&] { hipLaunchKernelGGL(gather_ro<4>, dim3(grid), dim3(256), 0, 0, v, d, n, out); }, 20);
    const float t8 = time_us([&] { hipLaunchKernelGGL(gather_ro<8>, dim3(grid), dim3(256), 0, 0, v, d, n, out); }, 20);
    const float t8s = time_us([&] { hipLaunchKernelGGL(gather_ro<8>, dim3(grid), dim3(256), 0, 0, v, ds, n, out); }, 20);
    const float r4 = time_us([&] { hipLaunchKernelGGL(rmw2<4>, dim3(grid), dim3(256), 0, 0, v, s, d, n); }, 20);
    const float r4s = time_us([&] { hipLaunchKernelGGL(rmw2<4>, dim3(grid), dim3(256), 0, 0, v, s, ds, n); }, 20);
    printf("grid %5d  read-only UNR1 %6.1f us (%5.2f TB/s)  UNR4 %6.1f (%5.2f)  UNR8 %6.1f (%5.2f)  UNR8 sorted %6.1f (%5.2f)"
           "  |  RMW v+slot UNR4 %6.1f us (%5.2f TB/s moved)  sorted %6.1f (%5.2f)\n",
           grid, t1, gb / t1 * 1e3, t4, gb / t4 * 1e3, t8, gb / t8 * 1e3, t8s, gb / t8s * 1e3, r4, 4 * gb / r4 * 1e3,
           r4s, 4 * gb / r4s * 1e3);
  }
  return 0;
}
