// Micro-benchmark + bitwise check of the in-tree radix sort (fast_tffm_amd/csrc/hip/radix_sort.hip)
// against rocPRIM's onesweep (the dedup chain's FM_SORT=rocprim backend; its best measured config, 1024x8
// match ranking, 9-bit digits) on Criteo-shaped batches (n = 5.1M occurrences, ~85% on ~2k hot
// keys, power law).  Interleaved rounds in one process.  Build (in-tree, CPU side):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ifast_tffm_amd/csrc tools/bench_fmsort.hip -o tools/bench_fmsort
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "hip/fm_common.h"
namespace fm {
#include "hip/radix_sort.hip"
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using Cfg9 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 9,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 5111808;
  int bad_total = 0;
  for (int bits : {24, 27, 18, 32}) {
    const uint32_t range = bits >= 32 ? 0xffffffffu : (1u << bits);
    std::mt19937_64 rng(bits);
    std::vector<uint32_t> keys(n), hot(2048);
    for (auto& h : hot) h = (uint32_t)(rng() % range);
    std::uniform_real_distribution<double> U(0, 1);
    for (int i = 0; i < n; ++i) {
      if (U(rng) < 0.85) keys[i] = hot[(size_t)(std::pow(U(rng), 3.0) * hot.size()) % hot.size()];
      else keys[i] = (uint32_t)(rng() % range);
    }
    uint32_t *k, *ko, *ko2;
    int *v, *vo, *vo2;
    CK(hipMalloc(&k, n * 4)); CK(hipMalloc(&ko, n * 4)); CK(hipMalloc(&ko2, n * 4));
    CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&vo, n * 4)); CK(hipMalloc(&vo2, n * 4));
    CK(hipMemcpy(k, keys.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<int> iota(n);
    for (int i = 0; i < n; ++i) iota[i] = i;
    CK(hipMemcpy(v, iota.data(), n * 4, hipMemcpyHostToDevice));
    size_t rb = 0;
    CK(rocprim::radix_sort_pairs<Cfg9>(nullptr, rb, k, ko, v, vo, n, 0, bits, 0));
    void* rtmp;
    CK(hipMalloc(&rtmp, rb));
    const size_t wb = fm::radix_sort_ws_bytes(n);
    void* ws;
    CK(hipMalloc(&ws, wb));
    CK(hipMemset(ws, 0, wb));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto t_roc = [&](int it) {
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < it; ++i) CK(rocprim::radix_sort_pairs<Cfg9>(rtmp, rb, k, ko, v, vo, n, 0, bits, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1000.f / it;
    };
    auto t_fm = [&](int it) {
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < it; ++i) {
        const int r = fm::launch_radix_sort(k, v, ko2, vo2, n, bits, ws, wb, st);
        if (r) { fprintf(stderr, "launch_radix_sort %d\n", r); exit(1); }
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms * 1000.f / it;
    };
    t_roc(2);
    t_fm(2);
    std::vector<float> a, b;
    for (int round = 0; round < 5; ++round) {
      a.push_back(t_roc(20));
      b.push_back(t_fm(20));
    }
    std::vector<uint32_t> hk1(n), hk2(n);
    std::vector<int> hv1(n), hv2(n);
    CK(hipMemcpy(hk1.data(), ko, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hk2.data(), ko2, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hv1.data(), vo, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hv2.data(), vo2, n * 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int i = 0; i < n; ++i) bad += (hk1[i] != hk2[i]) || (hv1[i] != hv2[i]);
    int err = 0;
    CK(hipMemcpy(&err, fm::radix_sort_error(ws, n), 4, hipMemcpyDeviceToHost));
    if (err) printf("look-back error word %d\n", err);
    bad_total += bad != 0 || err != 0;
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    printf("n=%d bits=%d: rocPRIM onesweep 9-bit %.1f us (min %.1f) | in-tree %.1f us (min %.1f) | %s (%ld mismatches)\n",
           n, bits, a[2], a[0], b[2], b[0], bad ? "MISMATCH" : "bitwise equal", bad);
    CK(hipFree(k)); CK(hipFree(ko)); CK(hipFree(ko2)); CK(hipFree(v)); CK(hipFree(vo)); CK(hipFree(vo2));
    CK(hipFree(rtmp)); CK(hipFree(ws));
    CK(hipStreamDestroy(st));
  }
  return bad_total;
}
