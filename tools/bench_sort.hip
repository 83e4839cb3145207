// Micro-benchmark: rocPRIM onesweep radix sort of (27-bit key, int32 payload)
// pairs shaped like one Criteo-like FM batch (n = 5.1M occurrences, ~85% on
// ~2k hot keys), for several onesweep configurations. Interleaved rounds in
// one process (cdna_hip_programming.md §5.4 rule 24). Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench_sort.hip -o /tmp/bench_sort
#include <cstring>
#include <cmath>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

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

using rocprim::block_radix_rank_algorithm;
using rocprim::kernel_config;

template <unsigned BS, unsigned IPT, unsigned BITS, block_radix_rank_algorithm ALG>
using OS = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                      rocprim::radix_sort_onesweep_config<kernel_config<1024, 8>,
                                                                          kernel_config<BS, IPT>, BITS, ALG>,
                                      0>;

struct Buffers {
  uint32_t *k, *ko;
  int *v, *vo;
  void* tmp;
  size_t tmp_bytes;
  int n;
};

template <class Cfg>
float run(Buffers& b, int bits, int iters, hipStream_t st) {
  size_t need = 0;
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, need, b.k, b.ko, b.v, b.vo, b.n, 0, bits, st));
  if (need > b.tmp_bytes) {
    fprintf(stderr, "tmp too small %zu > %zu\n", need, b.tmp_bytes);
    exit(1);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(rocprim::radix_sort_pairs<Cfg>(b.tmp, need, b.k, b.ko, b.v, b.vo, b.n, 0, bits, st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i)
    CK(rocprim::radix_sort_pairs<Cfg>(b.tmp, need, b.k, b.ko, b.v, b.vo, b.n, 0, bits, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 5111808;
  const int bits = 27;
  std::mt19937_64 rng(1);
  std::vector<uint32_t> keys(n);
  std::vector<uint32_t> hot(2048);
  for (auto& h : hot) h = rng() % 125000000u;
  std::uniform_real_distribution<double> U(0, 1);
  for (int i = 0; i < n; ++i) {
    if (U(rng) < 0.85) {
      // power-law over the hot set
      const double r = std::pow(U(rng), 3.0);
      keys[i] = hot[(size_t)(r * hot.size()) % hot.size()];
    } else {
      keys[i] = rng() % 125000000u;
    }
  }
  Buffers b;
  b.n = n;
  CK(hipMalloc(&b.k, n * 4));
  CK(hipMalloc(&b.ko, n * 4));
  CK(hipMalloc(&b.v, n * 4));
  CK(hipMalloc(&b.vo, n * 4));
  b.tmp_bytes = 256u << 20;
  CK(hipMalloc(&b.tmp, b.tmp_bytes));
  CK(hipMemcpy(b.k, keys.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<int> iota(n);
  for (int i = 0; i < n; ++i) iota[i] = i;
  CK(hipMemcpy(b.v, iota.data(), n * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));

  const char* names[] = {"default", "1024x8 b8 match", "512x8 b8 match", "256x16 b8 match", "1024x8 b9 match",
                         "512x8 b9 match", "1024x8 b10 match", "512x16 b10 match", "1024x8 b11 match",
                         "512x8 b11 match", "256x8 b8 basic", "1024x12 b9 match"};
  const int NC = sizeof(names) / sizeof(names[0]);
  std::vector<std::vector<float>> t(NC);
  for (int round = 0; round < 5; ++round) {
    int c = 0;
    t[c++].push_back(run<rocprim::default_config>(b, bits, 20, st));
    t[c++].push_back(run<OS<1024, 8, 8, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<512, 8, 8, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<256, 16, 8, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<1024, 8, 9, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<512, 8, 9, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<1024, 8, 10, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<512, 16, 10, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<1024, 8, 11, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<512, 8, 11, block_radix_rank_algorithm::match>>(b, bits, 20, st));
    t[c++].push_back(run<OS<256, 8, 8, block_radix_rank_algorithm::basic>>(b, bits, 20, st));
    t[c++].push_back(run<OS<1024, 12, 9, block_radix_rank_algorithm::match>>(b, bits, 20, st));
  }
  printf("rocPRIM onesweep radix_sort_pairs, n=%d, %d key bits (us per sort: median / min over 5 rounds x 20)\n",
         n, bits);
  for (int c = 0; c < NC; ++c) {
    std::sort(t[c].begin(), t[c].end());
    printf("  %-20s %8.1f %8.1f\n", names[c], t[c][t[c].size() / 2], t[c][0]);
  }
  // correctness spot check of the last config's output ordering
  std::vector<uint32_t> out(n);
  CK(hipMemcpy(out.data(), b.ko, n * 4, hipMemcpyDeviceToHost));
  for (int i = 1; i < n; ++i)
    if (out[i - 1] > out[i]) {
      printf("NOT SORTED at %d\n", i);
      return 1;
    }
  printf("sorted ok\n");
  return 0;
}
