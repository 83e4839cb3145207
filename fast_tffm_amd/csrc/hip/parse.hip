// GPU libsvm tokenizer: a batch of text lines -> CSR on the device.
//
// The host loader (csrc/cpu/loader.h, raw mode) does file I/O, the shuffle
// window and gathers the chosen lines into one contiguous buffer; this file
// parses it on the GPU (the reference parses on one CPU thread per op call,
// cc/fm_parser_op.cc:39-45, 58-109), so file-fed training is not bound by host
// parsing.  Two passes, one wave64 per line:
//   1. count: tokens of line i = its ' ' count (minus a trailing space);
//      exclusive scan -> CSR offsets;
//   2. parse: the line is staged in LDS; lane j tests byte 64*w + j for a token
//      start (previous byte ' '), a ballot + popcount gives each starting lane
//      its output slot, and the lane parses its token (decimal id or Hash64 of
//      the token bytes modulo vocab, optional ':' value) sequentially from LDS;
//      lane 0 parses the label.
// Supported syntax is the common subset of the reference grammar: label and
// values are plain decimals ([+-]digits[.digits][e[+-]digits], <= 15
// significant digits), ids plain digits, single spaces.  Anything else --
// including every malformed line -- sets `fallback`, and the host re-parses the
// whole batch with the CPU parser, which produces the reference's exact
// results and error messages.  Values are converted through double (m * 10^e,
// correctly rounded) then to float: equal to strtof except in rare double-
// rounding ties (<= 1 ulp).
#include "fm_common.h"
#include "../hash64.h"
#include <rocprim/rocprim.hpp>

namespace fm {

constexpr int kParseMaxLine = 2048;        // bytes of one line staged in LDS (longer: fallback)
constexpr int kParseWaves = 4;             // waves (lines in flight) per workgroup

struct ParseArgs {
  const char* buf;               // batch bytes
  const long long* line_start;   // [n + 1]: line i is [line_start[i], line_start[i+1]) (incl. its '\n')
  int n;
  long long vocab;
  int hash;
  int require_vals;              // 1: every token must carry ':value' (serving lines), else fallback
  int* counts;                   // [n] tokens per line (pass 1)
  const int* offsets;            // [n + 1] exclusive scan of counts (pass 2)
  float* labels;                 // [n]
  int* ids;                      // [nnz]
  float* vals;                   // [nnz]
  int* status;                   // [4]: fallback flag, max tokens per line, any value != 1, (spare)
};

__device__ inline int line_len(const ParseArgs& a, int i, long long& s) {
  s = a.line_start[i];
  long long e = a.line_start[i + 1];
  if (e > s && a.buf[e - 1] == '\n') --e;
  if (e > s && a.buf[e - 1] == '\r') --e;
  return (int)(e - s);
}

__global__ __launch_bounds__(kWave * kParseWaves) void parse_count_kernel(ParseArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = blockIdx.x * kParseWaves + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * kParseWaves;
  for (int i = wave; i < a.n; i += nwaves) {
    long long s;
    const int len = line_len(a, i, s);
    int sp = 0;
    for (int p = lane; p < len; p += kWave) sp += a.buf[s + p] == ' ';
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) sp += __shfl_xor(sp, o, kWave);
    if (lane == 0) {
      const int trailing = len > 0 && a.buf[s + len - 1] == ' ';
      const int cnt = sp - trailing;
      a.counts[i] = cnt;
      atomicMax(&a.status[1], cnt);
      if (len > kParseMaxLine || len == 0) atomicOr(&a.status[0], 1);
    }
  }
}

// Plain decimal [+-]d*[.d*][(e|E)[+-]d+] over [p, end): false if the text is
// anything else (then the CPU parser decides).
__device__ inline bool parse_decimal(const char* p, const char* end, float& out) {
  bool neg = false;
  if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
  unsigned long long m = 0;
  int digits = 0, exp10 = 0, sig = 0;
  while (p < end && *p >= '0' && *p <= '9') {
    if (m != 0 || *p != '0') {
      if (sig >= 15) return false;
      ++sig;
    }
    m = m * 10 + (unsigned)(*p - '0');
    ++p; ++digits;
  }
  if (p < end && *p == '.') {
    ++p;
    while (p < end && *p >= '0' && *p <= '9') {
      if (m != 0 || *p != '0') {
        if (sig >= 15) return false;
        ++sig;
      }
      m = m * 10 + (unsigned)(*p - '0');
      --exp10;
      ++p; ++digits;
    }
  }
  if (digits == 0) return false;
  if (p < end && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < end && (*p == '+' || *p == '-')) { eneg = *p == '-'; ++p; }
    int e = 0, ed = 0;
    while (p < end && *p >= '0' && *p <= '9') {
      if (e < 1000) e = e * 10 + (*p - '0');
      ++p; ++ed;
    }
    if (ed == 0) return false;
    exp10 += eneg ? -e : e;
  }
  if (p != end) return false;
  double d = (double)m;  // exact: < 10^15 < 2^53
  if (m != 0) {
    if (exp10 > 22 || exp10 < -22) return false;
    // powers of ten up to 1e22 are exact doubles: one correctly rounded multiply / divide
    double pw = 1.0;
    for (int k = 0; k < (exp10 < 0 ? -exp10 : exp10); ++k) pw *= 10.0;
    d = exp10 < 0 ? d / pw : d * pw;
  }
  out = (float)(neg ? -d : d);
  return true;
}

__global__ __launch_bounds__(kWave * kParseWaves) void parse_tokens_kernel(ParseArgs a) {
  __shared__ char lds[kParseWaves][kParseMaxLine + 4];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x >> 6;
  char* L = lds[wv];
  const int nwaves = gridDim.x * kParseWaves;
  for (int i = blockIdx.x * kParseWaves + wv; i < a.n; i += nwaves) {
    long long s;
    const int len = line_len(a, i, s);
    if (len > kParseMaxLine || len == 0) continue;  // fallback already flagged by pass 1
    for (int p = lane; p < len; p += kWave) L[p] = a.buf[s + p];
    if (lane == 0) L[len] = '\0';
    // LDS written by the whole wave, read by single lanes below
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int out0 = a.offsets[i];
    const int cnt = a.counts[i];
    bool bad = false;
    bool nonunit = false;
    // label: bytes up to the first ' ' (or the end)
    if (lane == 0) {
      int q = 0;
      while (q < len && L[q] != ' ') ++q;
      float lab;
      if (!parse_decimal(L, L + q, lab)) bad = true;
      else a.labels[i] = lab;
    }
    int base = 0;
    for (int w = 0; w * kWave < len; ++w) {
      const int p = w * kWave + lane;
      const bool start = p > 0 && p < len && L[p - 1] == ' ';
      const unsigned long long mask = __ballot(start);
      if (start) {
        const int k = base + __popcll(mask & ((1ull << lane) - 1));
        if (L[p] == ' ' || k >= cnt) {
          bad = true;  // double space (strtoll would skip it: CPU decides) / count mismatch
        } else {
          int q = p;
          long long id = 0;
          if (a.hash) {
            while (q < len && L[q] != ' ' && L[q] != ':') ++q;
            id = (long long)(hash64(L + p, (size_t)(q - p)) % (unsigned long long)a.vocab);
          } else {
            int nd = 0;
            while (q < len && L[q] >= '0' && L[q] <= '9') {
              if (nd < 18) id = id * 10 + (L[q] - '0');
              ++q; ++nd;
            }
            if (nd == 0 || nd >= 18 || id >= a.vocab || (q < len && L[q] != ' ' && L[q] != ':')) bad = true;
          }
          float v = 1.f;
          if (a.require_vals && !(q < len && L[q] == ':')) bad = true;
          if (!bad && q < len && L[q] == ':') {
            int r = q + 1;
            while (r < len && L[r] != ' ') ++r;
            if (!parse_decimal(L + q + 1, L + r, v)) bad = true;
            q = r;
          }
          if (!bad) {
            a.ids[out0 + k] = (int)id;
            a.vals[out0 + k] = v;
            nonunit |= v != 1.f;
          }
        }
      }
      base += __popcll(mask);
    }
    if (base != cnt) bad = true;
    if (__ballot(bad)) {
      if (lane == 0) atomicOr(&a.status[0], 1);
    }
    if (__ballot(nonunit)) {
      if (lane == 0) atomicOr(&a.status[2], 1);
    }
    __builtin_amdgcn_wave_barrier();  // every lane is done with L before the next line overwrites it
  }
}

size_t parse_workspace_bytes(int n) {
  size_t b = 0;
  (void)rocprim::exclusive_scan((void*)nullptr, b, (const int*)nullptr, (int*)nullptr, 0, (size_t)n + 1,
                                rocprim::plus<int>(), 0);
  return b;
}

// counts must hold n + 1 ints (counts[n] = 0 is scanned into offsets[n] = nnz).
int launch_parse(ParseArgs a, void* ws, size_t ws_bytes, int* offsets, hipStream_t st) {
  if (a.n <= 0) return 0;
  (void)hipMemsetAsync(a.status, 0, 4 * sizeof(int), st);
  (void)hipMemsetAsync(a.counts + a.n, 0, sizeof(int), st);
  const int grid = fill_grid(a.n, kParseWaves, 8192);
  hipLaunchKernelGGL(parse_count_kernel, dim3(grid), dim3(kWave * kParseWaves), 0, st, a);
  size_t b = ws_bytes;
  hipError_t e = rocprim::exclusive_scan(ws, b, a.counts, offsets, 0, (size_t)a.n + 1, rocprim::plus<int>(), st);
  if (e != hipSuccess) return (int)e;
  a.offsets = offsets;
  hipLaunchKernelGGL(parse_tokens_kernel, dim3(grid), dim3(kWave * kParseWaves), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm
