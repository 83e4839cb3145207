// Batch de-duplication on gfx950: the replacement for tf.unique
// (reference tffm/fm_model.py:72, :133, :173) and for the implicit grouping the
// reference's FmGrad gets from 168M fp32 atomicAdds (cc/fm_grad_op.h:84-104).
//
// Pipeline (every data-dependent size stays on the device, so the chain needs
// no host sync and is hipGraph-capturable):
//   1. stable LSD radix sort of (key, payload) pairs over only the key bits in
//      use (rocPRIM onesweep).  The payload is the occurrence index, or -- when
//      the caller needs neither the inverse map nor per-occurrence values --
//      directly the example index, which saves the gather in step 3;
//   2. ONE inclusive scan of a packed 64-bit flag per sorted position:
//      high word = "segment head" (key differs from its left neighbour), low
//      word = "chunk start" (head, or position % CH == 0).  The flags are
//      computed on the fly by a transform iterator (no flag array);
//   3. one emit kernel: unique keys, segment starts, first chunk of each
//      segment, chunk starts and chunk->segment map, U and #chunks, plus the
//      optional inverse map and per-sorted-occurrence example index / value.
// Chunks cut every segment at CH-aligned sorted positions, so no chunk is
// longer than CH and a hot id (tens of thousands of occurrences in Criteo's
// low-cardinality fields) is spread over many lane groups in the backward.
#include "fm_common.h"
#include <rocprim/rocprim.hpp>

namespace fm {

struct FlagOp {
  const uint32_t* skeys;
  int CH;
  __device__ __host__ unsigned long long operator()(int j) const {
    const bool head = (j == 0) || (skeys[j] != skeys[j - 1]);
    const bool cstart = head || (j % CH == 0);
    return ((unsigned long long)(head ? 1u : 0u) << 32) | (cstart ? 1ull : 0ull);
  }
};

struct EmitArgs {
  int n, CH;
  const uint32_t* skeys;          // sorted keys
  const int* spay;                // sorted payload (occurrence or example index)
  const unsigned long long* incl; // inclusive scan of packed flags
  uint32_t* uniq;                 // [n] unique keys (first U valid)
  int* seg_start;                 // [n+1]
  int* seg_chunk;                 // [n+1] first chunk of each segment
  int* chunk_start;               // [n+1]
  int* chunk_seg;                 // [n]
  int* counts;                    // device [2]: U, #chunks
  int* inv;                       // [n] occurrence -> segment (payload = occurrence)
  const int* ex_of_occ;           // [n] (payload = occurrence)
  int* sorted_ex;                 // [n] (payload = occurrence)
  const float* vals;              // [n] (payload = occurrence)
  float* sorted_x;                // [n] (payload = occurrence)
};

__global__ __launch_bounds__(kBlock) void rle_emit_kernel(EmitArgs a) {
  for (int j = blockIdx.x * kBlock + threadIdx.x; j < a.n; j += gridDim.x * kBlock) {
    const unsigned long long v = a.incl[j];
    const unsigned long long vp = j > 0 ? a.incl[j - 1] : 0ull;
    const int s = (int)(v >> 32) - 1;
    const int c = (int)(v & 0xffffffffull) - 1;
    const bool head = (v >> 32) != (vp >> 32);
    const bool cstart = (v & 0xffffffffull) != (vp & 0xffffffffull);
    if (head) {
      a.uniq[s] = a.skeys[j];
      a.seg_start[s] = j;
      a.seg_chunk[s] = c;
    }
    if (cstart) {
      a.chunk_start[c] = j;
      a.chunk_seg[c] = s;
    }
    if (j == a.n - 1) {
      a.counts[0] = s + 1;
      a.counts[1] = c + 1;
      a.seg_start[s + 1] = a.n;
      a.seg_chunk[s + 1] = c + 1;
      a.chunk_start[c + 1] = a.n;
    }
    if (a.inv || a.sorted_ex || a.sorted_x) {
      const int p = a.spay[j];
      if (a.inv) a.inv[p] = s;
      if (a.sorted_ex) a.sorted_ex[j] = a.ex_of_occ[p];
      if (a.sorted_x) a.sorted_x[j] = a.vals[p];
    }
  }
}

static int grid_for(long long n) {
  long long b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (int)b;
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

using FlagIter = rocprim::transform_iterator<rocprim::counting_iterator<int>, FlagOp, unsigned long long>;

static size_t temp_bytes(int n, hipStream_t st) {
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const int*)nullptr, (int*)nullptr, n, 0, 32, st);
  FlagIter it(rocprim::counting_iterator<int>(0), FlagOp{nullptr, 1});
  (void)rocprim::inclusive_scan((void*)nullptr, scan_bytes, it, (unsigned long long*)nullptr, (size_t)n,
                                rocprim::plus<unsigned long long>(), st);
  return align_up(sort_bytes > scan_bytes ? sort_bytes : scan_bytes);
}

// Workspace layout: [rocprim temp | u64 incl(n)]
size_t dedup_workspace_bytes(int n) {
  if (n <= 0) return 256;
  return temp_bytes(n, 0) + align_up(sizeof(unsigned long long) * (size_t)n) + 256;
}

struct DedupArgs {
  int n;
  int end_bit;             // number of key bits to sort on
  int CH;                  // chunk length of the backward plan
  const uint32_t* keys;    // [n]
  const int* payload;      // [n] values carried by the sort
  uint32_t* skeys;         // [n]
  int* spay;               // [n] sorted payload ("perm")
  uint32_t* uniq;          // [n]
  int* seg_start;          // [n+1]
  int* seg_chunk;          // [n+1]
  int* chunk_start;        // [n+1]
  int* chunk_seg;          // [n]
  int* counts;             // device [2]
  int* inv;                // nullable
  const int* ex_of_occ;    // nullable
  int* sorted_ex;          // nullable
  const float* vals;       // nullable
  float* sorted_x;         // nullable
  void* ws;
  size_t ws_bytes;
};

int launch_dedup(const DedupArgs& a, hipStream_t st) {
  if (a.n <= 0) {
    (void)hipMemsetAsync(a.counts, 0, 2 * sizeof(int), st);
    (void)hipMemsetAsync(a.seg_start, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.seg_chunk, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.chunk_start, 0, sizeof(int), st);
    return (int)hipGetLastError();
  }
  const size_t tmp = temp_bytes(a.n, st);
  auto* incl = reinterpret_cast<unsigned long long*>(static_cast<char*>(a.ws) + tmp);
  if (tmp + sizeof(unsigned long long) * (size_t)a.n > a.ws_bytes) return -2;

  size_t sort_bytes = tmp;
  hipError_t e = rocprim::radix_sort_pairs(a.ws, sort_bytes, a.keys, a.skeys, a.payload, a.spay, a.n, 0,
                                           a.end_bit, st);
  if (e != hipSuccess) return (int)e;
  FlagIter it(rocprim::counting_iterator<int>(0), FlagOp{a.skeys, a.CH});
  size_t scan_bytes = tmp;
  e = rocprim::inclusive_scan(a.ws, scan_bytes, it, incl, (size_t)a.n, rocprim::plus<unsigned long long>(), st);
  if (e != hipSuccess) return (int)e;
  EmitArgs em{a.n, a.CH, a.skeys, a.spay, incl, a.uniq, a.seg_start, a.seg_chunk, a.chunk_start, a.chunk_seg,
              a.counts, a.inv, a.ex_of_occ, a.sorted_ex, a.vals, a.sorted_x};
  hipLaunchKernelGGL(rle_emit_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, st, em);
  return (int)hipGetLastError();
}

}  // namespace fm
