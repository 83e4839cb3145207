// Batch de-duplication on gfx950: the replacement for tf.unique
// (reference tffm/fm_model.py:72, :133, :173) and for the implicit grouping the
// reference's FmGrad gets from 168M fp32 atomicAdds (cc/fm_grad_op.h:84-104).
//
// Pipeline (all sizes that depend on the data stay on the device, so the whole
// chain is hipGraph-capturable and needs no host sync):
//   1. stable LSD radix sort of (key, occurrence) pairs, only over the key bits
//      actually used (rocPRIM onesweep);
//   2. head flags + inclusive scan -> segment id of every sorted occurrence;
//   3. emit: unique keys, segment starts, U, inverse map occurrence->segment,
//      and the per-sorted-occurrence example index / value the backward reads
//      contiguously;
//   4. chunk plan: rows with more than CH occurrences (hot ids) are cut into
//      CH-sized chunks so that no lane group of the backward runs much longer
//      than the others.
#include "fm_common.h"
#include <rocprim/rocprim.hpp>

namespace fm {

__global__ __launch_bounds__(kBlock) void mark_heads_kernel(const uint32_t* keys, int n, int* heads) {
  for (int j = blockIdx.x * kBlock + threadIdx.x; j < n; j += gridDim.x * kBlock)
    heads[j] = (j == 0 || keys[j] != keys[j - 1]) ? 1 : 0;
}

struct EmitArgs {
  int n;
  const uint32_t* skeys;   // sorted keys
  const int* perm;         // sorted occurrence index
  const int* incl;         // inclusive scan of heads
  uint32_t* uniq;          // [n] unique keys (first U valid)
  int* seg_start;          // [n+1]
  int* num_unique;         // device scalar
  int* inv;                // [n] occurrence -> segment (nullable)
  const int* ex_of_occ;    // [n] example of occurrence (nullable)
  int* sorted_ex;          // [n] (nullable)
  const float* vals;       // [n] (nullable)
  float* sorted_x;         // [n] (nullable)
};

__global__ __launch_bounds__(kBlock) void rle_emit_kernel(EmitArgs a) {
  for (int j = blockIdx.x * kBlock + threadIdx.x; j < a.n; j += gridDim.x * kBlock) {
    const int s = a.incl[j] - 1;
    const bool head = (j == 0) || (a.incl[j - 1] != a.incl[j]);
    if (head) {
      a.uniq[s] = a.skeys[j];
      a.seg_start[s] = j;
    }
    if (j == a.n - 1) {
      *a.num_unique = s + 1;
      a.seg_start[s + 1] = a.n;
    }
    const int p = a.perm[j];
    if (a.inv) a.inv[p] = s;
    if (a.sorted_ex) a.sorted_ex[j] = a.ex_of_occ[p];
    if (a.sorted_x) a.sorted_x[j] = a.vals[p];
  }
}

__global__ __launch_bounds__(kBlock) void chunk_count_kernel(int n, const int* num_unique, const int* seg_start,
                                                             int CH, int* counts) {
  const int U = *num_unique;
  for (int u = blockIdx.x * kBlock + threadIdx.x; u < n; u += gridDim.x * kBlock) {
    int c = 0;
    if (u < U) {
      const int len = seg_start[u + 1] - seg_start[u];
      c = len > CH ? (len + CH - 1) / CH : 1;
    }
    counts[u] = c;
  }
}

__global__ __launch_bounds__(kBlock) void chunk_emit_kernel(int n, const int* num_unique, const int* chunk_start,
                                                            int* chunk_seg, int* num_chunks) {
  const int U = *num_unique;
  for (int u = blockIdx.x * kBlock + threadIdx.x; u < U; u += gridDim.x * kBlock) {
    const int c0 = chunk_start[u], c1 = chunk_start[u + 1];
    for (int c = c0; c < c1; ++c) chunk_seg[c] = u;
    if (u == U - 1) *num_chunks = c1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && U == 0) *num_chunks = 0;
}

static int grid_for(long long n) {
  long long b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (int)b;
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// Workspace layout: [rocprim temp | int heads/incl(n) | int counts(n)]
size_t dedup_workspace_bytes(int n) {
  if (n <= 0) return 256;
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                            (const int*)nullptr, (int*)nullptr, n, 0, 32, 0);
  (void)rocprim::inclusive_scan((void*)nullptr, scan_bytes, (const int*)nullptr, (int*)nullptr, (size_t)n,
                          rocprim::plus<int>(), 0);
  const size_t tmp = align_up(sort_bytes > scan_bytes ? sort_bytes : scan_bytes);
  return tmp + 2 * align_up(sizeof(int) * (size_t)n) + align_up(sizeof(int) * ((size_t)n + 1)) + 256;
}

struct DedupArgs {
  int n;
  int end_bit;             // number of key bits to sort on
  const uint32_t* keys;    // [n]
  const int* iota;         // [n] 0..n-1 (values to sort)
  uint32_t* skeys;         // [n]
  int* perm;               // [n]
  uint32_t* uniq;          // [n]
  int* seg_start;          // [n+1]
  int* num_unique;         // device scalar
  int* inv;                // nullable
  const int* ex_of_occ;    // nullable
  int* sorted_ex;          // nullable
  const float* vals;       // nullable
  float* sorted_x;         // nullable
  void* ws;                // workspace (dedup_workspace_bytes)
  size_t ws_bytes;
};

int launch_dedup(const DedupArgs& a, hipStream_t st) {
  if (a.n <= 0) {
    (void)hipMemsetAsync(a.num_unique, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.seg_start, 0, sizeof(int), st);
    return (int)hipGetLastError();
  }
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, sort_bytes, a.keys, a.skeys, a.iota, a.perm, a.n, 0, a.end_bit, st);
  (void)rocprim::inclusive_scan((void*)nullptr, scan_bytes, (const int*)nullptr, (int*)nullptr, (size_t)a.n,
                          rocprim::plus<int>(), st);
  const size_t tmp = align_up(sort_bytes > scan_bytes ? sort_bytes : scan_bytes);
  char* base = static_cast<char*>(a.ws);
  int* heads = reinterpret_cast<int*>(base + tmp);
  int* incl = reinterpret_cast<int*>(base + tmp + align_up(sizeof(int) * (size_t)a.n));
  if (tmp + 2 * align_up(sizeof(int) * (size_t)a.n) > a.ws_bytes) return -2;

  hipError_t e = rocprim::radix_sort_pairs(a.ws, sort_bytes, a.keys, a.skeys, a.iota, a.perm, a.n, 0,
                                           a.end_bit, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(mark_heads_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, st, a.skeys, a.n, heads);
  e = rocprim::inclusive_scan(a.ws, scan_bytes, heads, incl, (size_t)a.n, rocprim::plus<int>(), st);
  if (e != hipSuccess) return (int)e;
  EmitArgs em{a.n, a.skeys, a.perm, incl, a.uniq, a.seg_start, a.num_unique, a.inv,
              a.ex_of_occ, a.sorted_ex, a.vals, a.sorted_x};
  hipLaunchKernelGGL(rle_emit_kernel, dim3(grid_for(a.n)), dim3(kBlock), 0, st, em);
  return (int)hipGetLastError();
}

// chunk_start must hold n+1 ints; chunk_seg n ints.
int launch_chunk_plan(int n, const int* num_unique, const int* seg_start, int CH, int* chunk_start,
                      int* chunk_seg, int* num_chunks, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) {
    (void)hipMemsetAsync(num_chunks, 0, sizeof(int), st);
    (void)hipMemsetAsync(chunk_start, 0, sizeof(int), st);
    return (int)hipGetLastError();
  }
  size_t scan_bytes = 0;
  (void)rocprim::inclusive_scan((void*)nullptr, scan_bytes, (const int*)nullptr, (int*)nullptr, (size_t)n,
                          rocprim::plus<int>(), st);
  const size_t tmp = align_up(scan_bytes);
  int* counts = reinterpret_cast<int*>(static_cast<char*>(ws) + tmp);
  if (tmp + align_up(sizeof(int) * (size_t)n) > ws_bytes) return -2;
  hipLaunchKernelGGL(chunk_count_kernel, dim3(grid_for(n)), dim3(kBlock), 0, st, n, num_unique, seg_start, CH,
                     counts);
  (void)hipMemsetAsync(chunk_start, 0, sizeof(int), st);
  hipError_t e = rocprim::inclusive_scan(ws, scan_bytes, counts, chunk_start + 1, (size_t)n,
                                         rocprim::plus<int>(), st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(chunk_emit_kernel, dim3(grid_for(n)), dim3(kBlock), 0, st, n, num_unique, chunk_start,
                     chunk_seg, num_chunks);
  return (int)hipGetLastError();
}

}  // namespace fm
