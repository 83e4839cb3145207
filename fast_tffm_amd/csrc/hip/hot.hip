// Hot rows of the local step: the occurrences of a small set of very frequent table rows leave
// the sort-based dedup and the occurrence-gather backward; their gradient comes from the
// dense-row GEMM on the matrix cores instead (fm_bwd.hip fm_bwd_dense_kernel, counts written
// by the forward).
//
// A Criteo-shaped batch spends most of its occurrences on the values of the low-cardinality
// fields: the 256 most frequent rows hold ~47% of them (profiles/r2/hot_row_knockout.txt).  In
// the dedup they are sorted element by element like every cold occurrence (the onesweep radix
// sort's cost is per element) and in the backward they are long runs of r1 gathers.  Here the
// dedup input is filtered first -- an order-preserving compaction of (key, occurrence code)
// over the batch's CSR, by example groups of 64:
//   hot_count_kernel: per group, the number of occurrences whose row is NOT hot;
//   hot_emit_kernel:  per group, the sum of the counts before it (<= B / 64 L2-resident words,
//                     read by the whole wave: no scan kernel), then each kept occurrence's key
//                     and packed code (example << slot_bits | slot, as csr_rows) at its
//                     compacted position; the last group writes the kept total.
// Hot membership: an LDS open-addressing table of the <= kMaxDense keys per workgroup (the
// forward's dense counting uses the same table shape).  Order is kept, so the sort sees exactly
// the non-hot subsequence of the usual input and the plan is deterministic.
#include "fm_common.h"

namespace fm {

struct HotFilterArgs {
  int B;
  const int* offsets;       // [B + 1]
  const int* ids;           // [nnz] table rows
  const int* hot;           // [kMaxDense] hot row keys
  const int* hot_n;         // device scalar: number of hot keys (<= kMaxDense)
  int slot_bits;
  int* gcnt;                // [ceil(B / 64)] kept occurrences per example group
  int* keys_out;            // [nnz] kept keys, CSR order
  int* codes_out;           // [nnz] their packed occurrence codes
  int* n_out;               // device scalar: kept total
};

__device__ inline void hot_table_build(const HotFilterArgs& a, int* hkey) {
  const int nh = min(*a.hot_n, kMaxDense);
  for (int k = threadIdx.x; k < kDenseHash; k += kBlock) hkey[k] = -1;
  __syncthreads();
  for (int h = threadIdx.x; h < nh; h += kBlock) {
    const int key = a.hot[h];
    int slot = dense_hash(key);
    while (atomicCAS(&hkey[slot], -1, key) != -1) slot = (slot + 1) & (kDenseHash - 1);
  }
  __syncthreads();
}

__device__ inline bool hot_member(const int* hkey, int key) {
  int slot = dense_hash(key);
  for (int probe = 0; probe < kDenseHash; ++probe) {
    const int k = hkey[slot];
    if (k == key) return true;
    if (k < 0) return false;
    slot = (slot + 1) & (kDenseHash - 1);
  }
  return false;
}

__global__ __launch_bounds__(kBlock) void hot_count_kernel(HotFilterArgs a) {
  __shared__ int hkey[kDenseHash];
  hot_table_build(a, hkey);
  const int lane = threadIdx.x & (kWave - 1);
  const int ngroups = (a.B + kWave - 1) / kWave;
  const int nwaves = gridDim.x * kWavesPerBlock;
  for (int g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
    const int i0 = g * kWave;
    const int s = a.offsets[i0], e = a.offsets[min(a.B, i0 + kWave)];
    int kept = 0;
    for (int base = s; base < e; base += kWave) {
      const int p = base + lane;
      const bool keep = p < e && !hot_member(hkey, a.ids[p]);
      kept += __popcll(__ballot(keep));
    }
    if (lane == 0) a.gcnt[g] = kept;
  }
}

__global__ __launch_bounds__(kBlock) void hot_emit_kernel(HotFilterArgs a) {
  __shared__ int hkey[kDenseHash];
  hot_table_build(a, hkey);
  const int lane = threadIdx.x & (kWave - 1);
  const int ngroups = (a.B + kWave - 1) / kWave;
  const int nwaves = gridDim.x * kWavesPerBlock;
  for (int g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
    int pre = 0;  // kept occurrences of the groups before g
    for (int j = lane; j < g; j += kWave) pre += a.gcnt[j];
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) pre += __shfl_xor(pre, o, kWave);
    const int i0 = g * kWave;
    const int n = min(kWave, a.B - i0);
    const int o = a.offsets[i0 + min(lane, n)];  // lanes >= n hold the group's end
    const int s = __shfl(o, 0);
    const int e = a.offsets[i0 + n];
    int pos = pre;
    for (int base = s; base < e; base += kWave) {  // wave-uniform trip count: every lane shuffles
      const int p = base + lane;
      int k = 0;  // example of occurrence p within the group (binary search over the offsets)
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1) {
        const int c = k + step;
        if (__shfl(o, c) <= p) k = c;
      }
      const int ok = __shfl(o, k);
      const int key = p < e ? a.ids[p] : 0;
      const bool keep = p < e && !hot_member(hkey, key);
      const uint64_t m = __ballot(keep);
      if (keep) {
        const int q = pos + __popcll(m & ((1ull << lane) - 1ull));
        a.keys_out[q] = key;
        const int ex = i0 + k;
        a.codes_out[q] = a.slot_bits > 0 ? (ex << a.slot_bits) | (p - ok) : ex;
      }
      pos += __popcll(m);
    }
    if (g == ngroups - 1 && lane == 0) *a.n_out = pos;
  }
}

int launch_hot_filter(const HotFilterArgs& a, hipStream_t st) {
  if (a.B <= 0) return (int)hipMemsetAsync(a.n_out, 0, sizeof(int), st);
  const int ngroups = (a.B + kWave - 1) / kWave;
  const int grid = fill_grid(ngroups, kWavesPerBlock, 4096);
  hipLaunchKernelGGL(hot_count_kernel, dim3(grid), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hot_emit_kernel, dim3(grid), dim3(kBlock), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm
