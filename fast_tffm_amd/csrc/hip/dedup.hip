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
//   2. run-length encoding in two passes over the sorted keys: rle_count_kernel
//      flags "segment head" (key differs from its left neighbour) and "chunk
//      start" (head, or position % CH == 0) per 2048-element tile and stores
//      the tile's two counts; rle_emit_kernel re-derives the flags, sums the
//      counts of the tiles before it (<= a few thousand 8-byte words, L2
//      resident: no scan kernel, no cross-workgroup wait), block-scans, and
//      writes the unique keys, segment starts, first chunk of each segment,
//      chunk starts, chunk->segment and the optional inverse map /
//      per-sorted-occurrence example index and value.  (A one-pass version with
//      a decoupled look-back over published tile counts measured 55-131 us next
//      to the backward vs ~30 here: the first ~2000 tiles start together and
//      walk back serially over each other's status words, profiles/r3.)
// Chunks cut every segment at CH-aligned sorted positions, so no chunk is
// longer than CH and a hot id (tens of thousands of occurrences in Criteo's
// low-cardinality fields) is spread over many lane groups in the backward.
#include "fm_common.h"
#include <rocprim/rocprim.hpp>
#include <string>

namespace fm {

constexpr int kRleItems = 8;                     // elements per thread
constexpr int kRleTile = kBlock * kRleItems;     // 2048 elements per tile
constexpr int kMaxTiles = 1 << 20;               // tile-count words per call (n < 2^31)

struct RleArgs {
  int n, CH, ntiles;              // n: occurrences, ntiles over n
  const uint32_t* skeys;          // sorted keys
  const int* spay;                // sorted payload (occurrence or example index)
  int ex_shift;                   // > 0: payload / ex_of_occ hold packed codes (example << ex_shift | slot)
  const int* offsets;             // [B+1] CSR offsets (packed codes -> occurrence index)
  unsigned long long* tile_cnt;   // [ntiles] heads << 32 | chunk starts (rle_count_kernel)
  uint32_t* uniq;                 // [n] unique keys (first U valid)
  int* seg_start;                 // [n+1]
  int* seg_chunk;                 // [n+1] first chunk of each segment
  int* chunk_start;               // [n+1]
  int* chunk_seg;                 // [n] segment id | kChunkFirst | kChunkSingle
  int* chunk_key;                 // [n] key of the chunk's segment
  int* counts;                    // device [8]: U, #chunks, #multi-chunk rows, -, bwd hot rows, -
  int* inv;                       // [n] occurrence -> segment (payload = occurrence)
  const int* ex_of_occ;           // [n] (payload = occurrence)
  int* sorted_ex;                 // [n] (payload = occurrence)
  const float* vals;              // [n] (payload = occurrence)
  float* sorted_x;                // [n] (payload = occurrence)
  const int* sort_err;            // in-tree sort's look-back error word (null: rocPRIM)
};

// v[q] = p[j0 + q] (fill outside [0, n)); two 16-byte loads when in range (j0 % 8 == 0).
template <typename T>
__device__ inline void load8(const T* p, int j0, int n, T (&v)[8], T fill) {
  if (j0 >= 0 && j0 + 8 <= n) {
    const uint4 x = *reinterpret_cast<const uint4*>(p + j0);
    const uint4 y = *reinterpret_cast<const uint4*>(p + j0 + 4);
    v[0] = (T)x.x; v[1] = (T)x.y; v[2] = (T)x.z; v[3] = (T)x.w;
    v[4] = (T)y.x; v[5] = (T)y.y; v[6] = (T)y.z; v[7] = (T)y.w;
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = (j0 + q >= 0 && j0 + q < n) ? p[j0 + q] : fill;
  }
}

// Flags of one thread's 8 consecutive sorted positions j0..j0+7.
//   head:   first occurrence of a key;
//   cstart: chunk boundary = head or CH-aligned position.
struct Rle8 {
  uint32_t k[8];
  bool hd[8], cs[8];
};

__device__ inline void rle_flags8(const RleArgs& a, int j0, Rle8& r) {
  constexpr uint32_t kNone = 0xffffffffu;  // keys are non-negative int32: never a key
  load8(a.skeys, j0, a.n, r.k, kNone);
  const uint32_t kp = (j0 > 0 && j0 <= a.n) ? a.skeys[j0 - 1] : kNone;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int j = j0 + q;
    const bool ok = j < a.n;
    r.hd[q] = ok && (j == 0 || r.k[q] != (q ? r.k[q - 1] : kp));
    r.cs[q] = r.hd[q] || (ok && j % a.CH == 0);
  }
}

// Block-wide exclusive scan of NC per-thread counts (segment heads, chunk
// starts).
template <int NC>
__device__ inline void block_excl_scan(const unsigned (&v)[NC], unsigned (&ex)[NC], unsigned (&tot)[NC]) {
  __shared__ unsigned sh[NC][kWavesPerBlock];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  unsigned inc[NC];  // inclusive wave scan
#pragma unroll
  for (int i = 0; i < NC; ++i) inc[i] = v[i];
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const unsigned up = __shfl_up(inc[i], o, kWave);
      if (lane >= o) inc[i] += up;
    }
  }
  if (lane == kWave - 1) {
#pragma unroll
    for (int i = 0; i < NC; ++i) sh[i][wv] = inc[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    unsigned b = 0, t = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) {
      if (w < wv) b += sh[i][w];
      t += sh[i][w];
    }
    ex[i] = b + inc[i] - v[i];
    tot[i] = t;
  }
  __syncthreads();
}

// Per tile: head and chunk-start counts.  Block 0 also zeroes the counts no later kernel of the
// chain writes (no memset launches).
__global__ __launch_bounds__(kBlock) void rle_count_kernel(RleArgs a) {
  const int tile = blockIdx.x;
  Rle8 r;
  rle_flags8(a, tile * kRleTile + threadIdx.x * kRleItems, r);
  unsigned v[2] = {0u, 0u}, ex[2], tot[2];
#pragma unroll
  for (int q = 0; q < kRleItems; ++q) {
    v[0] += r.hd[q];
    v[1] += r.cs[q];
  }
  block_excl_scan<2>(v, ex, tot);
  if (threadIdx.x == 0) {
    a.tile_cnt[tile] = ((unsigned long long)tot[0] << 32) | tot[1];
    if (tile == 0) {
      a.counts[3] = 0;
      a.counts[5] = a.counts[6] = 0;
      // the sort's verdict: counts[7] != 0 = this plan is invalid (DedupOut.sync raises), and the
      // sticky device word keeps it for the host's periodic check (check_device_errors)
      const int e = a.sort_err ? *a.sort_err : 0;
      a.counts[7] = e;
      if (e) atomicOr(&g_fm_dev_error, kDevErrSort);
    }
  }
}

__global__ __launch_bounds__(kBlock) void rle_emit_kernel(RleArgs a) {
  __shared__ unsigned s_pre[2];
  const int tile = blockIdx.x;
  const int last = a.n > 0 ? (a.n - 1) / kRleTile : 0;  // the last tile holding elements writes the totals
  if (tile > last) return;
  // global offsets: the counts of tiles 0..tile-1 (written by rle_count_kernel)
  unsigned pv[2] = {0u, 0u}, pex[2], ptot[2];
  for (int i = threadIdx.x; i < tile; i += kBlock) {
    const unsigned long long w = a.tile_cnt[i];
    pv[0] += (unsigned)(w >> 32);
    pv[1] += (unsigned)w;
  }
  block_excl_scan<2>(pv, pex, ptot);
  const int j0 = tile * kRleTile + threadIdx.x * kRleItems;
  Rle8 r;
  rle_flags8(a, j0, r);
  unsigned v[2] = {0u, 0u}, ex[2], tot[2];
#pragma unroll
  for (int q = 0; q < kRleItems; ++q) {
    v[0] += r.hd[q];
    v[1] += r.cs[q];
  }
  block_excl_scan<2>(v, ex, tot);
  if (threadIdx.x == 0) {
    s_pre[0] = ptot[0];
    s_pre[1] = ptot[1];
    if (tile == last) {  // totals, sentinels; the backward's two counters start at 0
      const unsigned U = ptot[0] + tot[0], C = ptot[1] + tot[1];
      a.counts[0] = (int)U;
      a.counts[1] = (int)C;
      a.counts[2] = 0;
      a.counts[4] = 0;
      a.seg_start[U] = a.n;
      a.seg_chunk[U] = (int)C;
      a.chunk_start[C] = a.n;
    }
  }
  __syncthreads();
  // running (inclusive) segment / chunk ids of this thread's elements
  int s = (int)(s_pre[0] + ex[0]) - 1;
  int ch = (int)(s_pre[1] + ex[1]) - 1;
  int sq[kRleItems];
#pragma unroll
  for (int q = 0; q < kRleItems; ++q) {
    const int j = j0 + q;
    s += r.hd[q];
    ch += r.cs[q];
    sq[q] = s;
    if (j >= a.n) continue;
    if (r.hd[q]) {
      a.uniq[s] = r.k[q];
      a.seg_start[s] = j;
      a.seg_chunk[s] = ch;
    }
    if (r.cs[q]) {
      // a head chunk is the row's only one iff the row ends before the next CH-aligned cut
      const int b = (j / a.CH + 1) * a.CH;
      const bool single = r.hd[q] && (b >= a.n || a.skeys[b] != r.k[q]);
      a.chunk_start[ch] = j;
      a.chunk_seg[ch] = (int)((unsigned)s | (r.hd[q] ? (unsigned)kChunkFirst : 0u) | (single ? kChunkSingle : 0u));
      a.chunk_key[ch] = (int)r.k[q];
    }
  }
  const bool need_all = a.inv || a.sorted_ex || a.sorted_x;
  if (need_all) {
    // payload = occurrence (or packed code): all 8 random gathers / scatters of the thread in flight at once
    int p[kRleItems];
    load8(a.spay, j0, a.n, p, 0);
    if (a.ex_shift > 0) {  // packed code -> occurrence index (offsets is small and L2-resident)
      const int mask = (1 << a.ex_shift) - 1;
#pragma unroll
      for (int q = 0; q < kRleItems; ++q)
        p[q] = j0 + q < a.n ? a.offsets[p[q] >> a.ex_shift] + (p[q] & mask) : 0;
    }
    int exv[kRleItems];
    float xv[kRleItems];
#pragma unroll
    for (int q = 0; q < kRleItems; ++q) {
      const bool ok = j0 + q < a.n;
      exv[q] = (a.sorted_ex && ok) ? a.ex_of_occ[p[q]] : 0;
      xv[q] = (a.sorted_x && ok) ? a.vals[p[q]] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kRleItems; ++q) {
      if (j0 + q >= a.n) break;
      if (a.inv) a.inv[p[q]] = sq[q];
      if (a.sorted_ex) a.sorted_ex[j0 + q] = exv[q];
      if (a.sorted_x) a.sorted_x[j0 + q] = xv[q];
    }
  }
}

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// Onesweep configuration measured on MI355X for 5.1M (key, int32) pairs with
// 27-bit keys (tools/bench_sort.hip, interleaved rounds): rocPRIM's default
// 260 us; 1024x8 "match" ranking with 8-bit digits 203 us, 9-bit 150 us,
// 10-bit 164 us, 11-bit 273 us.  The digit width is chosen so that the key bits
// are covered in the fewest passes of 9-10 bits.
template <unsigned BITS>
using OnesweepCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, BITS,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

static int digit_bits(int key_bits) {
  if (key_bits <= 18) return 9;   // 2 passes
  if (key_bits <= 20) return 10;  // 2 passes
  if (key_bits <= 27) return 9;   // 3 passes
  if (key_bits <= 30) return 10;  // 3 passes
  return 8;                       // 4 passes
}

template <unsigned BITS>
static hipError_t sort_pairs_bits(void* tmp, size_t& bytes, const uint32_t* k, uint32_t* ko, const int* v, int* vo,
                                  int n, int end_bit, hipStream_t st) {
  return rocprim::radix_sort_pairs<OnesweepCfg<BITS>>(tmp, bytes, k, ko, v, vo, n, 0, end_bit, st);
}

static hipError_t sort_pairs(void* tmp, size_t& bytes, const uint32_t* k, uint32_t* ko, const int* v, int* vo,
                             int n, int end_bit, hipStream_t st) {
  switch (digit_bits(end_bit)) {
    case 10: return sort_pairs_bits<10>(tmp, bytes, k, ko, v, vo, n, end_bit, st);
    case 8: return sort_pairs_bits<8>(tmp, bytes, k, ko, v, vo, n, end_bit, st);
    default: return sort_pairs_bits<9>(tmp, bytes, k, ko, v, vo, n, end_bit, st);
  }
}

static size_t sort_temp_bytes(int n, hipStream_t st) {
  size_t best = 0;
  for (int bits : {16, 20, 27, 30, 32}) {  // the largest requirement over all dispatch targets
    size_t b = 0;
    (void)sort_pairs(nullptr, b, nullptr, nullptr, nullptr, nullptr, n, bits, st);
    if (b > best) best = b;
  }
  return align_up(best);
}

#include "radix_sort.hip"

// Sort backend: the in-tree onesweep radix sort (radix_sort.hip, default) or rocPRIM's onesweep
// (FM_SORT=rocprim); bitwise the same stable order (profiles/r5/sort_ab.txt)
static int g_sort_algo = -1;
static bool sort_in_tree() {
  if (g_sort_algo < 0) {
    const char* e = getenv("FM_SORT");
    g_sort_algo = (e && std::string(e) == "rocprim") ? 0 : 1;
  }
  return g_sort_algo == 1;
}
void set_sort_algo(int in_tree) { g_sort_algo = in_tree ? 1 : 0; }
int sort_algo() { return sort_in_tree() ? 1 : 0; }

// Workspace layout: [sort temp (the larger of the two backends') | pad (8 B), tile_cnt[ntiles]]
static size_t lb_bytes(int ntiles) { return 8 + 8 * (size_t)ntiles; }

static size_t sort_ws_bytes(int n, hipStream_t st) {
  const size_t a = sort_temp_bytes(n, st), b = align_up(radix_sort_ws_bytes(n));
  return a > b ? a : b;
}

size_t dedup_workspace_bytes(int n) {
  if (n <= 0) return 256;
  const size_t ntiles = ((size_t)n + kRleTile - 1) / kRleTile;
  return sort_ws_bytes(n, 0) + align_up(lb_bytes((int)ntiles)) + 256;
}

struct DedupArgs {
  int n;                   // occurrences
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
  int* chunk_key;          // [n]
  int* counts;             // device [4]
  int* inv;                // nullable
  const int* ex_of_occ;    // nullable
  int* sorted_ex;          // nullable
  const float* vals;       // nullable
  float* sorted_x;         // nullable
  int payload_is_ex;       // payload carries the example index (sorted payload == sorted example)
  int ex_shift;            // > 0: the payload is the packed code (example << ex_shift | slot), see csr_rows
  const int* offsets;      // [B+1] (ex_shift > 0)
  void* ws;
  size_t ws_bytes;
  // fused producers (in-tree sort: inside its histogram / first pass; rocPRIM: the separate kernels first)
  const int* ids = nullptr;  // non-null: keys = sharded keys of ids (kW, kRps), written to the keys array
  int kW = 1, kRps = 0;
  int gen_codes = 0;         // payload = packed occurrence codes of the CSR offsets (written to payload)
  int B = 0;                 // examples (gen_codes)
};

int launch_shard_keys(int n, const int* ids, int W, int Rps, int* keys, hipStream_t st);  // shard.hip

// ---------------------------------------------------------------------------
// Segment index (key -> segment id without an inverse map).  The row-sharded forward reads
// each occurrence's wire row by its segment id.  The dedup's inverse map delivers that as one
// random 4-byte scatter per occurrence (5.1M per Criteo-shaped batch: rle_tile_emit 24 ->
// 112 us, the local step +85 us when it is forced on, profiles/r2/inv_cost.txt).  Instead a
// bucket index over the sorted unique keys is built -- idx[b] = first segment whose key >>
// shift >= b, nb + 1 entries, every one written once per batch by the segment that starts it
// (no clear, no atomics) -- and the forward finds a key's segment from idx[b], idx[b + 1] and,
// only when the bucket holds several keys, a short scan of the sorted keys.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void seg_index_kernel(int n_max, const uint32_t* uniq, const int* counts, int shift,
                                                           int nb, int* idx) {
  const int U = min(counts[0], n_max);
  const int tid = blockIdx.x * kBlock + threadIdx.x, nth = gridDim.x * kBlock;
  for (int s = tid; s < U; s += nth) {  // buckets (previous key's bucket, this key's bucket]
    const int lo = s == 0 ? 0 : (int)(uniq[s - 1] >> shift) + 1;
    const int hi = (int)(uniq[s] >> shift);
    for (int b = lo; b <= hi; ++b) idx[b] = s;
  }
  // buckets after the last key (keys rarely fill the whole 2^key_bits range: spread over the grid)
  const int tail0 = U > 0 ? (int)(uniq[U - 1] >> shift) + 1 : 0;
  for (int b = tail0 + tid; b <= nb; b += nth) idx[b] = U;
}

int launch_seg_index(int n_max, const uint32_t* uniq, const int* counts, int shift, int nb, int* idx, hipStream_t st) {
  if (n_max < 0 || nb < 1 || shift < 0 || shift > 31) return -1;
  hipLaunchKernelGGL(seg_index_kernel, dim3(fill_grid(n_max + 1, kBlock, 2048)), dim3(kBlock), 0, st, n_max, uniq,
                     counts, shift, nb, idx);
  return (int)hipGetLastError();
}

int launch_dedup(const DedupArgs& a, hipStream_t st) {
  // counts[0..2] = U, #chunks, #multi-chunk rows; counts[4] = the backward's
  // hot-row count: both backward counters start at 0 here, on the dedup's stream (off the
  // compute stream's critical path), written by the RLE kernels
  if (a.n <= 0) {
    (void)hipMemsetAsync(a.counts, 0, 8 * sizeof(int), st);
    (void)hipMemsetAsync(a.seg_start, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.seg_chunk, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.chunk_start, 0, sizeof(int), st);
    return (int)hipGetLastError();
  }
  const int ntiles = (a.n + kRleTile - 1) / kRleTile;
  if (ntiles > kMaxTiles) return -3;
  const size_t tmp = sort_ws_bytes(a.n, st);
  char* base = static_cast<char*>(a.ws);
  char* lb = base + tmp;
  if (tmp + align_up(lb_bytes(ntiles)) > a.ws_bytes) return -2;

  if (a.gen_codes && (!a.offsets || a.B < 1)) return -4;
  if (sort_in_tree()) {
    RsSrc src;
    src.ids = a.ids;
    src.W = a.kW;
    src.Rps = a.kRps;
    if (a.gen_codes) {
      src.offsets = a.offsets;
      src.B = a.B;
      src.code_shift = a.ex_shift;
    }
    const int e = launch_radix_sort(a.keys, a.payload, a.skeys, a.spay, a.n, a.end_bit, a.ws, tmp, st, src);
    if (e != 0) return e;
  } else {
    if (a.ids) {
      const int e = launch_shard_keys(a.n, a.ids, a.kW, a.kRps, const_cast<int*>(reinterpret_cast<const int*>(a.keys)), st);
      if (e != 0) return e;
    }
    if (a.gen_codes) {
      const int e = launch_csr_rows(a.B, a.offsets, const_cast<int*>(a.payload), a.ex_shift, st);
      if (e != 0) return e;
    }
    size_t sort_bytes = tmp;
    const hipError_t e = sort_pairs(a.ws, sort_bytes, a.keys, a.skeys, a.payload, a.spay, a.n, a.end_bit, st);
    if (e != hipSuccess) return (int)e;
  }
  RleArgs r{a.n, a.CH, ntiles, a.skeys, a.spay, a.ex_shift,
            a.offsets, reinterpret_cast<unsigned long long*>(lb + 8), a.uniq, a.seg_start,
            a.seg_chunk, a.chunk_start, a.chunk_seg, a.chunk_key, a.counts, a.inv, a.ex_of_occ, a.sorted_ex,
            a.vals, a.sorted_x, sort_in_tree() ? radix_sort_error(a.ws, a.n) : nullptr};
  hipLaunchKernelGGL(rle_count_kernel, dim3(ntiles), dim3(kBlock), 0, st, r);
  hipLaunchKernelGGL(rle_emit_kernel, dim3(ntiles), dim3(kBlock), 0, st, r);
  return (int)hipGetLastError();
}

}  // namespace fm
