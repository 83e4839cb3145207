// In-tree stable LSD radix sort of (uint32 key, int32 value) pairs for the dedup chain
// (reference tf.unique, tffm/fm_model.py:72-73, is a hash table; this framework groups a batch's
// occurrences by sorting them: dedup.hip).
//
// Per digit pass (8 or 9 bits, 2-4 passes over the key bits in use) three kernels, no global
// atomics and no spin-waits.  (A onesweep form -- one histogram kernel, one kernel per pass with a
// decoupled look-back reading 64 predecessor tiles per load -- measured 479 us for 24-bit keys
// against this form's 161 and rocPRIM's 148: the ~600 tiles that start together resolve their
// prefixes over tile / 64 round trips per digit batch; profiles/r5/sort_ab.txt.)
//   count: each 8192-element tile counts its digits -> cnt[tile][digit] (one coalesced row);
//   scan:  per digit, exclusive prefixes over the tiles (in place) and the digit's total;
//   scatter: each tile re-ranks its elements (stable), scans the digit totals into digit bases,
//          stages the tile in LDS in digit order and writes every element to
//          base[d] + prefix[d][tile] + its rank among the tile's digit-d elements; consecutive
//          threads write consecutive positions of one digit's run (coalesced stores).
// Ranking is wave-local and order-preserving: a wave owns 512 consecutive elements, slot i of lane
// l is element 64 i + l, and for each slot the lanes holding the same digit are found by one
// ballot per digit bit ("match"); the lowest such lane adds the group's size to the wave's digit
// counter in LDS, every lane's rank is the counter before it plus its position in the group.  The
// tile's digit d elements are ordered (wave, slot, lane) = element order, so the sort is stable
// and its output is the unique stable order -- bitwise what any stable sort produces.
// Memory per pass: keys read twice (count + scatter), values once, both written once.
// (Included by module.hip inside namespace fm.)

constexpr int kRsThreads = 512;                   // threads per tile block
constexpr int kRsWaves = kRsThreads / kWave;      // 8
constexpr int kRsItems = 16;                      // elements per thread
constexpr int kRsWaveElems = kRsItems * kWave;    // 1024 consecutive elements per wave
constexpr int kRsTile = kRsThreads * kRsItems;    // 8192: digit runs of 16-32 elements per tile
constexpr int kRsMaxDigits = 512;                 // 9-bit digits at most

struct RsPass {
  int n, ntiles, shift;
  uint32_t dmask;  // digit bits of this pass (the last pass stops at the sort's end bit)
  const uint32_t* kin;
  const int* vin;
  uint32_t* kout;
  int* vout;
  unsigned* cnt;   // [ntiles][D] tile digit counts -> exclusive prefixes over tiles
  unsigned* tot;   // [D] digit totals
};

__device__ inline uint64_t rs_lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// Lanes (among `live`) whose digit equals this lane's.
template <int DB>
__device__ inline uint64_t rs_match(uint32_t d, uint64_t live) {
  uint64_t m = live;
#pragma unroll
  for (int b = 0; b < DB; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

// Wave-local stable ranking of the wave's 1024 elements: wcnt (this wave's D counters in LDS,
// zeroed by the caller) ends as the wave's digit counts; rank[i] = position of slot i's element
// among the wave's elements of its digit.
#ifndef FM_RS_RANK_ATOMIC
#define FM_RS_RANK_ATOMIC 1
#endif
template <int DB>
__device__ inline void rs_rank_wave(const uint32_t (&dig)[kRsItems], const bool (&ok)[kRsItems], unsigned* wcnt,
                                    unsigned (&rank)[kRsItems]) {
#if FM_RS_RANK_ATOMIC
  // ds_add_rtn_u32 per element: the LDS serves the lanes of one instruction that hit the same counter
  // in ascending lane order (checked bitwise against a stable sort: tests/test_kernels.py, bench_fmsort)
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) rank[i] = ok[i] ? atomicAdd(&wcnt[dig[i]], 1u) : 0u;
#else
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t lt = rs_lanemask_lt(lane);
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) {
    const uint64_t live = __ballot(ok[i]);
    const uint64_t peers = rs_match<DB>(dig[i], live);
    const unsigned below = (unsigned)__popcll(peers & lt);
    unsigned base = 0;
    if (ok[i]) base = wcnt[dig[i]];
    rank[i] = base + below;
    if (ok[i] && below == 0) wcnt[dig[i]] = base + (unsigned)__popcll(peers);
  }
#endif
}

template <int DB>
__device__ inline void rs_load(const RsPass& p, int tile, uint32_t (&key)[kRsItems], uint32_t (&dig)[kRsItems],
                               bool (&ok)[kRsItems]) {
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  const int e0 = tile * kRsTile + wv * kRsWaveElems + lane;
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) {
    const int e = e0 + i * kWave;
    ok[i] = e < p.n;
    key[i] = ok[i] ? p.kin[e] : 0u;
    dig[i] = (key[i] >> p.shift) & p.dmask;
  }
}

// 1. tile digit counts (LDS atomics into per-wave counters: no ranking needed)
template <int DB>
__global__ __launch_bounds__(kRsThreads) void rs_count_kernel(RsPass p) {
  constexpr int D = 1 << DB;
  __shared__ unsigned wc[kRsWaves][D];
  const int wv = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < kRsWaves * D; t += kRsThreads) (&wc[0][0])[t] = 0u;
  __syncthreads();
  const int tile = blockIdx.x;
  uint32_t key[kRsItems], dig[kRsItems];
  bool ok[kRsItems];
  rs_load<DB>(p, tile, key, dig, ok);
#pragma unroll
  for (int i = 0; i < kRsItems; ++i)
    if (ok[i]) atomicAdd(&wc[wv][dig[i]], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += kRsThreads) {
    unsigned s = 0;
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) s += wc[w][d];
    p.cnt[(size_t)tile * D + d] = s;
  }
}

// 2. per digit: exclusive prefix over tiles, in place, and the digit's total.  A block of 1024
// threads takes 64 digits: thread (group g, digit lane dl) sums tiles [g * per, (g + 1) * per) of
// its digit (rows of 64 consecutive digits: 256-byte loads), the 16 group sums are scanned in LDS,
// then each thread rewrites its range as prefixes.
constexpr int kRsScanThreads = 1024, kRsScanDigits = 64, kRsScanGroups = kRsScanThreads / kRsScanDigits;
template <int DB>
__global__ __launch_bounds__(kRsScanThreads) void rs_scan_kernel(RsPass p) {
  constexpr int D = 1 << DB;
  __shared__ unsigned gs[kRsScanGroups][kRsScanDigits];
  const int dl = threadIdx.x % kRsScanDigits, g = threadIdx.x / kRsScanDigits;
  const int d = blockIdx.x * kRsScanDigits + dl;
  const int per = (p.ntiles + kRsScanGroups - 1) / kRsScanGroups;
  const int t0 = g * per, t1 = min(p.ntiles, t0 + per);
  unsigned s = 0;
#pragma unroll 8
  for (int t = t0; t < t1; ++t) s += p.cnt[(size_t)t * D + d];
  gs[g][dl] = s;
  __syncthreads();
  unsigned base = 0;
  for (int h = 0; h < g; ++h) base += gs[h][dl];
  if (g == kRsScanGroups - 1) p.tot[d] = base + s;
#pragma unroll 8
  for (int t = t0; t < t1; ++t) {
    unsigned* c = p.cnt + (size_t)t * D + d;
    const unsigned v = *c;
    *c = base;
    base += v;
  }
}

// Block-wide exclusive scan of one value per thread (kRsThreads threads); returns the total too.
__device__ inline unsigned rs_block_excl(unsigned v, unsigned* sh /*[kRsWaves]*/, unsigned& total) {
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  unsigned inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned up = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += up;
  }
  if (lane == kWave - 1) sh[wv] = inc;
  __syncthreads();
  unsigned b = 0, t = 0;
#pragma unroll
  for (int w = 0; w < kRsWaves; ++w) {
    const unsigned s = sh[w];
    if (w < wv) b += s;
    t += s;
  }
  __syncthreads();
  total = t;
  return b + inc - v;
}

// 3. stable rank + scatter of one tile
template <int DB>
__global__ __launch_bounds__(kRsThreads) void rs_scatter_kernel(RsPass p) {
  constexpr int D = 1 << DB;
  __shared__ unsigned wc[kRsWaves][D];   // wave digit counts -> tile positions of the waves' digit runs
  __shared__ int gofs[D];                // global position of the tile's digit-d run minus its tile position
  __shared__ uint32_t stage[kRsTile];    // the tile in digit order: keys, then values
  __shared__ unsigned sh[kRsWaves];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
  const int tile = blockIdx.x;
  for (int t = threadIdx.x; t < kRsWaves * D; t += kRsThreads) (&wc[0][0])[t] = 0u;
  __syncthreads();
  uint32_t key[kRsItems], dig[kRsItems];
  bool ok[kRsItems];
  rs_load<DB>(p, tile, key, dig, ok);
  int val[kRsItems];
  const int e0 = tile * kRsTile + wv * kRsWaveElems + lane;
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) val[i] = ok[i] ? p.vin[e0 + i * kWave] : 0;
  unsigned rank[kRsItems];
  rs_rank_wave<DB>(dig, ok, wc[wv], rank);
  __syncthreads();
  // per digit: wave offsets (exclusive over waves) and the tile's count; digit bases from the totals
  constexpr int DPT = (D + kRsThreads - 1) / kRsThreads;  // digits per thread (1)
  unsigned tcount[DPT], gtot[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int d = threadIdx.x + j * kRsThreads;
    unsigned s = 0;
    if (d < D) {
#pragma unroll
      for (int w = 0; w < kRsWaves; ++w) {
        const unsigned c = wc[w][d];
        wc[w][d] = s;
        s += c;
      }
    }
    tcount[j] = s;
    gtot[j] = d < D ? p.tot[d] : 0u;
  }
  static_assert(DPT == 1, "one digit per thread");
  unsigned ttot, gsum;
  const unsigned tstart = rs_block_excl(tcount[0], sh, ttot);   // tile-local start of digit d's run
  const unsigned gbase = rs_block_excl(gtot[0], sh, gsum);      // global start of digit d
  if (threadIdx.x < D)
    gofs[threadIdx.x] = (int)(gbase + p.cnt[(size_t)tile * D + threadIdx.x]) - (int)tstart;
  // tile-local positions: the tile start of the digit's run is needed per element -> stash it in wc
  // (wave offset + run start) so one LDS read gives the full local position
  __syncthreads();
  if (threadIdx.x < D) {
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) wc[w][threadIdx.x] += tstart;
  }
  __syncthreads();
  unsigned pos[kRsItems];
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) {
    pos[i] = wc[wv][dig[i]] + rank[i];
    if (ok[i]) stage[pos[i]] = key[i];
  }
  __syncthreads();
  const int tn = min(kRsTile, p.n - tile * kRsTile);
  int gpos[kRsItems];
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) {
    const int j = threadIdx.x + i * kRsThreads;
    gpos[i] = -1;
    if (j < tn) {
      const uint32_t k = stage[j];
      gpos[i] = gofs[(k >> p.shift) & p.dmask] + j;
      p.kout[gpos[i]] = k;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kRsItems; ++i)
    if (ok[i]) stage[pos[i]] = (uint32_t)val[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) {
    const int j = threadIdx.x + i * kRsThreads;
    if (gpos[i] >= 0) p.vout[gpos[i]] = (int)stage[j];
  }
}

// Passes and digit width for the key bits in use: the fewest passes of 8-9 bits.
static inline void rs_plan(int end_bit, int& passes, int& db) {
  end_bit = end_bit < 1 ? 1 : (end_bit > 32 ? 32 : end_bit);
  passes = (end_bit + 8) / 9;            // 9-bit digits cover the most bits per pass
  if (passes * 9 < end_bit) ++passes;
  db = (end_bit + passes - 1) / passes;  // <= 9
  if (db < 8) db = 8;                    // (8-bit digits when they need no extra pass)
}

static inline size_t rs_align(size_t x) { return (x + 255) & ~size_t(255); }

// Workspace: [alt keys n][alt values n][cnt ntiles x D][tot D]
size_t radix_sort_ws_bytes(int n) {
  if (n <= 0) return 256;
  const size_t ntiles = ((size_t)n + kRsTile - 1) / kRsTile;
  return rs_align(4 * (size_t)n) * 2 + rs_align(4 * (size_t)kRsMaxDigits * ntiles) + rs_align(4 * kRsMaxDigits);
}

template <int DB>
static void rs_launch_pass(const RsPass& p, hipStream_t st) {
  hipLaunchKernelGGL(rs_count_kernel<DB>, dim3(p.ntiles), dim3(kRsThreads), 0, st, p);
  hipLaunchKernelGGL(rs_scan_kernel<DB>, dim3((1 << DB) / kRsScanDigits), dim3(kRsScanThreads), 0, st, p);
  hipLaunchKernelGGL(rs_scatter_kernel<DB>, dim3(p.ntiles), dim3(kRsThreads), 0, st, p);
}

// Stable sort of (keys[i], vals[i]) by keys' bits [0, end_bit) into (kout, vout); keys / vals are
// not modified.  0 or a hip error code; -2: workspace too small.
int launch_radix_sort(const uint32_t* keys, const int* vals, uint32_t* kout, int* vout, int n, int end_bit,
                      void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  if (ws_bytes < radix_sort_ws_bytes(n)) return -2;
  end_bit = end_bit < 1 ? 1 : (end_bit > 32 ? 32 : end_bit);
  int passes, db;
  rs_plan(end_bit, passes, db);
  const int ntiles = (n + kRsTile - 1) / kRsTile;
  char* b = static_cast<char*>(ws);
  uint32_t* alt_k = reinterpret_cast<uint32_t*>(b);
  int* alt_v = reinterpret_cast<int*>(b + rs_align(4 * (size_t)n));
  unsigned* cnt = reinterpret_cast<unsigned*>(b + 2 * rs_align(4 * (size_t)n));
  unsigned* tot = reinterpret_cast<unsigned*>(b + 2 * rs_align(4 * (size_t)n) + rs_align(4 * (size_t)kRsMaxDigits * ntiles));
  const uint32_t* kin = keys;
  const int* vin = vals;
  for (int i = 0; i < passes; ++i) {
    // the last pass writes the output, the one before it the alternate buffers, and so on
    const bool to_out = ((passes - 1 - i) % 2) == 0;
    const int shift = i * db, bits = end_bit - shift < db ? end_bit - shift : db;
    const uint32_t dmask = bits >= 32 ? 0xffffffffu : (1u << bits) - 1u;
    RsPass p{n, ntiles, shift, dmask, kin, vin, to_out ? kout : alt_k, to_out ? vout : alt_v, cnt, tot};
    if (db == 9) rs_launch_pass<9>(p, st);
    else rs_launch_pass<8>(p, st);
    kin = p.kout;
    vin = p.vout;
  }
  return (int)hipGetLastError();
}
