// In-tree stable LSD radix sort of (uint32 key, int32 value) pairs for the dedup chain
// (reference tf.unique, tffm/fm_model.py:72-73, is a hash table; this framework groups a batch's
// occurrences by sorting them: dedup.hip).  The default sort backend (FM_SORT=rocprim: rocPRIM's
// onesweep); profiles/r5/sort_ab.txt.
//
// Onesweep form, 8- or 9-bit digits, 2-4 passes over the key bits in use:
//   hist: one kernel counts every pass's digits at once (digit totals do not depend on the order;
//         per-wave LDS counters, 16-byte key loads) and zeroes the look-back state;
//   pass: ONE kernel per pass.  A tile (8192 elements, numbered in block start order, so it only
//         ever waits for tiles that are already running) ranks its elements, publishes its digit
//         counts, finds its exclusive prefix per digit by a decoupled look-back -- one thread per
//         digit, four predecessor tiles per load round, stopping at the nearest published inclusive
//         prefix -- publishes that, stages the tile in LDS in digit order and writes every element
//         to base[d] + prefix[d] + its position in the tile's digit-d run (coalesced runs).
// Ranking is wave-local and order-preserving: a wave owns 1024 consecutive elements, slot i of lane
// l is element 64 i + l, and rank = ds_add_rtn_u32 on the wave's digit counter in LDS (the LDS
// serves the lanes of one instruction that hit the same counter in ascending lane order), so a
// tile's digit-d elements keep element order: the sort is stable and its output is bitwise what any
// stable sort produces (tests/test_radix_sort_gpu.py, tools/bench_fmsort.hip against rocPRIM).
// Memory per pass: keys and values read once and written once (+ the keys once for all passes).
// Spins are bounded (an error word in the workspace instead of a hang); dedup.hip carries that word into
// the dedup's counts[7] and the module's sticky device error word (g_fm_dev_error), which the host
// checks (ops/kernels.py check_device_errors: bench, trainer log points, DedupOut.sync).
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
};

// Wave-local stable ranking of the wave's 1024 elements: wcnt (this wave's D counters in LDS,
// zeroed by the caller) ends as the wave's digit counts; rank[i] = position of slot i's element
// among the wave's elements of its digit.
template <int DB>
__device__ inline void rs_rank_wave(const uint32_t (&dig)[kRsItems], const bool (&ok)[kRsItems], unsigned* wcnt,
                                    unsigned (&rank)[kRsItems]) {
#pragma unroll
  for (int i = 0; i < kRsItems; ++i) rank[i] = ok[i] ? atomicAdd(&wcnt[dig[i]], 1u) : 0u;
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

// Block-wide exclusive scan of one 64-bit value per thread (kRsThreads threads): two 32-bit counts
// scanned at once (neither field's sum carries into the other).
__device__ inline uint64_t rs_block_excl(uint64_t v, uint64_t* sh /*[kRsWaves]*/) {
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint64_t up = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += up;
  }
  if (lane == kWave - 1) sh[wv] = inc;
  __syncthreads();
  uint64_t b = 0;
#pragma unroll
  for (int w = 0; w < kRsWaves; ++w)
    if (w < wv) b += sh[w];
  return b + inc - v;
}

constexpr unsigned kOsAgg = 1u << 30, kOsInc = 2u << 30, kOsCnt = (1u << 30) - 1u;
constexpr int kOsMaxPasses = 4;
constexpr int kOsHistBlocks = 1024;
constexpr int kOsSpinCap = 1 << 20;
// look-back spin bound of the pass kernels (set_sort_spin_cap; < 0: every tile but the first reports
// the error without waiting -- the tests' fault injection)
static int g_os_spin_cap = kOsSpinCap;
void set_sort_spin_cap(int cap) { g_os_spin_cap = cap; }
#ifndef FM_OS_LOOKBACK
#define FM_OS_LOOKBACK 4
#endif
constexpr int kOsLookback = FM_OS_LOOKBACK;  // predecessor tiles read per look-back round

// Fused producers of the sort's input (the dedup chain's two map kernels folded into the sort):
// keys from row ids under the sharded-key map, written by the histogram kernel, and the payload
// generated in the first pass as packed occurrence codes from the CSR offsets (csr_rows_kernel's
// output, fm_fwd.hip, without its 20 MB write + read).
struct RsSrc {
  const int* ids = nullptr;      // non-null: keys[e] = (ids[e] % W) * Rps + ids[e] / W (the keys array is the output)
  int W = 1, Rps = 0;
  const int* offsets = nullptr;  // non-null: vals[e] = example << code_shift | (e - offsets[example]); code_shift
  int B = 0, code_shift = 0;     //   0: the example (the vals array is not read)
};

struct OsSort {
  int n, passes, db, end_bit;
  const uint32_t* keys;
  const int* ids;     // RsSrc::ids (keys written to kw)
  uint32_t* kw;
  int W, Rps;
  unsigned* hist;     // [passes][D] digit totals (zeroed by the launcher's memset)
  unsigned* status;   // [passes][ntiles][D]
  int* ctr;           // [kOsMaxPasses + 1]: tile counters, [kOsMaxPasses] = error flag
  size_t nstatus;     // words of status to zero
};

__device__ inline uint32_t os_digit(uint32_t k, int shift, int db, int end_bit) {
  const int bits = min(db, end_bit - shift);
  return (k >> shift) & ((1u << bits) - 1u);
}

// digit totals of every pass, and the look-back state zeroed for the pass kernels that follow on the
// stream.  One 8192-key chunk per block (four 16-byte loads per thread in flight) and one LDS histogram
// per block (8 KB: the kernel runs beside the forward / backward, and per-wave copies -- 50 KB of LDS
// per block, 256 looping blocks -- took 154 us there against 11 us alone)
template <int DB>
__global__ __launch_bounds__(512) void os_hist_kernel(OsSort s) {
  constexpr int D = 1 << DB;
  __shared__ unsigned h[kOsMaxPasses * D];
  for (int t = threadIdx.x; t < s.passes * D; t += 512) h[t] = 0u;
  for (size_t t = (size_t)blockIdx.x * 512 + threadIdx.x; t < s.nstatus; t += (size_t)gridDim.x * 512) s.status[t] = 0u;
  if (blockIdx.x == 0 && threadIdx.x <= kOsMaxPasses) s.ctr[threadIdx.x] = 0;
  __syncthreads();
  auto count = [&](uint32_t k) {
#pragma unroll
    for (int q = 0; q < kOsMaxPasses; ++q)
      if (q < s.passes) atomicAdd(&h[q * D + os_digit(k, q * DB, DB, s.end_bit)], 1u);
  };
  auto key_of = [&](uint32_t id) { return (uint32_t)(((int)id % s.W) * s.Rps + (int)id / s.W); };
  constexpr int kChunk = 512 * 16;
  const void* in = s.ids ? static_cast<const void*>(s.ids) : static_cast<const void*>(s.keys);
  const bool vec = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(s.kw)) & 15) == 0;
  const int nfull = vec ? s.n / kChunk : 0;
  for (int c = blockIdx.x; c < nfull; c += gridDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(static_cast<const uint32_t*>(in) + (size_t)c * kChunk);
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = src[j * 512 + threadIdx.x];
    if (s.ids) {
      uint4* dst = reinterpret_cast<uint4*>(s.kw + (size_t)c * kChunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = make_uint4(key_of(v[j].x), key_of(v[j].y), key_of(v[j].z), key_of(v[j].w));
        dst[j * 512 + threadIdx.x] = v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      count(v[j].x);
      count(v[j].y);
      count(v[j].z);
      count(v[j].w);
    }
  }
  for (int e = nfull * kChunk + blockIdx.x * 512 + threadIdx.x; e < s.n; e += gridDim.x * 512) {
    uint32_t k;
    if (s.ids) {
      k = key_of((uint32_t)s.ids[e]);
      s.kw[e] = k;
    } else {
      k = s.keys[e];
    }
    count(k);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < s.passes * D; t += 512) {
    const unsigned c = h[t];
    if (c) atomicAdd(&s.hist[t], c);
  }
}

struct OsPass {
  RsPass p;
  const unsigned* hist;   // [D] this pass's digit totals
  unsigned* status;       // [ntiles][D]
  int* tile_ctr;
  int* err;
  int spin_cap;
  const int* offsets;  // RsSrc::offsets (first pass only: generated payload)
  int B, code_shift;
};

// Largest b in [0, B) with offsets[b] <= p (p wave-uniform, offsets[0] <= p): 64 probes per step.
__device__ inline int rs_find_example(const int* offsets, int B, int p, int lane) {
  int lo = 0, hi = B;
  while (hi - lo > kWave) {
    const int step = (hi - lo + kWave - 1) / kWave;
    const int q = lo + lane * step;
    const uint64_t m = __ballot(q < hi && offsets[q] <= p);
    lo += (m ? 63 - __clzll(m) : 0) * step;
    hi = min(hi, lo + step);
  }
  const int q = lo + lane;
  const uint64_t m = __ballot(q < hi && offsets[q] <= p);
  return lo + (m ? 63 - __clzll(m) : 0);
}

// Lane l: start of example wb + l (past the batch: INT_MAX, never <= an element)
__device__ inline int rs_window(const int* offsets, int B, int wb, int lane) {
  const int q = wb + lane;
  return q <= B ? offsets[q] : 0x7fffffff;
}

template <int DB, bool GEN>
__global__ __launch_bounds__(kRsThreads) void os_pass_kernel(OsPass o) {
  constexpr int D = 1 << DB;
  const RsPass& p = o.p;
  __shared__ unsigned wc[kRsWaves][D];
  __shared__ int gofs[D];
  __shared__ uint32_t stage[kRsTile];
  __shared__ uint64_t sh[kRsWaves];
  __shared__ int tile_s;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
  if (threadIdx.x == 0) tile_s = atomicAdd(o.tile_ctr, 1);
  const unsigned hd = threadIdx.x < D ? o.hist[threadIdx.x] : 0u;  // (loaded early: used after the ranking)
  for (int t = threadIdx.x; t < kRsWaves * D; t += kRsThreads) (&wc[0][0])[t] = 0u;
  __syncthreads();
  const int tile = tile_s;
  uint32_t key[kRsItems], dig[kRsItems];
  bool ok[kRsItems];
  rs_load<DB>(p, tile, key, dig, ok);
  int val[kRsItems];
  const int e0 = tile * kRsTile + wv * kRsWaveElems + lane;
  if constexpr (GEN) {
    // packed occurrence codes: each lane finds its element's example in a window of 64 example starts
    // (csr_rows_kernel's shuffle search); the wave's 1024 elements span ~26 Criteo examples, so the
    // window moves (by 63 examples) only for short examples
    const int w0 = e0 - lane;
    int wb = w0 < p.n ? rs_find_example(o.offsets, o.B, w0, lane) : 0;
    int ow = rs_window(o.offsets, o.B, wb, lane);
#pragma unroll
    for (int i = 0; i < kRsItems; ++i) {
      const int e = e0 + i * kWave;
      int ex = -1, st = 0;
      for (;;) {  // (at most B / 63 + 1 rounds over the whole tile)
        int k = 0;
#pragma unroll
        for (int step = kWave / 2; step > 0; step >>= 1) {
          const int c = k + step;
          if (__shfl(ow, c) <= e) k = c;
        }
        const int sk = __shfl(ow, k);
        if (ok[i] && ex < 0 && k < kWave - 1) {
          ex = wb + k;
          st = sk;
        }
        if (!__ballot(ok[i] && ex < 0)) break;
        wb += kWave - 1;
        ow = rs_window(o.offsets, o.B, wb, lane);
      }
      val[i] = ok[i] ? (o.code_shift > 0 ? (ex << o.code_shift) | (e - st) : ex) : 0;
    }
  } else {
#pragma unroll
    for (int i = 0; i < kRsItems; ++i) val[i] = ok[i] ? p.vin[e0 + i * kWave] : 0;
  }
  unsigned rank[kRsItems];
  rs_rank_wave<DB>(dig, ok, wc[wv], rank);
  __syncthreads();
  const int d = threadIdx.x;
  unsigned tcount = 0;
  if (d < D) {
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) {
      const unsigned c = wc[w][d];
      wc[w][d] = tcount;
      tcount += c;
    }
    // publish the tile's count as soon as it is known (tile 0: already its inclusive prefix)
    __hip_atomic_store(o.status + (size_t)tile * D + d, (tile == 0 ? kOsInc : kOsAgg) | tcount, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // tile-local start of digit d's run (low half) and the global start of digit d (high half)
  const uint64_t ex2 = rs_block_excl(((uint64_t)hd << 32) | tcount, sh);
  const unsigned tstart = (unsigned)ex2, gbase = (unsigned)(ex2 >> 32);
  // look-back: thread d walks back over the tiles before this one, kOsLookback per round
  unsigned excl = 0;
  if (d < D && tile > 0 && o.spin_cap < 0) atomicOr(o.err, 1);  // (injected failure: tests)
  if (d < D && tile > 0) {
    int t = tile - 1;
    for (int round = 0; t >= 0; ++round) {
      unsigned w4[kOsLookback];
#pragma unroll
      for (int k = 0; k < kOsLookback; ++k)
        w4[k] = t - k >= 0 ? __hip_atomic_load(o.status + (size_t)(t - k) * D + d, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : kOsInc;  // (before tile 0: an inclusive prefix of 0)
      bool stop = false, wait = false;
#pragma unroll
      for (int k = 0; k < kOsLookback; ++k) {
        if (stop || wait) continue;
        const unsigned f = w4[k] >> 30;
        if (f == 0) {
          wait = true;  // not published yet: read it again
        } else {
          excl += w4[k] & kOsCnt;
          --t;
          stop = f == 2;
        }
      }
      if (stop) break;
      if (wait) {
        if (round >= o.spin_cap) {
          atomicOr(o.err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __hip_atomic_store(o.status + (size_t)tile * D + d, kOsInc | (excl + tcount), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (d < D) {
    gofs[d] = (int)(gbase + excl) - (int)tstart;
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) wc[w][d] += tstart;
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

// Workspace: [alt keys n][alt values n][status passes x ntiles x D][hist passes x D][ctr]
size_t radix_sort_ws_bytes(int n) {
  if (n <= 0) return 256;
  const size_t ntiles = ((size_t)n + kRsTile - 1) / kRsTile;
  return rs_align(4 * (size_t)n) * 2 + rs_align(4 * (size_t)kOsMaxPasses * ntiles * kRsMaxDigits) +
         rs_align(4 * (size_t)kOsMaxPasses * kRsMaxDigits) + rs_align(4 * (kOsMaxPasses + 1));
}

// Stable sort of (keys[i], vals[i]) by keys' bits [0, end_bit) into (kout, vout); keys / vals are
// not modified.  0 or a hip error code; -2: workspace too small; -5: n >= 2^30.  radix_sort_error(ws, n) locates the
// look-back error word (nonzero: a spin bound was hit, the output is not valid).
int launch_radix_sort(const uint32_t* keys, const int* vals, uint32_t* kout, int* vout, int n, int end_bit,
                      void* ws, size_t ws_bytes, hipStream_t st, const RsSrc& src = RsSrc()) {
  if (n <= 0) return 0;
  if ((unsigned)n > kOsCnt) return -5;  // (look-back words hold 30-bit prefixes)
  if (ws_bytes < radix_sort_ws_bytes(n)) return -2;
  if ((src.ids && (src.W < 1 || src.Rps < 0)) || (src.offsets && (src.B < 1 || src.code_shift < 0))) return -4;
  end_bit = end_bit < 1 ? 1 : (end_bit > 32 ? 32 : end_bit);
  int passes, db;
  rs_plan(end_bit, passes, db);
  if (passes > kOsMaxPasses || (db == 9 && passes > kOsMaxPasses - 1)) return -3;
  const int ntiles = (n + kRsTile - 1) / kRsTile;
  const int D = 1 << db;
  char* b = static_cast<char*>(ws);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = b + off;
    off += rs_align(bytes);
    return q;
  };
  uint32_t* alt_k = reinterpret_cast<uint32_t*>(take(4 * (size_t)n));
  int* alt_v = reinterpret_cast<int*>(take(4 * (size_t)n));
  unsigned* status = reinterpret_cast<unsigned*>(take(4 * (size_t)kOsMaxPasses * ntiles * kRsMaxDigits));
  unsigned* hist = reinterpret_cast<unsigned*>(take(4 * (size_t)kOsMaxPasses * kRsMaxDigits));
  int* ctr = reinterpret_cast<int*>(take(4 * (kOsMaxPasses + 1)));
  hipError_t e = hipMemsetAsync(hist, 0, 4 * (size_t)passes * D, st);
  if (e != hipSuccess) return (int)e;
  OsSort s{n, passes, db, end_bit, keys, src.ids, const_cast<uint32_t*>(keys), src.W, src.Rps, hist, status, ctr,
           (size_t)passes * ntiles * D};
  const int hb = min(kOsHistBlocks, (n + 512 * 16 - 1) / (512 * 16));
  if (db == 9) hipLaunchKernelGGL(os_hist_kernel<9>, dim3(hb), dim3(512), 0, st, s);
  else hipLaunchKernelGGL(os_hist_kernel<8>, dim3(hb), dim3(512), 0, st, s);
  const uint32_t* kin = keys;
  const int* vin = vals;
  for (int i = 0; i < passes; ++i) {
    // the last pass writes the output, the one before it the alternate buffers, and so on
    const bool to_out = ((passes - 1 - i) % 2) == 0;
    const int shift = i * db, bits = end_bit - shift < db ? end_bit - shift : db;
    const uint32_t dmask = bits >= 32 ? 0xffffffffu : (1u << bits) - 1u;
    RsPass p{n, ntiles, shift, dmask, kin, vin, to_out ? kout : alt_k, to_out ? vout : alt_v};
    OsPass o{p, hist + (size_t)i * D, status + (size_t)i * ntiles * D, ctr + i, ctr + kOsMaxPasses,
             g_os_spin_cap, src.offsets, src.B, src.code_shift};
    const bool gen = i == 0 && src.offsets;
    if (db == 9) {
      if (gen) hipLaunchKernelGGL((os_pass_kernel<9, true>), dim3(ntiles), dim3(kRsThreads), 0, st, o);
      else hipLaunchKernelGGL((os_pass_kernel<9, false>), dim3(ntiles), dim3(kRsThreads), 0, st, o);
    } else {
      if (gen) hipLaunchKernelGGL((os_pass_kernel<8, true>), dim3(ntiles), dim3(kRsThreads), 0, st, o);
      else hipLaunchKernelGGL((os_pass_kernel<8, false>), dim3(ntiles), dim3(kRsThreads), 0, st, o);
    }
    kin = p.kout;
    vin = p.vout;
  }
  return (int)hipGetLastError();
}

const int* radix_sort_error(const void* ws, int n) {
  const size_t ntiles = ((size_t)n + kRsTile - 1) / kRsTile;
  const size_t off = rs_align(4 * (size_t)n) * 2 + rs_align(4 * (size_t)kOsMaxPasses * ntiles * kRsMaxDigits) +
                     rs_align(4 * (size_t)kOsMaxPasses * kRsMaxDigits);
  return reinterpret_cast<const int*>(static_cast<const char*>(ws) + off) + kOsMaxPasses;
}
