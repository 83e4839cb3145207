// Hot-dictionary dedup: the local step's batch grouping without radix-sorting every occurrence.
//
// Same output as launch_dedup (dedup.hip) with the onesweep sort -- occurrences grouped by key in
// ascending key order, stable (ties in occurrence order), chunks cut at heads and CH-aligned
// positions -- bitwise, but the radix sort runs over the long tail only:
//
//   * a dictionary of <= kHdMaxH "hot" table rows (the most frequent rows of an earlier plan,
//     ascending keys, index h = rank; rebuilt on the device by hd_dict_*) is probed per occurrence
//     from an LDS hash table.  On a Criteo-shaped batch 4096 rows hold ~82% of the occurrences;
//   * hot occurrences are grouped by a one-pass stable counting sort over h: per-tile LDS
//     histograms (hd_classify), an exclusive prefix over tiles per h (hd_hot_scan), then each
//     tile places its occurrences in order (hd_hot_scatter: per-wave LDS cursors, the lanes of one
//     h ranked by a ballot match over h's bits);
//   * the rest ("cold": rarely repeated rows) is compacted per wave subtile by the same classify
//     pass (phase 1), counted, and -- the host reads the count -- sorted by rocPRIM's onesweep
//     radix sort (phase 2);
//   * the two key-ordered groupings are merged by binary searches (a cold segment is preceded by
//     the hot rows with smaller keys and vice versa), written straight to their final positions,
//     and the chunk plan is cut over the merged segments (hd_plan_*).
//
// The dictionary only decides which path an occurrence takes, never the result: any dictionary
// (empty, stale, rows absent from the batch) gives the same plan.
//
// Replaces the sort of all 5.1M occurrences of a Criteo-shaped batch (onesweep, three 9-bit
// passes) for the reference's tf.unique (tffm/fm_model.py:72) and the grouping its FmGrad gets
// from fp32 atomics (cc/fm_grad_op.h:84-104).
#include "fm_common.h"
#include <rocprim/rocprim.hpp>

namespace fm {

constexpr int kHdMaxH = 4096;                       // dictionary rows (12-bit index)
constexpr int kHdSlots = 2 * kHdMaxH;               // LDS open-addressing table (load <= 0.5)
constexpr int kHdSlotBits = 13;
constexpr int kHdThreads = 512;                     // classify / hot-scatter workgroup (8 waves)
constexpr int kHdWaves = kHdThreads / kWave;
constexpr int kHdTile = 8192;                       // classify / hot-scatter tile
constexpr int kHdQ = kHdTile / kHdWaves;            // 1024 elements per wave: one cold subtile
constexpr int kHdR = kHdQ / kWave;                  // 16 rounds of 64
constexpr int kHdScanWaves = 16;                    // hot column scan: tile ranges per column
constexpr int kHdIt = 2;                            // cold-RLE / plan items per thread
constexpr int kHdRle = kBlock * kHdIt;              // cold-RLE / plan tile
constexpr int kHdInline = 8;                        // chunks a plan thread writes per segment
constexpr int kHdMinCount = 16;                     // dictionary rows occur at least this often
static_assert(kHdSlots == 1 << kHdSlotBits, "slot bits");
static_assert(kHdQ < 65536, "16-bit per-wave counters");

__device__ inline int hd_slot(uint32_t key) { return (int)((key * 0x9E3779B1u) >> (32 - kHdSlotBits)); }

__device__ inline unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & (kWave - 1);
  return lane ? (~0ull >> (kWave - lane)) : 0ull;
}

// Lanes of this wave holding the same `d` (nb low bits), among the lanes with `valid`.
__device__ inline unsigned long long match_bits(bool valid, int d, int nb) {
  unsigned long long peers = __ballot(valid);
  for (int b = 0; b < nb; ++b) {
    const bool bit = (d >> b) & 1;
    const unsigned long long m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Number of entries of the ascending array a[0, n) below x.
template <typename T>
__device__ inline int lower_bound_dev(const T* a, int n, T x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

struct HdDict {          // persistent dictionary (device)
  int* keys;             // [kHdMaxH] ascending, first *n valid
  int* n;                // [1]
  int* ht_key;           // [kHdSlots] (-1: empty)
  int* ht_idx;           // [kHdSlots]
  int* sel;              // [kHdMaxH] refresh scratch: selected keys (unordered)
  int* meta;             // [40]: [0..31] log2 count bins, [32] #selected
};

struct HdArgs {
  int n, kb, CH;
  int ntiles;            // ceil(n / kHdTile)
  int nsub;              // kHdWaves * ntiles: cold subtiles (one per classify wave)
  int scan_ct;           // tiles per range of the hot column scan
  int rle_tiles;         // ceil(n / kHdRle): plan tiles (capacity)
  int n_c;               // phase 2: cold occurrences (read by the host after phase 1)
  const uint32_t* keys;  // [n]
  const int* pay;        // [n]
  HdDict d;
  // workspace
  int16_t* hidx;         // [n] dictionary index per occurrence (-1: cold)
  uint32_t* ctk;         // [ntiles * kHdTile] per-subtile cold lists (keys)
  int* ctv;              //   (payload)
  int* sub_cold;         // [nsub] cold count per subtile -> exclusive prefix
  uint32_t* ck; int* cv;         // [n] compacted cold pairs
  uint32_t* cks; int* cvs;       // [n] sorted cold pairs
  void* sort_tmp; size_t sort_bytes;
  int* hist;             // [ntiles * kHdMaxH] per-tile hot counts -> exclusive prefix within its range
  int* csum;             // [kHdScanWaves * kHdMaxH] exclusive prefix over the ranges
  int* hot_cnt;          // [kHdMaxH]
  int* hot_pre;          // [kHdMaxH + 1] exclusive prefix of hot_cnt (occurrences)
  int* hp;               // [kHdMaxH + 1] exclusive prefix of (hot_cnt > 0) (segments)
  int* fo;               // [kHdMaxH] final start of each present hot row
  int* hc;               // [8] device: n_c, U_c, #present hot rows, hot occurrences, #long segments
  int* tile_cnt;         // [rle_tiles] per-tile counts (cold heads, then plan chunks)
  uint32_t* cuniq;       // [n] cold unique keys
  int* css;              // [n + 1] cold segment starts (cold-sorted positions)
  int* long_list;        // [n] segments with more than kHdInline chunks
  // outputs: the plan (dedup.hip DedupArgs)
  uint32_t* skeys;       // nullable
  int* spay;
  uint32_t* uniq;
  int* seg_start;
  int* seg_chunk;
  int* chunk_start;
  int* chunk_seg;
  int* chunk_key;
  int* counts;
};

// ---------------------------------------------------------------------------
// Phase 1. classify: dictionary probe, per-tile hot histogram, per-wave cold lists (occurrence
// order); every key / payload of the wave is loaded up front (16 rounds in flight)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kHdThreads) void hd_classify_kernel(HdArgs a) {
  __shared__ int s_key[kHdSlots];
  __shared__ int16_t s_idx[kHdSlots];
  __shared__ unsigned s_cnt[kHdMaxH];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6;
  const int Hn = min(*a.d.n, kHdMaxH);
  const int tile = blockIdx.x;
  const int base = tile * kHdTile + wv * kHdQ;
  uint32_t key[kHdR];
  int pay[kHdR];
#pragma unroll
  for (int r = 0; r < kHdR; ++r) {
    const int j = base + r * kWave + lane;
    key[r] = j < a.n ? a.keys[j] : 0u;
    pay[r] = j < a.n ? a.pay[j] : 0;
  }
  if (Hn > 0) {
    for (int i = tid; i < kHdSlots; i += kHdThreads) {
      s_key[i] = a.d.ht_key[i];
      s_idx[i] = (int16_t)a.d.ht_idx[i];
    }
  }
  for (int i = tid; i < Hn; i += kHdThreads) s_cnt[i] = 0u;
  __syncthreads();
  const int sub = tile * kHdWaves + wv;
  uint32_t* ok_k = a.ctk + (long long)sub * kHdQ;
  int* ok_v = a.ctv + (long long)sub * kHdQ;
  int c = 0;
#pragma unroll
  for (int r = 0; r < kHdR; ++r) {
    const int j = base + r * kWave + lane;
    const bool ok = j < a.n;
    int h = -1;
    if (ok && Hn > 0) {
      int s = hd_slot(key[r]);
#pragma unroll 1
      for (int probe = 0; probe < kHdSlots; ++probe) {
        const int k = s_key[s];
        if (k == (int)key[r]) { h = s_idx[s]; break; }
        if (k < 0) break;
        s = (s + 1) & (kHdSlots - 1);
      }
    }
    if (ok) a.hidx[j] = (int16_t)h;
    if (h >= 0) atomicAdd(&s_cnt[h], 1u);
    const bool cold = ok && h < 0;
    const unsigned long long m = __ballot(cold);
    if (cold) {
      const int p = c + __popcll(m & lanemask_lt());
      ok_k[p] = key[r];
      ok_v[p] = pay[r];
    }
    c += __popcll(m);
  }
  if (lane == 0) a.sub_cold[sub] = c;
  __syncthreads();
  int* hrow = a.hist + (long long)tile * kHdMaxH;
  for (int i = tid; i < Hn; i += kHdThreads) hrow[i] = (int)s_cnt[i];
}

// Block-wide exclusive scan (kBlock threads).
__device__ inline void hd_block_scan(unsigned v, unsigned& ex, unsigned& tot) {
  __shared__ unsigned sh[kWavesPerBlock];
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
  for (int w = 0; w < kWavesPerBlock; ++w) {
    if (w < wv) b += sh[w];
    t += sh[w];
  }
  ex = b + inc - v;
  tot = t;
  __syncthreads();
}

// sum of cnt[0, upto) over the block (the counts of the tiles before this one; L2-resident)
__device__ inline unsigned hd_prefix_of_tiles(const int* cnt, int upto) {
  __shared__ unsigned sh[kWavesPerBlock];
  unsigned s = 0;
  for (int i = threadIdx.x; i < upto; i += kBlock) s += (unsigned)cnt[i];
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = s;
  __syncthreads();
  unsigned t = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) t += sh[w];
  __syncthreads();
  return t;
}

// cold subtile counts -> exclusive prefix (in place) and the total n_c: one workgroup of 1024
// threads, each owning a run of consecutive subtiles
__global__ __launch_bounds__(1024) void hd_cold_prefix_kernel(HdArgs a) {
  __shared__ unsigned s_w[16];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6;
  const int per = (a.nsub + 1023) / 1024;
  const int i0 = tid * per, i1 = min(a.nsub, i0 + per);
  unsigned own = 0;
  for (int i = i0; i < i1; ++i) own += (unsigned)a.sub_cold[i];
  unsigned inc = own;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned up = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += up;
  }
  if (lane == kWave - 1) s_w[wv] = inc;
  __syncthreads();
  unsigned run = inc - own, tot = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wv) run += s_w[w];
    tot += s_w[w];
  }
  for (int i = i0; i < i1; ++i) {
    const unsigned c = (unsigned)a.sub_cold[i];
    a.sub_cold[i] = (int)run;
    run += c;
  }
  if (tid == 0) a.hc[0] = (int)tot;
}

// ---------------------------------------------------------------------------
// Phase 2.
// ---------------------------------------------------------------------------
// cold lists -> one contiguous array (occurrence order kept)
__global__ __launch_bounds__(kHdThreads) void hd_cold_compact_kernel(HdArgs a) {
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  const int sub = blockIdx.x * kHdWaves + wv;
  if (sub >= a.nsub) return;
  const int o0 = a.sub_cold[sub];
  const int o1 = sub + 1 < a.nsub ? a.sub_cold[sub + 1] : a.n_c;
  const uint32_t* sk = a.ctk + (long long)sub * kHdQ;
  const int* sv = a.ctv + (long long)sub * kHdQ;
  for (int i = lane; i < o1 - o0; i += kWave) {
    a.ck[o0 + i] = sk[i];
    a.cv[o0 + i] = sv[i];
  }
}

// hot counts: per column h, the exclusive prefix over tiles (in place, within each of kHdScanWaves
// tile ranges; csum = the ranges' exclusive prefix) and the column total.  64 columns per
// workgroup, one wave per tile range.
__global__ __launch_bounds__(kWave * kHdScanWaves) void hd_hot_scan_kernel(HdArgs a) {
  __shared__ int s_tot[kHdScanWaves][kWave];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  const int h = blockIdx.x * kWave + lane;
  const int Hn = min(*a.d.n, kHdMaxH);
  const int t0 = wv * a.scan_ct, t1 = min(a.ntiles, t0 + a.scan_ct);
  int s = 0;
  if (h < Hn) {
    int t = t0;
    for (; t + 8 <= t1; t += 8) {
      int v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = a.hist[(long long)(t + q) * kHdMaxH + h];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a.hist[(long long)(t + q) * kHdMaxH + h] = s;
        s += v[q];
      }
    }
    for (; t < t1; ++t) {
      int* p = a.hist + (long long)t * kHdMaxH + h;
      const int v = *p;
      *p = s;
      s += v;
    }
  }
  s_tot[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && h < Hn) {
    int run = 0;
    for (int w = 0; w < kHdScanWaves; ++w) {
      a.csum[w * kHdMaxH + h] = run;
      run += s_tot[w][lane];
    }
    a.hot_cnt[h] = run;
  }
}

// prefixes over the dictionary rows: occurrences (hot_pre) and present rows (hp); one workgroup
__global__ __launch_bounds__(1024) void hd_hot_rows_kernel(HdArgs a) {
  constexpr int kPer = kHdMaxH / 1024;
  __shared__ int s_w[2][16];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6;
  const int Hn = min(*a.d.n, kHdMaxH);
  int tot[kPer], pres[kPer];
  int st = 0, sp = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int h = tid * kPer + i;
    tot[i] = h < Hn ? a.hot_cnt[h] : 0;
    pres[i] = tot[i] > 0;
    st += tot[i];
    sp += pres[i];
  }
  int it = st, ip = sp;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int ut = __shfl_up(it, o, kWave), up = __shfl_up(ip, o, kWave);
    if (lane >= o) { it += ut; ip += up; }
  }
  if (lane == kWave - 1) { s_w[0][wv] = it; s_w[1][wv] = ip; }
  __syncthreads();
  int bt = 0, bp = 0, at = 0, ap = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wv) { bt += s_w[0][w]; bp += s_w[1][w]; }
    at += s_w[0][w];
    ap += s_w[1][w];
  }
  int rt = bt + it - st, rp = bp + ip - sp;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int h = tid * kPer + i;
    if (h < Hn) {
      a.hot_pre[h] = rt;
      a.hp[h] = rp;
    }
    rt += tot[i];
    rp += pres[i];
  }
  if (tid == 0) {
    a.hot_pre[Hn] = at;
    a.hp[Hn] = ap;
    a.hc[2] = ap;  // present rows
    a.hc[3] = at;  // hot occurrences
    a.hc[4] = 0;   // long segments (plan)
  }
}

// cold run-length encoding + final placement of the cold occurrences and segments
__global__ __launch_bounds__(kBlock) void hd_crle_count_kernel(HdArgs a) {
  const int n_c = a.n_c, t = blockIdx.x;
  const int j0 = t * kHdRle + threadIdx.x * kHdIt;
  unsigned v = 0;
  for (int q = 0; q < kHdIt; ++q) {
    const int j = j0 + q;
    if (j < n_c) v += (j == 0 || a.cks[j] != a.cks[j - 1]);
  }
  unsigned ex, tot;
  hd_block_scan(v, ex, tot);
  if (threadIdx.x == 0) a.tile_cnt[t] = (int)tot;
}

__global__ __launch_bounds__(kBlock) void hd_crle_emit_kernel(HdArgs a) {
  __shared__ int s_dk[kHdMaxH];
  __shared__ unsigned s_pre;
  const int n_c = a.n_c, t = blockIdx.x, tid = threadIdx.x;
  const int Hn = min(*a.d.n, kHdMaxH);
  const int last = n_c > 0 ? (n_c - 1) / kHdRle : 0;
  for (int i = tid; i < Hn; i += kBlock) s_dk[i] = a.d.keys[i];
  const unsigned pre = hd_prefix_of_tiles(a.tile_cnt, t);
  const int j0 = t * kHdRle + tid * kHdIt;
  uint32_t k[kHdIt];
  int pv[kHdIt];
  bool hd[kHdIt];
  unsigned v = 0;
#pragma unroll
  for (int q = 0; q < kHdIt; ++q) {
    const int j = j0 + q;
    k[q] = j < n_c ? a.cks[j] : 0u;
    pv[q] = j < n_c ? a.cvs[j] : 0;
  }
#pragma unroll
  for (int q = 0; q < kHdIt; ++q) {
    const int j = j0 + q;
    hd[q] = j < n_c && (j == 0 || k[q] != (q ? k[q - 1] : a.cks[j - 1]));
    v += hd[q];
  }
  unsigned ex, tot;
  hd_block_scan(v, ex, tot);  // (its barriers also cover the s_dk fill)
  if (tid == 0) s_pre = pre;
  __syncthreads();
  int s = (int)(s_pre + ex) - 1;
  int hb = -1;  // dictionary keys below the current key (recomputed at each head)
#pragma unroll
  for (int q = 0; q < kHdIt; ++q) {
    const int j = j0 + q;
    if (j >= n_c) break;
    if (hd[q] || hb < 0) hb = lower_bound_dev(s_dk, Hn, (int)k[q]);
    s += hd[q];
    const int fpos = j + a.hot_pre[hb];
    a.spay[fpos] = pv[q];
    if (a.skeys) a.skeys[fpos] = k[q];
    if (hd[q]) {
      const int fs = s + a.hp[hb];
      a.uniq[fs] = k[q];
      a.seg_start[fs] = fpos;
      a.cuniq[s] = k[q];
      a.css[s] = j;
    }
  }
  if (tid == 0 && t == last) {
    const int Uc = (int)(s_pre + tot);
    a.hc[1] = Uc;
    a.css[Uc] = n_c;
  }
}

// hot segments: final index and start of each present dictionary row
__global__ __launch_bounds__(kBlock) void hd_hot_records_kernel(HdArgs a) {
  const int h = blockIdx.x * kBlock + threadIdx.x;
  const int Hn = min(*a.d.n, kHdMaxH);
  const int Uc = a.hc[1];
  if (h == 0) {
    const int U = Uc + a.hc[2];
    a.counts[0] = U;
    a.seg_start[U] = a.n;
  }
  if (h >= Hn || a.hot_cnt[h] == 0) return;
  const uint32_t key = (uint32_t)a.d.keys[h];
  const int nc = lower_bound_dev(a.cuniq, Uc, key);
  const int fs = a.hp[h] + nc;
  const int st = a.hot_pre[h] + a.css[nc];
  a.uniq[fs] = key;
  a.seg_start[fs] = st;
  a.fo[h] = st;
}

// hot scatter: each tile places its hot occurrences in order.  Per-wave 16-bit cursors, two per
// LDS word (the count of one row in one wave's 1024 occurrences fits), relative to the tile's
// base position of the row.
__device__ inline unsigned hd_get16(const unsigned* w, int h) { return (w[h >> 1] >> ((h & 1) * 16)) & 0xffffu; }

__global__ __launch_bounds__(kHdThreads) void hd_hot_scatter_kernel(HdArgs a) {
  __shared__ unsigned rel[kHdWaves][kHdMaxH / 2];
  __shared__ unsigned tbase[kHdMaxH];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6, tile = blockIdx.x;
  const int Hn = min(*a.d.n, kHdMaxH);
  if (Hn == 0) return;
  const int nb = 32 - __clz(max(Hn - 1, 1));
  const int base = tile * kHdTile + wv * kHdQ;
  int h[kHdR], p[kHdR];
#pragma unroll
  for (int r = 0; r < kHdR; ++r) {
    const int j = base + r * kWave + lane;
    h[r] = j < a.n ? (int)a.hidx[j] : -1;
  }
#pragma unroll
  for (int r = 0; r < kHdR; ++r) {
    const int j = base + r * kWave + lane;
    p[r] = h[r] >= 0 ? a.pay[j] : 0;
  }
  for (int i = tid; i < kHdWaves * (kHdMaxH / 2); i += kHdThreads) (&rel[0][0])[i] = 0u;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kHdR; ++r)
    if (h[r] >= 0) atomicAdd(&rel[wv][h[r] >> 1], 1u << ((h[r] & 1) * 16));
  __syncthreads();
  // counts -> per-wave exclusive offsets (a thread owns the word of rows 2i, 2i + 1)
  const int* hrow = a.hist + (long long)tile * kHdMaxH;
  const int* crow = a.csum + (long long)(tile / a.scan_ct) * kHdMaxH;
  for (int i = tid; i < (Hn + 1) / 2; i += kHdThreads) {
    unsigned r0 = 0, r1 = 0;
#pragma unroll
    for (int w = 0; w < kHdWaves; ++w) {
      const unsigned x = rel[w][i];
      rel[w][i] = r0 | (r1 << 16);
      r0 += x & 0xffffu;
      r1 += x >> 16;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int hh = 2 * i + q;
      if (hh < Hn && a.hot_cnt[hh] > 0) tbase[hh] = (unsigned)(a.fo[hh] + hrow[hh] + crow[hh]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kHdR; ++r) {
    const bool hot = h[r] >= 0;
    const unsigned long long peers = match_bits(hot, h[r], nb);
    if (hot) {
      const int rank = __popcll(peers & lanemask_lt());
      const int tot = __popcll(peers);
      const unsigned pos = tbase[h[r]] + hd_get16(rel[wv], h[r]) + (unsigned)rank;
      a.spay[pos] = p[r];
      if (a.skeys) a.skeys[pos] = (uint32_t)a.d.keys[h[r]];
      if (rank == tot - 1) atomicAdd(&rel[wv][h[r] >> 1], (unsigned)tot << ((h[r] & 1) * 16));
    }
  }
}

// chunk plan over the merged segments (chunks at heads and CH-aligned positions)
__device__ inline int hd_nchunks(int st, int en, int CH) { return en > st ? 1 + (en - 1) / CH - st / CH : 0; }

__global__ __launch_bounds__(kBlock) void hd_plan_count_kernel(HdArgs a) {
  const int U = a.counts[0], t = blockIdx.x;
  if (t * kHdRle >= U && t > 0) {
    if (threadIdx.x == 0) a.tile_cnt[t] = 0;
    return;
  }
  const int s0 = t * kHdRle + threadIdx.x * kHdIt;
  unsigned v = 0;
  for (int q = 0; q < kHdIt; ++q) {
    const int s = s0 + q;
    if (s < U) v += (unsigned)hd_nchunks(a.seg_start[s], a.seg_start[s + 1], a.CH);
  }
  unsigned ex, tot;
  hd_block_scan(v, ex, tot);
  if (threadIdx.x == 0) a.tile_cnt[t] = (int)tot;
}

__global__ __launch_bounds__(kBlock) void hd_plan_emit_kernel(HdArgs a) {
  __shared__ unsigned s_pre;
  const int U = a.counts[0], t = blockIdx.x, tid = threadIdx.x;
  const int last = U > 0 ? (U - 1) / kHdRle : 0;
  if (t > last) return;
  const unsigned pre = hd_prefix_of_tiles(a.tile_cnt, t);
  const int s0 = t * kHdRle + tid * kHdIt;
  int st[kHdIt + 1];
#pragma unroll
  for (int q = 0; q < kHdIt + 1; ++q) st[q] = s0 + q <= U ? a.seg_start[s0 + q] : a.n;
  unsigned v = 0;
  int nch[kHdIt];
#pragma unroll
  for (int q = 0; q < kHdIt; ++q) {
    nch[q] = s0 + q < U ? hd_nchunks(st[q], st[q + 1], a.CH) : 0;
    v += (unsigned)nch[q];
  }
  unsigned ex, tot;
  hd_block_scan(v, ex, tot);
  if (tid == 0) s_pre = pre;
  __syncthreads();
  int c = (int)(s_pre + ex);
  for (int q = 0; q < kHdIt; ++q) {
    const int s = s0 + q;
    if (s >= U) break;
    const int key = (int)a.uniq[s];
    a.seg_chunk[s] = c;
    a.chunk_start[c] = st[q];
    a.chunk_seg[c] = (int)((unsigned)s | (unsigned)kChunkFirst | (nch[q] == 1 ? kChunkSingle : 0u));
    a.chunk_key[c] = key;
    const int m1 = min(nch[q], kHdInline);
    for (int m = 1; m < m1; ++m) {
      a.chunk_start[c + m] = (st[q] / a.CH + m) * a.CH;
      a.chunk_seg[c + m] = s;
      a.chunk_key[c + m] = key;
    }
    if (nch[q] > kHdInline) a.long_list[atomicAdd(&a.hc[4], 1)] = s;
    c += nch[q];
  }
  if (tid == 0 && t == last) {
    const int C = (int)(s_pre + tot);
    a.counts[1] = C;
    a.counts[2] = 0;
    a.counts[3] = 0;
    a.counts[4] = 0;
    a.counts[5] = a.counts[6] = a.counts[7] = 0;
    a.seg_chunk[U] = C;
    a.chunk_start[C] = a.n;
  }
}

// chunks past the first kHdInline of the long segments (one workgroup per listed segment)
__global__ __launch_bounds__(kBlock) void hd_plan_long_kernel(HdArgs a) {
  const int nl = a.hc[4];
  for (int i = blockIdx.x; i < nl; i += gridDim.x) {
    const int s = a.long_list[i];
    const int st = a.seg_start[s], en = a.seg_start[s + 1];
    const int c0 = a.seg_chunk[s], nch = hd_nchunks(st, en, a.CH);
    const int key = (int)a.uniq[s];
    for (int m = kHdInline + threadIdx.x; m < nch; m += kBlock) {
      a.chunk_start[c0 + m] = (st / a.CH + m) * a.CH;
      a.chunk_seg[c0 + m] = s;
      a.chunk_key[c0 + m] = key;
    }
  }
}

// ---------------------------------------------------------------------------
// Dictionary refresh from a finished plan: the rows with the most occurrences (>= kHdMinCount,
// at most kHdMaxH: the count threshold is the smallest power of two that keeps them under the
// cap), ascending, and their LDS hash table.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void hd_dict_bins_kernel(HdDict d, const int* counts, const int* seg_start,
                                                              int n_max) {
  __shared__ unsigned sb[32];
  if (threadIdx.x < 32) sb[threadIdx.x] = 0u;
  __syncthreads();
  const int U = min(counts[0], n_max);
  for (int s = blockIdx.x * kBlock + threadIdx.x; s < U; s += gridDim.x * kBlock) {
    const int c = seg_start[s + 1] - seg_start[s];
    if (c >= kHdMinCount) atomicAdd(&sb[31 - __clz(c)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 32 && sb[threadIdx.x]) atomicAdd(&d.meta[threadIdx.x], (int)sb[threadIdx.x]);
}

__device__ inline int hd_dict_threshold(const int* meta) {
  int acc = 0, b = 31;
  for (; b >= 0; --b) {
    if (acc + meta[b] > kHdMaxH) break;
    acc += meta[b];
  }
  return max(kHdMinCount, b >= 30 ? 0x7fffffff : (1 << (b + 1)));
}

__global__ __launch_bounds__(kBlock) void hd_dict_select_kernel(HdDict d, const int* counts, const int* seg_start,
                                                                const uint32_t* uniq, int n_max) {
  __shared__ int s_thr;
  if (threadIdx.x == 0) s_thr = hd_dict_threshold(d.meta);
  __syncthreads();
  const int thr = s_thr;
  const int U = min(counts[0], n_max);
  for (int s = blockIdx.x * kBlock + threadIdx.x; s < U; s += gridDim.x * kBlock) {
    const int c = seg_start[s + 1] - seg_start[s];
    if (c >= thr) {
      const int i = atomicAdd(&d.meta[32], 1);
      if (i < kHdMaxH) d.sel[i] = (int)uniq[s];
    }
  }
}

__global__ __launch_bounds__(1024) void hd_dict_build_kernel(HdDict d) {
  __shared__ int s_k[kHdMaxH];
  __shared__ int s_tk[kHdSlots];
  __shared__ int s_ti[kHdSlots];
  const int tid = threadIdx.x;
  const int n = min(d.meta[32], kHdMaxH);
  for (int i = tid; i < kHdMaxH; i += 1024) s_k[i] = i < n ? d.sel[i] : 0x7fffffff;
  for (int i = tid; i < kHdSlots; i += 1024) { s_tk[i] = -1; s_ti[i] = 0; }
  __syncthreads();
  // bitonic sort of the selected keys (distinct, non-negative)
  for (int k = 2; k <= kHdMaxH; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < kHdMaxH; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const int x = s_k[i], y = s_k[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { s_k[i] = y; s_k[l] = x; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < n; i += 1024) {
    const int key = s_k[i];
    int s = hd_slot((uint32_t)key);
    for (int probe = 0; probe < kHdSlots; ++probe) {
      const int prev = atomicCAS(&s_tk[s], -1, key);
      if (prev == -1) { s_ti[s] = i; break; }
      s = (s + 1) & (kHdSlots - 1);
    }
  }
  __syncthreads();
  for (int i = tid; i < kHdMaxH; i += 1024) d.keys[i] = s_k[i];
  for (int i = tid; i < kHdSlots; i += 1024) { d.ht_key[i] = s_tk[i]; d.ht_idx[i] = s_ti[i]; }
  if (tid < 33) d.meta[tid] = 0;  // bins and the selection count start at 0 for the next refresh
  if (tid == 0) *d.n = n;
}

int launch_hd_dict_refresh(const HdDict& d, const int* counts, const int* seg_start, const uint32_t* uniq, int n_max,
                           hipStream_t st) {
  if (n_max <= 0) return 0;
  const int g = fill_grid(n_max, kBlock, 1024);
  hipLaunchKernelGGL(hd_dict_bins_kernel, dim3(g), dim3(kBlock), 0, st, d, counts, seg_start, n_max);
  hipLaunchKernelGGL(hd_dict_select_kernel, dim3(g), dim3(kBlock), 0, st, d, counts, seg_start, uniq, n_max);
  hipLaunchKernelGGL(hd_dict_build_kernel, dim3(1), dim3(1024), 0, st, d);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Workspace and launch
// ---------------------------------------------------------------------------
static size_t hd_align(size_t x) { return (x + 255) & ~size_t(255); }

struct HdLayout {
  int ntiles, nsub, scan_ct, rle_tiles;
  size_t hidx, ctk, ctv, sub_cold, ck, cv, cks, cvs, sort, hist, csum, hot_cnt, hot_pre, hp, fo, tile_cnt, cuniq,
      css, long_list, total;
};

static size_t hd_sort_bytes(int n) {
  size_t best = 0;
  for (int bits : {16, 20, 27, 30, 31}) {
    size_t b = 0;
    (void)sort_pairs(nullptr, b, nullptr, nullptr, nullptr, nullptr, n, bits, (hipStream_t)0);
    if (b > best) best = b;
  }
  return hd_align(best);
}

static HdLayout hd_layout(int n) {
  HdLayout L{};
  L.ntiles = (n + kHdTile - 1) / kHdTile;
  L.nsub = L.ntiles * kHdWaves;
  L.scan_ct = (L.ntiles + kHdScanWaves - 1) / kHdScanWaves;
  L.rle_tiles = (n + kHdRle - 1) / kHdRle;
  const size_t n4 = hd_align((size_t)n * 4), full4 = hd_align((size_t)L.ntiles * kHdTile * 4);
  size_t o = 0;
  L.hidx = o; o += hd_align((size_t)n * 2);
  L.ctk = o; o += full4;
  L.ctv = o; o += full4;
  L.sub_cold = o; o += hd_align((size_t)L.nsub * 4);
  L.ck = o; o += n4;
  L.cv = o; o += n4;
  L.cks = o; o += n4;
  L.cvs = o; o += n4;
  L.sort = o; o += hd_sort_bytes(n);
  L.hist = o; o += hd_align((size_t)L.ntiles * kHdMaxH * 4);
  L.csum = o; o += hd_align((size_t)kHdScanWaves * kHdMaxH * 4);
  L.hot_cnt = o; o += hd_align(kHdMaxH * 4);
  L.hot_pre = o; o += hd_align((kHdMaxH + 1) * 4);
  L.hp = o; o += hd_align((kHdMaxH + 1) * 4);
  L.fo = o; o += hd_align(kHdMaxH * 4);
  L.tile_cnt = o; o += hd_align((size_t)L.rle_tiles * 4);
  L.cuniq = o; o += n4;
  L.css = o; o += hd_align((size_t)(n + 1) * 4);
  L.long_list = o; o += n4;
  L.total = o;
  return L;
}

size_t hd_workspace_bytes(int n) { return n > 0 ? hd_layout(n).total : 256; }

struct HdLaunch {
  int n, kb, CH;
  const uint32_t* keys;
  const int* pay;
  HdDict d;
  void* ws;
  size_t ws_bytes;
  int* hc;               // [8] device counters (the host reads hc[0] = n_c between the phases)
  uint32_t* skeys;
  int* spay;
  uint32_t* uniq;
  int* seg_start;
  int* seg_chunk;
  int* chunk_start;
  int* chunk_seg;
  int* chunk_key;
  int* counts;
};

static int hd_args(const HdLaunch& p, HdArgs& a, HdLayout& L) {
  if (p.n <= 0 || p.kb < 1 || p.kb > 31 || p.CH < 1 || p.CH > kMaxCH || !p.hc) return -1;
  L = hd_layout(p.n);
  if (L.total > p.ws_bytes) return -2;
  char* w = static_cast<char*>(p.ws);
  a = HdArgs{};
  a.n = p.n; a.kb = p.kb; a.CH = p.CH;
  a.ntiles = L.ntiles; a.nsub = L.nsub; a.scan_ct = L.scan_ct; a.rle_tiles = L.rle_tiles;
  a.keys = p.keys; a.pay = p.pay; a.d = p.d;
  a.hidx = reinterpret_cast<int16_t*>(w + L.hidx);
  a.ctk = reinterpret_cast<uint32_t*>(w + L.ctk); a.ctv = reinterpret_cast<int*>(w + L.ctv);
  a.sub_cold = reinterpret_cast<int*>(w + L.sub_cold);
  a.ck = reinterpret_cast<uint32_t*>(w + L.ck); a.cv = reinterpret_cast<int*>(w + L.cv);
  a.cks = reinterpret_cast<uint32_t*>(w + L.cks); a.cvs = reinterpret_cast<int*>(w + L.cvs);
  a.sort_tmp = w + L.sort; a.sort_bytes = L.hist - L.sort;
  a.hist = reinterpret_cast<int*>(w + L.hist); a.csum = reinterpret_cast<int*>(w + L.csum);
  a.hot_cnt = reinterpret_cast<int*>(w + L.hot_cnt); a.hot_pre = reinterpret_cast<int*>(w + L.hot_pre);
  a.hp = reinterpret_cast<int*>(w + L.hp); a.fo = reinterpret_cast<int*>(w + L.fo);
  a.hc = p.hc; a.tile_cnt = reinterpret_cast<int*>(w + L.tile_cnt);
  a.cuniq = reinterpret_cast<uint32_t*>(w + L.cuniq); a.css = reinterpret_cast<int*>(w + L.css);
  a.long_list = reinterpret_cast<int*>(w + L.long_list);
  a.skeys = p.skeys; a.spay = p.spay; a.uniq = p.uniq; a.seg_start = p.seg_start; a.seg_chunk = p.seg_chunk;
  a.chunk_start = p.chunk_start; a.chunk_seg = p.chunk_seg; a.chunk_key = p.chunk_key; a.counts = p.counts;
  return 0;
}

// phase 1: classify + cold count (hc[0]); the hot column scan runs here too (it needs only the
// classify's histograms), so phase 2 starts with the cold sort
int launch_hd_phase1(const HdLaunch& p, hipStream_t st) {
  HdArgs a;
  HdLayout L;
  if (int e = hd_args(p, a, L)) return e;
  hipLaunchKernelGGL(hd_classify_kernel, dim3(L.ntiles), dim3(kHdThreads), 0, st, a);
  hipLaunchKernelGGL(hd_cold_prefix_kernel, dim3(1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(hd_hot_scan_kernel, dim3(kHdMaxH / kWave), dim3(kWave * kHdScanWaves), 0, st, a);
  hipLaunchKernelGGL(hd_hot_rows_kernel, dim3(1), dim3(1024), 0, st, a);
  return (int)hipGetLastError();
}

// phase 2, with the cold count n_c of phase 1
int launch_hd_phase2(const HdLaunch& p, int n_c, hipStream_t st) {
  HdArgs a;
  HdLayout L;
  if (int e = hd_args(p, a, L)) return e;
  if (n_c < 0 || n_c > p.n) return -3;
  a.n_c = n_c;
  hipLaunchKernelGGL(hd_cold_compact_kernel, dim3(L.ntiles), dim3(kHdThreads), 0, st, a);
  if (n_c > 0) {
    size_t sb = a.sort_bytes;
    const hipError_t e = sort_pairs(a.sort_tmp, sb, a.ck, a.cks, a.cv, a.cvs, n_c, p.kb, st);
    if (e != hipSuccess) return (int)e;
  }
  const int ct = std::max(1, (n_c + kHdRle - 1) / kHdRle);
  hipLaunchKernelGGL(hd_crle_count_kernel, dim3(ct), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hd_crle_emit_kernel, dim3(ct), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hd_hot_records_kernel, dim3(kHdMaxH / kBlock), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hd_hot_scatter_kernel, dim3(L.ntiles), dim3(kHdThreads), 0, st, a);
  hipLaunchKernelGGL(hd_plan_count_kernel, dim3(L.rle_tiles), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hd_plan_emit_kernel, dim3(L.rle_tiles), dim3(kBlock), 0, st, a);
  hipLaunchKernelGGL(hd_plan_long_kernel, dim3(256), dim3(kBlock), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm
