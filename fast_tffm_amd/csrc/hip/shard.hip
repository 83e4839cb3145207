// Owner-side kernels of the row-sharded exchange (parallel/exchange.py):
// gather requested table rows into a packed [v | w | pad] send buffer, and sum
// the gradient rows every peer returned for one table row before applying the
// optimizer once (replaces the PS-side embedding gather and SparseApplyAdagrad
// that the reference gets from TF's gRPC runtime, tffm/fm_model.py:291, :341-348).
#include <algorithm>
#include <rocprim/rocprim.hpp>
#include "fm_common.h"

namespace fm {

constexpr int kMaxRuns = 64;  // source ranks handled by the early-exchange kernels

// ---------------------------------------------------------------------------
// Row-sharded helpers
// ---------------------------------------------------------------------------
struct GatherArgs {
  int R;
  const int* req;           // [R] local table rows requested by peers
  const void* v; long long v_stride;
  const float* w; long long w_stride;
  int Kp;
  float* out; long long o_stride;   // [R, o_stride]: v at [0,Kp), w at Kp
  int skip0, skip1;         // requests [skip0, skip1) are not gathered (this rank's own: self rows)
};

template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(GatherArgs a) {
  using F = Frag<TV>;
  constexpr int EPL = F::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  const int nskip = a.skip1 - a.skip0;
  for (int q = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; q < a.R - nskip; q += ngroups) {
    const int p = q < a.skip0 ? q : q + nskip;
    const long long row = a.req[p];
    float vv[EPL];
    F::load(reinterpret_cast<const TV*>(a.v) + row * a.v_stride + tE * EPL, vv);
    if constexpr (F::kScaled) {
      const float s = row_scale<TV>(a.w, row, a.w_stride);
#pragma unroll
      for (int k = 0; k < EPL; ++k) vv[k] *= s;
    }
    float* dst = a.out + (long long)p * a.o_stride;
    if (tact) {
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(vv[k], vv[k + 1], vv[k + 2], vv[k + 3]);
    }
    if (t == 0) {
      dst[a.Kp] = a.w[row * a.w_stride];
      dst[a.Kp + 1] = 0.f; dst[a.Kp + 2] = 0.f; dst[a.Kp + 3] = 0.f;
    }
  }
}

// Wire-format gather (row-sharded exchange): the row leaves the owner in the
// format the requester's forward/backward read directly, so bf16 / fp8 tables
// cross xGMI at their storage size (exact: the stored bits are copied) and an
// fp32 table can optionally be sent as bf16 (comm_dtype = bf16, RNE).
// Wire row (RB bytes, RB % 16 == 0): [v: Kp elements of the wire dtype, padded
// to vb bytes (vb % 16 == 0)] [w fp32] [scale fp32 (fp8) / 0] [|v|^2 fp32 (fp8) / 0] [tag / 0].
struct GatherWireArgs {
  int R;
  const int* req;           // [R] local table rows requested by peers
  const void* v; long long v_bytes_stride;   // table rows (bytes between rows)
  const float* w; long long w_stride;        // fp8 tables: scale at w[row * w_stride + 1]
  int vbytes;               // bytes of a stored row's Kp elements
  int scaled;               // 1: fp8 table (copy the per-row scale)
  int to_bf16;              // 1: fp32 table -> bf16 wire (Kp % 8 == 0)
  unsigned char* out; long long rb;          // [R, rb] wire rows
  int vb;                   // byte offset of w inside a wire row
  // patch gathers (early row exchange): row p is req[idx[p]], and the tail's last word
  // carries its tag idx[p] - run_off[run of idx[p]] (its position in its source's run)
  const int* idx;           // [R] or null
  const int* run_off;       // [W+1] (with idx)
  int W;
  int skip0, skip1;         // (without idx) requests [skip0, skip1) are not gathered (self rows)
};

// One lane group per row; lane t moves 16 bytes of the wire row's v section
// (UNIT = 16) or 4 bytes (UNIT = 4, rows whose v section is not 16-byte sized).
template <int LPR, int UNIT>
__global__ __launch_bounds__(kBlock) void gather_wire_kernel(GatherWireArgs a) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int out_bytes = a.to_bf16 ? a.vbytes / 2 : a.vbytes;
  const int nunits = out_bytes / UNIT;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  const int nskip = a.skip1 - a.skip0;
  for (int q = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; q < a.R - nskip; q += ngroups) {
    const int p = q < a.skip0 ? q : q + nskip;
    const int ip = a.idx ? a.idx[p] : p;
    const long long row = a.req[ip];
    const unsigned char* src = reinterpret_cast<const unsigned char*>(a.v) + row * a.v_bytes_stride;
    unsigned char* dst = a.out + (long long)p * a.rb;
    for (int u = t; u < nunits; u += LPR) {
      if constexpr (UNIT == 16) {
        if (a.to_bf16) {  // 8 fp32 -> 8 bf16
          const float4 f0 = *reinterpret_cast<const float4*>(src + u * 32);
          const float4 f1 = *reinterpret_cast<const float4*>(src + u * 32 + 16);
          uint4 o;
          o.x = f32_to_bf16_bits(f0.x) | (f32_to_bf16_bits(f0.y) << 16);
          o.y = f32_to_bf16_bits(f0.z) | (f32_to_bf16_bits(f0.w) << 16);
          o.z = f32_to_bf16_bits(f1.x) | (f32_to_bf16_bits(f1.y) << 16);
          o.w = f32_to_bf16_bits(f1.z) | (f32_to_bf16_bits(f1.w) << 16);
          *reinterpret_cast<uint4*>(dst + u * 16) = o;
        } else {
          *reinterpret_cast<uint4*>(dst + u * 16) = *reinterpret_cast<const uint4*>(src + u * 16);
        }
      } else {
        *reinterpret_cast<uint32_t*>(dst + u * 4) = *reinterpret_cast<const uint32_t*>(src + u * 4);
      }
    }
    if (t == 0) {
      float* tail = reinterpret_cast<float*>(dst + a.vb);
      tail[0] = a.w[row * a.w_stride];
      tail[1] = a.scaled ? a.w[row * a.w_stride + 1] : 0.f;
      // fp8: the row's stored |v|^2 ([w, scale, norm, pad] table rows), read by the sharded forward
      tail[2] = a.scaled ? a.w[row * a.w_stride + kFp8Norm] : 0.f;
      int tag = 0;
      if (a.idx) {
        int q = 0;
        while (q + 1 < a.W && a.run_off[q + 1] <= ip) ++q;
        tag = ip - a.run_off[q];
      }
      reinterpret_cast<int*>(tail)[3] = tag;
    }
  }
}

int launch_gather_wire(const GatherWireArgs& a, hipStream_t st) {
  if (a.R <= 0) return 0;
  const int out_bytes = a.to_bf16 ? a.vbytes / 2 : a.vbytes;
  const bool u16 = out_bytes % 16 == 0;
  if (a.to_bf16 && !u16) return -7;
  if (a.skip1 < a.skip0 || a.skip0 < 0 || a.skip1 > a.R || (a.idx && a.skip1 > a.skip0)) return -10;
  const int lpr = std::min(64, next_pow2(std::max(1, u16 ? out_bytes / 16 : out_bytes / 4)));
  const int grid = fill_grid(std::max(1, a.R - (a.skip1 - a.skip0)), kWavesPerBlock * (kWave / lpr));
#define FM_GW(L)                                                                                        \
  case L:                                                                                               \
    if (u16) hipLaunchKernelGGL((gather_wire_kernel<L, 16>), dim3(grid), dim3(kBlock), 0, st, a);      \
    else hipLaunchKernelGGL((gather_wire_kernel<L, 4>), dim3(grid), dim3(kBlock), 0, st, a);           \
    break;
  switch (lpr) {
    FM_GW(1) FM_GW(2) FM_GW(4) FM_GW(8) FM_GW(16) FM_GW(32) FM_GW(64)
    default: return -1;
  }
#undef FM_GW
  return (int)hipGetLastError();
}

struct ApplyArgs {
  const int* num_unique;    // device scalar: number of distinct rows received
  const int* seg_start;     // [U+1] into perm
  const int* uniq;          // [U] local table row
  const int* perm;          // [R] position in grad_in of each sorted entry
  const float* grad_in; long long g_stride;  // [R, g_stride] words: v-grad fp32 (or bf16), w-grad at word g_wcol
  int g_wcol, g_bf16;
  int Kp;
  void* v; long long v_stride;
  float* w; long long w_stride;
  void* s0v; void* s1v; long long s_stride;  // fp32 (bf16 for fp8 tables: fm_common.h StateBf16)
  float* s0w; float* s1w;
  OptParams opt;
  // run-merge form (apply_runs): R received rows forming W ascending runs (one per
  // source rank) and the [R, W] cross-run match matrix of owner_match_kernel
  int R, W;
  const int* run_off;       // [W+1]
  const int* req;           // [R] local table row of each received gradient row
  const int* match;         // [R, W]: index of the same row in run q, or -1 (null when W == 1)
  const int* sr_counter;    // stochastic rounding of bf16 / fp8 row stores (null: round to nearest)
  // dense form (dense_apply): rows row0 .. row0 + R of a dense gradient buffer, touched ones
  // marked at word touch_col; grad_zero (== grad_in, writable) gets every applied row zeroed
  long long row0;
  int touch_col;
  float* grad_zero;
  // row-sharded step: run self_run holds this rank's own requests; the flagged (exclusive)
  // ones were applied in place by the backward (SelfRows) and are skipped here
  int self_run;             // -1: none
  const int* self_excl;     // [run length] 1 = exclusive; null = the whole run
};

// One table row's parameters + optimizer state in registers (this lane's EPL
// columns; lane t == 0 also holds w and its state).  load() is issued before the
// gradient sum so that the row's loads overlap it.
template <int LPR, typename TV, int EW = 0>
struct RowUpdate {
  using F = Frag<TV>;
  static constexpr int EPL = EW ? EW : F::N;  // (EW: the wide fp8 apply's 8 values per lane)
  float vv[EPL], st0[EPL], st1[EPL];
  float pw, q0, q1;
  TV* vrow;
  long long soff;

  __device__ inline void load(const ApplyArgs& a, long long row, int tE) {
    vrow = reinterpret_cast<TV*>(a.v) + row * a.v_stride + tE * EPL;
    frag_load<TV, EPL>(vrow, vv);
    if constexpr (F::kScaled) {
      const float s = row_scale<TV>(a.w, row, a.w_stride);
#pragma unroll
      for (int k = 0; k < EPL; ++k) vv[k] *= s;
    }
    soff = row * a.s_stride + tE * EPL;
    load_state<TV, EPL>(a.s0v, soff, st0);
    if (a.s1v) {
      load_state<TV, EPL>(a.s1v, soff, st1);
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) st1[k] = 0.f;
    }
    pw = a.w[row * a.w_stride];
    q0 = a.s0w[row];
    q1 = a.s1w ? a.s1w[row] : 0.f;
  }

  __device__ inline void step_store(const ApplyArgs& a, const float (&gr)[EPL], float gw, long long row, int t,
                                    bool tact, uint32_t sr) {
    opt_step_row<TV, EPL>(a.opt, gr, vv, st0, st1);
    store_row_e<LPR, TV, EPL>(vrow, vv, a.w, row, a.w_stride, t, tact, sr);
    if (tact) {
      const uint32_t col = (uint32_t)(t * EPL);
      store_state<TV, EPL>(a.s0v, soff, st0, sr ? sr ^ kSrSalt0 : 0u, (uint32_t)row, col);
      if (a.s1v) store_state<TV, EPL>(a.s1v, soff, st1, sr ? sr ^ kSrSalt1 : 0u, (uint32_t)row, col);
    }
    if (t == 0) {
      opt_step_tv<TV>(a.opt, gw, pw, q0, q1);
      a.w[row * a.w_stride] = pw;
      a.s0w[row] = q0;
      if (a.s1w) a.s1w[row] = q1;
    }
  }
};

template <int EPL>
__device__ inline void add_grad_row(const ApplyArgs& a, const float* src, int tE, float (&gr)[EPL], float& gw) {
  if (a.g_bf16) {
    float h[EPL];
    load_bf16x<EPL>(reinterpret_cast<const uint16_t*>(src) + tE * EPL, h);
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] += h[k];
  } else {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
      gr[k] += f.x; gr[k + 1] += f.y; gr[k + 2] += f.z; gr[k + 3] += f.w;
    }
  }
  gw += src[a.g_wcol];
}

// Owner-side: sum the gradient rows every peer sent for one table row (in
// source-rank order: the sort is stable and the receive buffer is rank-major)
// and apply the optimizer once.
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void apply_rows_kernel(ApplyArgs a) {
  const uint32_t sr = sr_step_seed(a.sr_counter);  // stochastic rounding seed (0: nearest)
  constexpr int EPL = Frag<TV>::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int U = *a.num_unique;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  for (int u = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; u < U; u += ngroups) {
    const long long row = a.uniq[u];
    RowUpdate<LPR, TV> ru;
    ru.load(a, row, tE);
    float gr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] = 0.f;
    float gw = 0.f;
    const int j1 = a.seg_start[u + 1];
    for (int j = a.seg_start[u]; j < j1; ++j)
      add_grad_row<EPL>(a, a.grad_in + (long long)a.perm[j] * a.g_stride, tE, gr, gw);
    ru.step_store(a, gr, gw, row, t, tact, sr);
  }
}

// ---------------------------------------------------------------------------
// Run-merge grouping (replaces a sort of the received requests).  The owner
// receives W runs, one per source rank, each holding that rank's unique rows
// in ascending order, so a row appears at most once per run.  One thread per
// (received row i, run q) binary-searches row req[i] in run q; the apply
// kernel then treats the first run holding a row as its leader and sums the
// row's gradients over the runs in rank order (deterministic, no atomics).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void owner_match_kernel(int R, int W, const int* run_off, const int* req,
                                                             int* match) {
  const long long n = (long long)R * W;
  for (long long p = blockIdx.x * (long long)kBlock + threadIdx.x; p < n; p += (long long)gridDim.x * kBlock) {
    const int i = (int)(p / W), q = (int)(p % W);
    const int key = req[i];
    int lo = run_off[q];
    const int end = run_off[q + 1];
    int hi = end;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (req[mid] < key) lo = mid + 1; else hi = mid;
    }
    match[p] = (lo < end && req[lo] == key) ? lo : -1;
  }
}

// Membership of every row of a (next step's) request list in a previous request
// list given as W ascending runs: flag[i] = 1 when some run holds req[i] (the row is
// updated by that step's apply, so its early-gathered copy must be patched).
__global__ __launch_bounds__(kBlock) void run_member_kernel(int R, const int* req, int W, const int* run_off,
                                                            const int* prev, int* flag) {
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < R; i += gridDim.x * kBlock) {
    const int key = req[i];
    int hit = 0;
    for (int q = 0; q < W && !hit; ++q) {
      int lo = run_off[q];
      const int end = run_off[q + 1];
      int hi = end;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (prev[mid] < key) lo = mid + 1; else hi = mid;
      }
      hit = lo < end && prev[lo] == key;
    }
    flag[i] = hit;
  }
}

// Early row exchange, owner side: flag[i] = 1 when request i (a row of the next step)
// is in the previous step's request runs (the previous step's apply updates it), and
// dcount[q] = number of flagged requests in run q of the next step (per source rank).
__global__ __launch_bounds__(kBlock) void dirty_scan_kernel(int R, const int* req, int W, const int* run_off,
                                                            int Wp, const int* prev_off, const int* prev, int* flag,
                                                            int* dcount, int skip0, int skip1) {
  __shared__ int cnt[kMaxRuns];
  __shared__ int off[kMaxRuns + 1];
  for (int q = threadIdx.x; q <= W; q += kBlock) {
    if (q < W) cnt[q] = 0;
    off[q] = run_off[q];
  }
  __syncthreads();
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < R; i += gridDim.x * kBlock) {
    const int key = req[i];
    int hit = 0;
    // (requests [skip0, skip1): this rank's own rows, read from the table -- never patched)
    for (int q = 0; q < Wp && !hit && (i < skip0 || i >= skip1); ++q) {
      int lo = prev_off[q];
      const int end = prev_off[q + 1];
      int hi = end;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (prev[mid] < key) lo = mid + 1; else hi = mid;
      }
      hit = lo < end && prev[lo] == key;
    }
    flag[i] = hit;
    if (hit) {
      int q = 0;
      while (q + 1 < W && off[q + 1] <= i) ++q;
      atomicAdd(&cnt[q], 1);
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < W; q += kBlock)
    if (cnt[q]) atomicAdd(&dcount[q], cnt[q]);
}

// Early row exchange, requester side: patch row p (rank-major by owner, recv_off) goes to
// gathered row sc_start[owner] + tag (the tag = its index among this rank's requests to
// that owner, written by the owner's patch gather).  One lane group moves one row.
__global__ __launch_bounds__(kBlock) void patch_scatter_kernel(int D, const unsigned char* recv, long long rb,
                                                               int W, const int* recv_off, const int* sc_start,
                                                               unsigned char* gathered) {
  constexpr int LPR = 16;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nunits = (int)(rb / 16);
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  for (int p = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; p < D; p += ngroups) {
    const unsigned char* src = recv + (long long)p * rb;
    int q = 0;
    while (q + 1 < W && recv_off[q + 1] <= p) ++q;
    const int tag = reinterpret_cast<const int*>(src + rb - 4)[0];
    unsigned char* dst = gathered + (long long)(sc_start[q] + tag) * rb;
    for (int u = t; u < nunits; u += LPR)
      reinterpret_cast<uint4*>(dst)[u] = reinterpret_cast<const uint4*>(src)[u];
  }
}

int launch_dirty_scan(int R, const int* req, int W, const int* run_off, int Wp, const int* prev_off, const int* prev,
                      int* flag, int* dcount, int skip0, int skip1, hipStream_t st) {
  if (W > kMaxRuns) return -8;
  (void)hipMemsetAsync(dcount, 0, sizeof(int) * W, st);
  if (R <= 0) return 0;
  hipLaunchKernelGGL(dirty_scan_kernel, dim3(fill_grid(R, kBlock, 2048)), dim3(kBlock), 0, st, R, req, W, run_off,
                     Wp, prev_off, prev, flag, dcount, skip0, skip1);
  return (int)hipGetLastError();
}

// Self rows of the row-sharded step: run `me` of the received requests is this rank's own
// requests; excl[i] = 1 when no other run (source rank) requested the same row this step,
// so the whole gradient of the row is this rank's and its backward can apply it in place.
__global__ __launch_bounds__(kBlock) void self_excl_kernel(const int* req, int W, const int* run_off, int me,
                                                           int* excl) {
  const int i0 = run_off[me], n = run_off[me + 1] - i0;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const int key = req[i0 + i];
    int hit = 0;
    for (int q = 0; q < W && !hit; ++q) {
      if (q == me) continue;
      int lo = run_off[q];
      const int end = run_off[q + 1];
      int hi = end;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (req[mid] < key) lo = mid + 1; else hi = mid;
      }
      hit = lo < end && req[lo] == key;
    }
    excl[i] = !hit;
  }
}

int launch_self_excl(const int* req, int W, const int* run_off, int me, int n, int* excl, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(self_excl_kernel, dim3(fill_grid(n, kBlock, 4096)), dim3(kBlock), 0, st, req, W, run_off, me,
                     excl);
  return (int)hipGetLastError();
}

size_t select_workspace_bytes(int n) {
  size_t b = 0;
  (void)rocprim::select((void*)nullptr, b, rocprim::counting_iterator<int>(0), (const int*)nullptr, (int*)nullptr,
                        (int*)nullptr, (size_t)n, (hipStream_t)0);
  return b;
}

// Stream compaction of the flagged positions (ascending): out[0..count) = i with flag[i] != 0.
int launch_select_flagged(int n, const int* flag, int* out, int* count, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return (int)hipMemsetAsync(count, 0, sizeof(int), st);
  size_t b = ws_bytes;
  return (int)rocprim::select(ws, b, rocprim::counting_iterator<int>(0), flag, out, count, (size_t)n, st);
}

int launch_patch_scatter(int D, const unsigned char* recv, long long rb, int W, const int* recv_off,
                         const int* sc_start, unsigned char* gathered, hipStream_t st) {
  if (D <= 0) return 0;
  if (rb % 16) return -9;
  hipLaunchKernelGGL(patch_scatter_kernel, dim3(fill_grid(D, kWavesPerBlock * 4)), dim3(kBlock), 0, st, D, recv, rb,
                     W, recv_off, sc_start, gathered);
  return (int)hipGetLastError();
}

int launch_run_member(int R, const int* req, int W, const int* run_off, const int* prev, int* flag,
                      hipStream_t st) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(run_member_kernel, dim3(fill_grid(R, kBlock, 8192)), dim3(kBlock), 0, st, R, req, W, run_off,
                     prev, flag);
  return (int)hipGetLastError();
}

template <int LPR, typename TV, int EW = 0>
__global__ __launch_bounds__(kBlock) void apply_runs_kernel(ApplyArgs a) {
  const uint32_t sr = sr_step_seed(a.sr_counter);  // stochastic rounding seed (0: nearest)
  constexpr int EPL = EW ? EW : Frag<TV>::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  for (int i = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; i < a.R; i += ngroups) {
    int r = 0;
    const int* mrow = nullptr;
    if (a.W > 1) while (a.run_off[r + 1] <= i) ++r;
    if (r == a.self_run && (a.self_excl == nullptr || a.self_excl[i - a.run_off[r]])) continue;  // done in place
    if (a.W > 1) {
      mrow = a.match + (long long)i * a.W;
      bool led = true;
      for (int q = 0; q < r; ++q) led &= mrow[q] < 0;
      if (!led) continue;  // an earlier run holds this row: its leader applies it
    }
    const long long row = a.req[i];
    RowUpdate<LPR, TV, EW> ru;
    ru.load(a, row, tE);
    float gr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] = 0.f;
    float gw = 0.f;
    add_grad_row<EPL>(a, a.grad_in + (long long)i * a.g_stride, tE, gr, gw);
    for (int q = r + 1; q < a.W; ++q) {
      const int j = mrow[q];
      if (j >= 0) add_grad_row<EPL>(a, a.grad_in + (long long)j * a.g_stride, tE, gr, gw);
    }
    ru.step_store(a, gr, gw, row, t, tact, sr);
  }
}

// Replicated-table (data-parallel) update from a dense, all-reduced gradient buffer:
// one lane group per buffer row; rows without the touch marker are all zero and
// skipped; a touched row gets one optimizer step and is zeroed for the next step, so
// the buffer is never cleared wholesale (reads: one word per untouched row).
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void dense_apply_kernel(ApplyArgs a) {
  const uint32_t sr = sr_step_seed(a.sr_counter);
  constexpr int EPL = Frag<TV>::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  for (int i = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; i < a.R; i += ngroups) {
    const float* grow = a.grad_in + (long long)i * a.g_stride;
    if (grow[a.touch_col] == 0.f) continue;  // (group-uniform)
    const long long row = a.row0 + i;
    RowUpdate<LPR, TV> ru;
    ru.load(a, row, tE);
    float gr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] = 0.f;
    float gw = 0.f;
    add_grad_row<EPL>(a, grow, tE, gr, gw);
    ru.step_store(a, gr, gw, row, t, tact, sr);
    if (a.grad_zero) {
      float4* z = reinterpret_cast<float4*>(a.grad_zero + (long long)i * a.g_stride);
      const int nq = (int)(a.g_stride / 4);
      for (int q = t; q < nq; q += LPR) z[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

int launch_dense_apply(const ApplyArgs& a, int dtype, hipStream_t st) {
  if (a.R <= 0) return 0;
  if (a.g_stride % 4 != 0 || a.touch_col >= a.g_stride) return -7;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int grid = fill_grid(a.R, kWavesPerBlock * (kWave / lpr), 16384);
  FM_DISPATCH(dtype, lpr, dense_apply_kernel, grid, st, a);
  return (int)hipGetLastError();
}

int launch_gather_rows(const GatherArgs& a, int dtype, hipStream_t st) {
  if (a.R <= 0) return 0;
  if (a.skip1 < a.skip0 || a.skip0 < 0 || a.skip1 > a.R) return -10;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int grid = fill_grid(std::max(1, a.R - (a.skip1 - a.skip0)), kWavesPerBlock * (kWave / lpr));
  FM_DISPATCH(dtype, lpr, gather_rows_kernel, grid, st, a);
  return (int)hipGetLastError();
}

int launch_apply_runs(const ApplyArgs& a, int* match, int dtype, hipStream_t st) {
  if (a.R <= 0) return 0;
  if (a.W > 1) {
    const long long n = (long long)a.R * a.W;
    hipLaunchKernelGGL(owner_match_kernel, dim3(fill_grid(n, kBlock, 16384)), dim3(kBlock), 0, st, a.R, a.W,
                       a.run_off, a.req, match);
  }
  const int lpr = lanes_per_row(a.Kp, dtype);
#ifndef FM_FP8_WIDE_APPLY
#define FM_FP8_WIDE_APPLY FM_FP8_WIDE  // (the owner apply alone: the "fp8narrowapply" variant, A/B)
#endif
#if FM_FP8_WIDE_APPLY
  // wide fp8 rows (k = 128: 16 lanes x 8 values; rows, state and gradient rows 8 / 16-byte aligned)
  if (dtype == kFP8 && lpr == 32 && a.Kp % 8 == 0 && a.v_stride % 8 == 0 && a.s_stride % 8 == 0 && a.g_stride % 4 == 0 &&
      (uintptr_t)a.v % 8 == 0 && (uintptr_t)a.s0v % 16 == 0 && (uintptr_t)a.s1v % 16 == 0 &&
      (uintptr_t)a.grad_in % 16 == 0) {
    const int grid = fill_grid(a.R, kWavesPerBlock * (kWave / 16));
    hipLaunchKernelGGL((apply_runs_kernel<16, fp8e4m3, 8>), dim3(grid), dim3(kBlock), 0, st, a);
    return (int)hipGetLastError();
  }
#endif
  const int grid = fill_grid(a.R, kWavesPerBlock * (kWave / lpr));
  FM_DISPATCH(dtype, lpr, apply_runs_kernel, grid, st, a);
  return (int)hipGetLastError();
}

int launch_apply_rows(const ApplyArgs& a, int dtype, long long max_unique, hipStream_t st) {
  if (max_unique <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int grid = fill_grid(max_unique, kWavesPerBlock * (kWave / lpr));
  FM_DISPATCH(dtype, lpr, apply_rows_kernel, grid, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm

namespace fm {

// Per-owner number of unique keys for the row-sharded exchange. The unique
// keys are sorted and encode owner * Rps + local_row, so owner w's requests are
// the contiguous run [lower_bound(w*Rps), lower_bound((w+1)*Rps)).  Reads U
// from the device: no host sync between the dedup and the count all-to-all.
// One wave per owner, a 64-way search: each round every lane tests one of 64 evenly spaced
// pivots and the ballot's popcount narrows [lo, hi) 64-fold, so a bound costs ~log64(U)
// dependent loads (3-4 at U ~ 400k) instead of a scalar binary search's ~19 (22 -> see
// profiles/r4/shard_w1_local.txt).
__device__ __forceinline__ int wave_lower_bound(const uint32_t* uniq, int U, unsigned long long key, int lane) {
  int lo = 0, hi = U;
  while (hi - lo > kWave) {
    const int step = (hi - lo + kWave - 1) / kWave;
    const int p = lo + (lane + 1) * step - 1;
    const bool below = p < hi && (unsigned long long)uniq[p] < key;
    const int c = __popcll(__ballot(below));
    // pivots 0..c-1 are below key (sorted): the bound lies in (lo + c*step - 1, lo + (c+1)*step - 1]
    const int nlo = lo + c * step;
    hi = min(hi, nlo + step);
    lo = nlo;
  }
  const int p = lo + lane;
  const bool below = p < hi && (unsigned long long)uniq[p] < key;
  return lo + __popcll(__ballot(below));
}

__global__ __launch_bounds__(kWave) void owner_counts_kernel(const uint32_t* uniq, const int* num_unique,
                                                             long long Rps, int W, long long* out, long long stride,
                                                             long long* out2) {
  const int w = blockIdx.x;
  const int lane = threadIdx.x;
  const int U = *num_unique;
  const int a = wave_lower_bound(uniq, U, (unsigned long long)w * Rps, lane);
  const int b = wave_lower_bound(uniq, U, (unsigned long long)(w + 1) * Rps, lane);
  if (lane == 0) {
    out[w * stride] = b - a;
    if (out2) out2[w * stride] = b - a;
  }
}

// Sharded key of every occurrence: owner (id % W) major, local row (id / W) minor,
// so that a sort groups each owner's requests contiguously.
__global__ void shard_keys_kernel(int n, const int* ids, int W, int Rps, int* keys) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int id = ids[i];
    keys[i] = (id % W) * Rps + id / W;
  }
}

int launch_shard_keys(int n, const int* ids, int W, int Rps, int* keys, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shard_keys_kernel, dim3(fill_grid(n, kBlock, 4096)), dim3(kBlock), 0, st, n, ids, W, Rps, keys);
  return (int)hipGetLastError();
}

// out[w * stride] (and out2[w * stride], nullable: the world-1 count exchange's received copy)
int launch_owner_counts(const uint32_t* uniq, const int* num_unique, long long Rps, int W, long long* out,
                        hipStream_t st, long long stride = 1, long long* out2 = nullptr) {
  if (W <= 0 || stride < 1) return 0;
  hipLaunchKernelGGL(owner_counts_kernel, dim3(W), dim3(kWave), 0, st, uniq, num_unique, Rps, W, out, stride, out2);
  return (int)hipGetLastError();
}

// Zero the rows buf[list[i]] for i < *count (device count, capped at max_n): the data-parallel
// dense step's gradient buffer keeps this rank's scattered rows of the slices other ranks own
// after its in-place reduce-scatter; they are cleared here instead of the whole buffer.  One
// wave per row, 16 bytes per lane (row_words a multiple of 4).
__global__ __launch_bounds__(kBlock) void zero_listed_rows_kernel(float* buf, long long row_words, const int* list,
                                                                 const int* count, int max_n) {
  const int n = min(*count, max_n);
  const int lane = threadIdx.x & (kWave - 1);
  const int nq = (int)(row_words / 4);
  for (int i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); i < n; i += gridDim.x * kWavesPerBlock) {
    float4* r = reinterpret_cast<float4*>(buf + (long long)list[i] * row_words);
    for (int q = lane; q < nq; q += kWave) r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

int launch_zero_listed_rows(float* buf, long long row_words, const int* list, const int* count, int max_n,
                            hipStream_t st) {
  if (max_n <= 0) return 0;
  if (row_words % 4 != 0) return -1;
  hipLaunchKernelGGL(zero_listed_rows_kernel, dim3(fill_grid(max_n, kWavesPerBlock, 4096)), dim3(kBlock), 0, st, buf,
                     row_words, list, count, max_n);
  return (int)hipGetLastError();
}

}  // namespace fm
