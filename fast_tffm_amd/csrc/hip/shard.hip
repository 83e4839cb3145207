// Owner-side kernels of the row-sharded exchange (parallel/exchange.py):
// gather requested table rows into a packed [v | w | pad] send buffer, and sum
// the gradient rows every peer returned for one table row before applying the
// optimizer once (replaces the PS-side embedding gather and SparseApplyAdagrad
// that the reference gets from TF's gRPC runtime, tffm/fm_model.py:291, :341-348).
#include "fm_common.h"

namespace fm {

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
  for (int p = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; p < a.R; p += ngroups) {
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

struct ApplyArgs {
  const int* num_unique;    // device scalar: number of distinct rows received
  const int* seg_start;     // [U+1] into perm
  const int* uniq;          // [U] local table row
  const int* perm;          // [R] position in grad_in of each sorted entry
  const float* grad_in; long long g_stride;  // [R, g_stride], w-grad at column Kp
  int Kp;
  void* v; long long v_stride;
  float* w; long long w_stride;
  float* s0v; float* s1v; long long s_stride;
  float* s0w; float* s1w;
  OptParams opt;
};

// Owner-side: sum the gradient rows every peer sent for one table row (in
// source-rank order: the sort is stable and the receive buffer is rank-major)
// and apply the optimizer once.
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void apply_rows_kernel(ApplyArgs a) {
  using F = Frag<TV>;
  constexpr int EPL = F::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int U = *a.num_unique;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  for (int u = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; u < U; u += ngroups) {
    // table row + optimizer state first: their loads overlap the gradient sum below
    const long long row = a.uniq[u];
    TV* vrow = reinterpret_cast<TV*>(a.v) + row * a.v_stride + tE * EPL;
    float vv[EPL], st0[EPL], st1[EPL];
    F::load(vrow, vv);
    if constexpr (F::kScaled) {
      const float s = row_scale<TV>(a.w, row, a.w_stride);
#pragma unroll
      for (int k = 0; k < EPL; ++k) vv[k] *= s;
    }
    float* s0 = a.s0v + row * a.s_stride + tE * EPL;
    float* s1 = a.s1v ? a.s1v + row * a.s_stride + tE * EPL : nullptr;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 q = *reinterpret_cast<const float4*>(s0 + k);
      st0[k] = q.x; st0[k + 1] = q.y; st0[k + 2] = q.z; st0[k + 3] = q.w;
      const float4 z = s1 ? *reinterpret_cast<const float4*>(s1 + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      st1[k] = z.x; st1[k + 1] = z.y; st1[k + 2] = z.z; st1[k + 3] = z.w;
    }
    float* wp = a.w + row * a.w_stride;
    float pw = *wp, q0 = a.s0w[row], q1 = a.s1w ? a.s1w[row] : 0.f;
    float gr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] = 0.f;
    float gw = 0.f;
    const int j1 = a.seg_start[u + 1];
    for (int j = a.seg_start[u]; j < j1; ++j) {
      const float* src = a.grad_in + (long long)a.perm[j] * a.g_stride;
#pragma unroll
      for (int k = 0; k < EPL; k += 4) {
        const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
        gr[k] += f.x; gr[k + 1] += f.y; gr[k + 2] += f.z; gr[k + 3] += f.w;
      }
      gw += src[a.Kp];
    }
#pragma unroll
    for (int k = 0; k < EPL; ++k) opt_step(a.opt, gr[k], vv[k], st0[k], st1[k]);
    store_row<LPR, TV>(vrow, vv, a.w, row, a.w_stride, t, tact);
    if (tact) {
#pragma unroll
      for (int k = 0; k < EPL; k += 4) {
        *reinterpret_cast<float4*>(s0 + k) = make_float4(st0[k], st0[k + 1], st0[k + 2], st0[k + 3]);
        if (s1) *reinterpret_cast<float4*>(s1 + k) = make_float4(st1[k], st1[k + 1], st1[k + 2], st1[k + 3]);
      }
    }
    if (t == 0) {
      opt_step(a.opt, gw, pw, q0, q1);
      *wp = pw;
      a.s0w[row] = q0;
      if (a.s1w) a.s1w[row] = q1;
    }
  }
}

int launch_gather_rows(const GatherArgs& a, int dtype, hipStream_t st) {
  if (a.R <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int grid = fill_grid(a.R, kWavesPerBlock * (kWave / lpr));
  FM_DISPATCH(dtype, lpr, gather_rows_kernel, grid, st, a);
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
__global__ void owner_counts_kernel(const uint32_t* uniq, const int* num_unique, long long Rps, int W,
                                    long long* out) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const int U = *num_unique;
  auto lower = [&](unsigned long long key) {
    int lo = 0, hi = U;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((unsigned long long)uniq[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  out[w] = lower((unsigned long long)(w + 1) * Rps) - lower((unsigned long long)w * Rps);
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

int launch_owner_counts(const uint32_t* uniq, const int* num_unique, long long Rps, int W, long long* out,
                        hipStream_t st) {
  hipLaunchKernelGGL(owner_counts_kernel, dim3((W + 63) / 64), dim3(64), 0, st, uniq, num_unique, Rps, W, out);
  return (int)hipGetLastError();
}

}  // namespace fm
