// gfx950 kernels for the FM hot path: fused forward(+loss), fused
// segmented backward + sparse optimizer step, and the row gather / row apply
// pair used by the row-sharded (all-to-all) mode.
//
// Parity map (reference -> here):
//   FmScorer  cc/fm_scorer_op.h:8-140  (BiasGenerator, FeatureRankGenerator,
//             pred/reg reductions)                       -> fm_fwd_kernel
//   loss ops  tffm/fm_model.py:311-333                   -> fm_fwd_kernel epilogue
//   FmGrad    cc/fm_grad_op.h:23-163   (FactorSum recompute, zero-fill,
//             168M atomicAdd scatter)                    -> fm_bwd_chunk_kernel +
//                                                           fm_bwd_combine_kernel
//   SparseApplyAdagrad [TF-lib] fm_model.py:341-348      -> opt_step in the
//                                                           backward epilogue
//
// Design (MI355X-first, not a translation):
//  * forward: one wave64 per example; the example's (row, value) pairs are
//    loaded once, lane-parallel, and broadcast with ds_bpermute; factor rows
//    are fetched 16 B per lane, G = 64/LPR rows per wave instruction, UNR row
//    groups in flight per lane; r1 = sum x*v is cached for the backward (the
//    reference recomputes it, G5) and the loss gradient dpred is emitted by
//    the same kernel (T6).
//  * backward: occurrences were sorted by table row (dedup.hip); each row's
//    occurrence list is cut into chunks of <= CH that one lane group reduces
//    in registers; single-chunk rows apply the optimizer immediately, long
//    (hot-id) rows are summed from per-chunk partials by a second kernel in
//    chunk order.  No float atomics, bitwise run-to-run deterministic.
#include "fm_common.h"
#include "../hash64.h"

namespace fm {

struct FwdArgs {
  int B;
  const int* offsets;   // [B+1] CSR offsets into rows/vals
  const int* rows;      // [nnz] row index into the v/w sources
  const float* vals;    // [nnz] feature values, nullptr => all 1
  const void* v;        // factor rows (TV), v_stride elements apart
  long long v_stride;
  const float* w;       // linear weights, w_stride elements apart
  long long w_stride;
  int Kp;               // padded factor count (multiple of 16B / sizeof(TV))
  const float* labels;  // [B] (loss only)
  const float* weights; // [B] or nullptr => 1
  int loss_type;        // LossType
  float grad_scale;     // dL/dpred scale (1/B for a batch mean)
  float* pred;          // [B]
  float* r1;            // [B, Kp] fp32 or nullptr
  float* dpred;         // [B] or nullptr
  float* loss_partial;  // [gridDim.x] or nullptr
  float* reg_partial;   // [2*gridDim.x] (sum |v|^2, sum w^2) or nullptr
};

template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void fm_fwd_kernel(FwdArgs a) {
  using F = Frag<TV>;
  constexpr int EPL = F::N;
  constexpr int G = kWave / LPR;
  constexpr int UNR = (16 / G) > 1 ? (16 / G) : 1;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;        // clamped: loads never leave the row
  const float tmask = tact ? 1.f : 0.f;
  const float wmask = (t == 0) ? 1.f : 0.f;
  const TV* vbase = reinterpret_cast<const TV*>(a.v) + tE * EPL;
  const int wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * kWavesPerBlock;

  float loss_acc = 0.f, regv_acc = 0.f, regw_acc = 0.f;
  for (int i = wave; i < a.B; i += nwaves) {
    const int s = a.offsets[i], e = a.offsets[i + 1];
    float s1[EPL], s2[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
    float lin = 0.f, rv = 0.f, rw = 0.f;
    for (int base = s; base < e; base += kWave) {
      const int m = min(kWave, e - base);
      int my_row = 0;
      float my_x = 0.f;
      if (lane < m) {
        my_row = a.rows[base + lane];
        my_x = a.vals ? a.vals[base + lane] : 1.f;
      }
      for (int q = 0; q < m; q += G * UNR) {
        float fr[UNR][EPL], fw[UNR], fx[UNR], fm[UNR];
        // Unconditional loads (invalid slots re-read a valid row and are masked
        // to zero): keeps all UNR loads in flight before the first use.
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int f = q + u * G + g;
          const int row = __shfl(my_row, f & (kWave - 1), kWave);
          const float x = __shfl(my_x, f & (kWave - 1), kWave);
          fm[u] = f < m ? 1.f : 0.f;
          fx[u] = x * fm[u];
          F::load(vbase + (long long)row * a.v_stride, fr[u]);
          fw[u] = a.w[(long long)row * a.w_stride];
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const float xm = fx[u] * tmask;
          const float rm = fm[u] * tmask;
#pragma unroll
          for (int k = 0; k < EPL; ++k) {
            const float xv = xm * fr[u][k];
            s1[k] += xv;
            s2[k] += xv * xv;
            rv += rm * fr[u][k] * fr[u][k];
          }
          lin += wmask * fx[u] * fw[u];
          rw += wmask * fm[u] * fw[u] * fw[u];
        }
      }
    }
    float part = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      s1[k] = across_groups_sum<LPR>(s1[k]);
      s2[k] = across_groups_sum<LPR>(s2[k]);
      part += s1[k] * s1[k] - s2[k];
    }
    part = group_sum<LPR>(part);
    lin = group_sum<kWave>(lin);
    const float pred = lin + 0.5f * part;
    if (a.r1 != nullptr && g == 0 && tact) {
      float* dst = a.r1 + (long long)i * a.Kp + t * EPL;
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<float4*>(dst + k) = make_float4(s1[k], s1[k + 1], s1[k + 2], s1[k + 3]);
    }
    if (a.reg_partial != nullptr) {
      rv = group_sum<kWave>(rv);
      rw = group_sum<kWave>(rw);
      regv_acc += rv;
      regw_acc += rw;
    }
    if (lane == 0) {
      a.pred[i] = pred;
      if (a.loss_type != kLossNone) {
        const float y = a.labels[i];
        const float wt = a.weights ? a.weights[i] : 1.f;
        float l, d;
        if (a.loss_type == kLossMse) {
          const float diff = pred - y;
          l = wt * diff * diff;
          d = 2.f * wt * diff;
        } else {
          // sigmoid_cross_entropy_with_logits, numerically stable form
          l = wt * (fmaxf(pred, 0.f) - pred * y + softplus_neg_abs(pred));
          d = wt * (sigmoidf(pred) - y);
        }
        loss_acc += l;
        if (a.dpred) a.dpred[i] = d * a.grad_scale;
      }
    }
  }
  if (a.loss_partial == nullptr && a.reg_partial == nullptr) return;
  __shared__ float red[3][kWavesPerBlock];
  const int wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = loss_acc;
    red[1][wv] = regv_acc;
    red[2][wv] = regw_acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, r0 = 0.f, r1v = 0.f;
    for (int k = 0; k < kWavesPerBlock; ++k) { l += red[0][k]; r0 += red[1][k]; r1v += red[2][k]; }
    if (a.loss_partial) a.loss_partial[blockIdx.x] = l;
    if (a.reg_partial) { a.reg_partial[2 * blockIdx.x] = r0; a.reg_partial[2 * blockIdx.x + 1] = r1v; }
  }
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
enum BwdMode : int { kBwdLocal = 0, kBwdEmit = 1 };

struct BwdArgs {
  int mode;                 // BwdMode
  const int* num_chunks;    // device scalar
  const int* chunk_seg;     // [chunks] -> segment id
  const int* chunk_start;   // [U+1] first chunk of each segment
  const int* num_unique;    // device scalar U
  const int* seg_start;     // [U+1] into the sorted occurrence arrays
  const int* uniq;          // [U] table row of each segment (LOCAL)
  const int* sorted_ex;     // [nnz] example index of each sorted occurrence
  const float* sorted_x;    // [nnz] value of each sorted occurrence or nullptr
  const float* dpred;       // [B]
  const float* r1;          // [B, Kp]
  int Kp, CH;
  void* v;                  // LOCAL: table (read/write); EMIT: gathered rows (read)
  long long v_stride;
  float* w;
  long long w_stride;
  float* s0v;               // optimizer state, same row layout as v (fp32)
  float* s1v;
  long long s_stride;
  float* s0w;
  float* s1w;
  float reg_v, reg_w;       // lambda_f * reg_grad, lambda_b * reg_grad
  OptParams opt;
  float* grad_out;          // EMIT: [U, g_stride], w-grad at column Kp
  long long g_stride;
  float* partial;           // [chunks, Kp + 4]
};

template <typename TV, int EPL>
__device__ inline void bwd_finalize(const BwdArgs& a, int u, int t, bool tact, int tE,
                                    const float (&A)[EPL], float Scx, float Sc, int n_u) {
  using F = Frag<TV>;
  const long long row = (a.mode == kBwdLocal) ? (long long)a.uniq[u] : (long long)u;
  TV* vrow = reinterpret_cast<TV*>(a.v) + row * a.v_stride + tE * EPL;
  float vv[EPL];
  F::load(vrow, vv);
  float* wp = a.w + row * a.w_stride;
  const float wv = *wp;
  const float nreg_v = a.reg_v * (float)n_u, nreg_w = a.reg_w * (float)n_u;
  float gr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) gr[k] = A[k] - Scx * vv[k] + nreg_v * vv[k];
  const float gw = Sc + nreg_w * wv;
  if (a.mode == kBwdEmit) {
    float* dst = a.grad_out + (long long)u * a.g_stride;
    if (tact) {
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(gr[k], gr[k + 1], gr[k + 2], gr[k + 3]);
    }
    if (t == 0) dst[a.Kp] = gw;
    return;
  }
  // LOCAL: optimizer step in place.
  float* s0 = a.s0v + row * a.s_stride + tE * EPL;
  float* s1 = a.s1v ? a.s1v + row * a.s_stride + tE * EPL : nullptr;
  float st0[EPL], st1[EPL];
#pragma unroll
  for (int k = 0; k < EPL; k += 4) {
    const float4 q = *reinterpret_cast<const float4*>(s0 + k);
    st0[k] = q.x; st0[k + 1] = q.y; st0[k + 2] = q.z; st0[k + 3] = q.w;
    if (s1) {
      const float4 z = *reinterpret_cast<const float4*>(s1 + k);
      st1[k] = z.x; st1[k + 1] = z.y; st1[k + 2] = z.z; st1[k + 3] = z.w;
    } else {
      st1[k] = st1[k + 1] = st1[k + 2] = st1[k + 3] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < EPL; ++k) opt_step(a.opt, gr[k], vv[k], st0[k], st1[k]);
  if (tact) {
    F::store(vrow, vv);
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      *reinterpret_cast<float4*>(s0 + k) = make_float4(st0[k], st0[k + 1], st0[k + 2], st0[k + 3]);
      if (s1) *reinterpret_cast<float4*>(s1 + k) = make_float4(st1[k], st1[k + 1], st1[k + 2], st1[k + 3]);
    }
  }
  if (t == 0) {
    float p = wv, q0 = a.s0w[row], q1 = a.s1w ? a.s1w[row] : 0.f;
    opt_step(a.opt, gw, p, q0, q1);
    *wp = p;
    a.s0w[row] = q0;
    if (a.s1w) a.s1w[row] = q1;
  }
}

// One lane group (LPR lanes) per chunk of <= CH sorted occurrences.
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void fm_bwd_chunk_kernel(BwdArgs a) {
  constexpr int EPL = Frag<TV>::N;
  constexpr int G = kWave / LPR;
  constexpr int UNR = 4;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int nchunks = *a.num_chunks;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  const int group0 = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g;
  // all lanes of a wave must run the same number of outer iterations (shuffle-free
  // loop body, but keep the trip count uniform for clean exec masks)
  for (int cbase = group0 - g; cbase < nchunks; cbase += ngroups) {
    const int c = cbase + g;
    if (c >= nchunks) continue;
    const int u = a.chunk_seg[c];
    const int c0 = a.chunk_start[u];
    const int nc = a.chunk_start[u + 1] - c0;
    const int sa = a.seg_start[u], sb = a.seg_start[u + 1];
    const int j0 = sa + (c - c0) * a.CH;
    const int j1 = min(sb, j0 + a.CH);
    float A[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) A[k] = 0.f;
    float Scx = 0.f, Sc = 0.f;
    for (int j = j0; j < j1; j += UNR) {
      float rr[UNR][EPL], cc[UNR], xx[UNR];
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
        const int jj = j + q;
        const bool ok = jj < j1;
        const int jc = ok ? jj : j1 - 1;
        const int ex = a.sorted_ex[jc];
        const float x = a.sorted_x ? a.sorted_x[jc] : 1.f;
        const float d = a.dpred[ex];
        cc[q] = ok ? d * x : 0.f;
        xx[q] = x;
        const float* src = a.r1 + (long long)ex * a.Kp + tE * EPL;
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          const float4 f = *reinterpret_cast<const float4*>(src + k);
          rr[q][k] = f.x; rr[q][k + 1] = f.y; rr[q][k + 2] = f.z; rr[q][k + 3] = f.w;
        }
      }
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) A[k] += cc[q] * rr[q][k];
        Scx += cc[q] * xx[q];
        Sc += cc[q];
      }
    }
    if (nc == 1) {
      bwd_finalize<TV, EPL>(a, u, t, tact, tE, A, Scx, Sc, sb - sa);
    } else {
      float* dst = a.partial + (long long)c * (a.Kp + 4);
      if (tact) {
#pragma unroll
        for (int k = 0; k < EPL; k += 4)
          *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(A[k], A[k + 1], A[k + 2], A[k + 3]);
      }
      if (t == 0) { dst[a.Kp] = Scx; dst[a.Kp + 1] = Sc; }
    }
  }
}

// One lane group per multi-chunk segment: ordered sum of its chunk partials.
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void fm_bwd_combine_kernel(BwdArgs a) {
  constexpr int EPL = Frag<TV>::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int U = *a.num_unique;
  const int ngroups = gridDim.x * kWavesPerBlock * G;
  const int group0 = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g;
  for (int u = group0; u < U; u += ngroups) {
    const int c0 = a.chunk_start[u], c1 = a.chunk_start[u + 1];
    if (c1 - c0 <= 1) continue;
    float A[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) A[k] = 0.f;
    float Scx = 0.f, Sc = 0.f;
    for (int c = c0; c < c1; ++c) {
      const float* src = a.partial + (long long)c * (a.Kp + 4);
#pragma unroll
      for (int k = 0; k < EPL; k += 4) {
        const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
        A[k] += f.x; A[k + 1] += f.y; A[k + 2] += f.z; A[k + 3] += f.w;
      }
      Scx += src[a.Kp];
      Sc += src[a.Kp + 1];
    }
    bwd_finalize<TV, EPL>(a, u, t, tact, tE, A, Scx, Sc, a.seg_start[u + 1] - a.seg_start[u]);
  }
}

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
    float gr[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) gr[k] = 0.f;
    float gw = 0.f;
    for (int j = a.seg_start[u]; j < a.seg_start[u + 1]; ++j) {
      const float* src = a.grad_in + (long long)a.perm[j] * a.g_stride;
#pragma unroll
      for (int k = 0; k < EPL; k += 4) {
        const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
        gr[k] += f.x; gr[k + 1] += f.y; gr[k + 2] += f.z; gr[k + 3] += f.w;
      }
      gw += src[a.Kp];
    }
    const long long row = a.uniq[u];
    TV* vrow = reinterpret_cast<TV*>(a.v) + row * a.v_stride + tE * EPL;
    float vv[EPL], st0[EPL], st1[EPL];
    F::load(vrow, vv);
    float* s0 = a.s0v + row * a.s_stride + tE * EPL;
    float* s1 = a.s1v ? a.s1v + row * a.s_stride + tE * EPL : nullptr;
#pragma unroll
    for (int k = 0; k < EPL; ++k) { st0[k] = s0[k]; st1[k] = s1 ? s1[k] : 0.f; }
#pragma unroll
    for (int k = 0; k < EPL; ++k) opt_step(a.opt, gr[k], vv[k], st0[k], st1[k]);
    if (tact) {
      F::store(vrow, vv);
#pragma unroll
      for (int k = 0; k < EPL; ++k) { s0[k] = st0[k]; if (s1) s1[k] = st1[k]; }
    }
    if (t == 0) {
      float* wp = a.w + row * a.w_stride;
      float p = *wp, q0 = a.s0w[row], q1 = a.s1w ? a.s1w[row] : 0.f;
      opt_step(a.opt, gw, p, q0, q1);
      *wp = p;
      a.s0w[row] = q0;
      if (a.s1w) a.s1w[row] = q1;
    }
  }
}

// Expand CSR offsets into the example index of every occurrence.
__global__ __launch_bounds__(kBlock) void csr_rows_kernel(int B, const int* offsets, int* ex_of_occ) {
  const int lane = threadIdx.x & (kWave - 1);
  const int nwaves = gridDim.x * kWavesPerBlock;
  for (int i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); i < B; i += nwaves) {
    const int s = offsets[i], e = offsets[i + 1];
    for (int j = s + lane; j < e; j += kWave) ex_of_occ[j] = i;
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
static int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }

int lanes_per_row(int Kp, int dtype) {
  const int epl = dtype == kBF16 ? 8 : 4;
  return next_pow2((Kp + epl - 1) / epl);
}

static int fill_grid(long long work_groups, int groups_per_block, int cap = 8192) {
  long long blocks = (work_groups + groups_per_block - 1) / groups_per_block;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  return (int)blocks;
}

#define FM_DISPATCH_LPR(LPR_VAL, KERNEL, TV, GRID, STREAM, ARGS)                                   \
  switch (LPR_VAL) {                                                                                \
    case 1: hipLaunchKernelGGL((KERNEL<1, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break;  \
    case 2: hipLaunchKernelGGL((KERNEL<2, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break;  \
    case 4: hipLaunchKernelGGL((KERNEL<4, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break;  \
    case 8: hipLaunchKernelGGL((KERNEL<8, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break;  \
    case 16: hipLaunchKernelGGL((KERNEL<16, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break; \
    case 32: hipLaunchKernelGGL((KERNEL<32, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break; \
    case 64: hipLaunchKernelGGL((KERNEL<64, TV>), dim3(GRID), dim3(kBlock), 0, STREAM, ARGS); break; \
    default: return -1;                                                                             \
  }

#define FM_DISPATCH(DTYPE, LPR_VAL, KERNEL, GRID, STREAM, ARGS)                       \
  if ((DTYPE) == kBF16) {                                                            \
    FM_DISPATCH_LPR(LPR_VAL, KERNEL, __hip_bfloat16, GRID, STREAM, ARGS)             \
  } else {                                                                           \
    FM_DISPATCH_LPR(LPR_VAL, KERNEL, float, GRID, STREAM, ARGS)                      \
  }

int fwd_grid(int B) { return fill_grid(B, kWavesPerBlock, 4096); }

int launch_fwd(const FwdArgs& a, int dtype, int grid, hipStream_t st) {
  if (a.B <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  FM_DISPATCH(dtype, lpr, fm_fwd_kernel, grid, st, a);
  return (int)hipGetLastError();
}

int launch_bwd(const BwdArgs& a, int dtype, long long max_chunks, long long max_unique, hipStream_t st) {
  if (max_chunks <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int G = kWave / lpr;
  const int g1 = fill_grid(max_chunks, kWavesPerBlock * G);
  FM_DISPATCH(dtype, lpr, fm_bwd_chunk_kernel, g1, st, a);
  const int g2 = fill_grid(max_unique, kWavesPerBlock * G, 2048);
  FM_DISPATCH(dtype, lpr, fm_bwd_combine_kernel, g2, st, a);
  return (int)hipGetLastError();
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

int launch_csr_rows(int B, const int* offsets, int* ex_of_occ, hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(csr_rows_kernel, dim3(fill_grid(B, kWavesPerBlock, 4096)), dim3(kBlock), 0, st, B,
                     offsets, ex_of_occ);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Table init (reference fm_model.py:278-281: U(-r, r) over all K+1 columns).
// Counter-based: the value of (global id g, reference column c) depends only on
// (seed, g, c), so a table sharded over any world size -- or restored into
// another layout -- starts from bit-identical parameters.
// ---------------------------------------------------------------------------
__device__ inline float init_uniform(unsigned long long seed, long long gid, int col, float range) {
  const unsigned long long h = mix64(seed ^ mix64((unsigned long long)gid * 0x100000001b3ull + (unsigned long long)col));
  const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0, 1)
  return range * (2.f * u - 1.f);
}

struct InitArgs {
  void* v; long long v_stride; float* w; long long w_stride;
  long long rows; int K, Kp, dtype;
  long long gid_mul, gid_add;    // global id of local row r = r * gid_mul + gid_add
  unsigned long long seed; float range;
};

__global__ __launch_bounds__(kBlock) void init_rows_kernel(InitArgs a) {
  const long long total = a.rows * (long long)(a.Kp + 1);
  for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < total; e += (long long)gridDim.x * kBlock) {
    const long long r = e / (a.Kp + 1);
    const int c = (int)(e - r * (a.Kp + 1));
    const long long gid = r * a.gid_mul + a.gid_add;
    if (c < a.Kp) {
      const float val = c < a.K ? init_uniform(a.seed, gid, c + 1, a.range) : 0.f;
      if (a.dtype == kBF16)
        reinterpret_cast<uint16_t*>(a.v)[r * a.v_stride + c] = (uint16_t)f32_to_bf16_bits(val);
      else
        reinterpret_cast<float*>(a.v)[r * a.v_stride + c] = val;
    } else {
      a.w[r * a.w_stride] = init_uniform(a.seed, gid, 0, a.range);
    }
  }
}

int launch_init_rows(const InitArgs& a, hipStream_t st) {
  if (a.rows <= 0) return 0;
  const long long total = a.rows * (long long)(a.Kp + 1);
  long long blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(init_rows_kernel, dim3((int)blocks), dim3(kBlock), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm
