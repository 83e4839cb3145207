// Fused FM backward + sparse optimizer step on gfx950.
//
// Parity: reference FmGrad (cc/fm_grad_op.h:23-163: FactorSum recompute,
// zero-fill, ~168M fp32 atomicAdd scatter per sample-cfg step) followed by TF's
// SparseApplyAdagrad on the parameter servers (tffm/fm_model.py:341-348).
//
// Per unique table row u with sorted occurrences (example i, value x):
//   g_v = sum c * r1_i - v * sum c*x + reg_v * n_u * v,   c = dpred_i * x
//   g_w = sum c                      + reg_w * n_u * w
// (d pred / d v = x (r1 - x v), d pred / d w = x; the per-occurrence L2 term of
// reg_score, cc/fm_grad_op.h:88-103, contributes lambda * reg_grad * param per
// occurrence).
//
// Work decomposition (no float atomics, bitwise run-to-run deterministic):
//  * dedup.hip cut the sorted occurrence array into chunks of <= CH that never
//    straddle two rows; one lane group (LPR lanes, 16 B each) reduces a chunk
//    in registers, after prefetching the chunk's (example, dpred*x) pairs
//    lane-parallel and broadcasting them with ds_bpermute;
//  * a row that fits in one chunk (the vast majority) applies the optimizer at
//    once; otherwise the chunk writes a partial row;
//  * rows split over <= kSmallChunks chunks are combined by one lane group
//    (ordered sum), hotter rows (Criteo's 3-value fields: ~40k occurrences per
//    row at B=128k) by a whole workgroup that sums the partials in a fixed
//    interleaved order and reduces through LDS; the chunk kernel lists both
//    kinds, and both combines run in one launch (fm_bwd_combine_kernel).
#include "fm_common.h"

namespace fm {

// LOCAL: parameters read from and the optimizer applied to table rows uniq[u];
// EMIT: parameters read from gathered rows u, gradient row written to grad_out[u];
// EMIT_TABLE (replicated-table data parallelism): parameters read from table rows
// uniq[u], gradient row scattered to grad_out[uniq[u]] of a persistent dense buffer
// with a touch marker (1.0) in the word after the w-gradient.
enum BwdMode : int { kBwdLocal = 0, kBwdEmit = 1, kBwdEmitTable = 2 };
constexpr int kMaxCH = 32;        // chunk length cap (prefetch registers)
constexpr int kSmallChunks = 16;  // rows with more chunks go to the workgroup combine
constexpr int kMaxPieceOwners = 64;  // owners of a split backward piece
// r1 rows in flight per lane in the chunk kernel: 8 beat 4 / 6 (fewer VGPRs, more waves) and 12 /
// 16 on k64 fp32, k64 bf16 and k128 fp8 in round 1 (profiles/r1s3/chunk_unroll_ab.txt); still the
// best for k <= 64 with the round-4 kernels, but not for k = 128 (below)
#ifndef FM_CHUNK_UNR
#define FM_CHUNK_UNR 8
#endif
constexpr int kChunkUnr = FM_CHUNK_UNR;
#ifndef FM_R1_MASK
#define FM_R1_MASK 1
#endif
#ifndef FM_CHUNK_PERM
#define FM_CHUNK_PERM 0
#endif
// The local kernels' 32-lane rows (k = 128): 12 r1 rows in flight per lane.  Same-box A/B
// (profiles/r4/chunk_unr_ab.txt): k128 fp8 FTRL 0.874 -> 0.807 ms with 12, 0.856 with 16; 16-lane and
// 4-lane rows (k64 / k16) lose with 12 or 16 (k64 fp32 0.615 -> 0.625-0.640), and so does the
// row-sharded step's general kernel (k128 fp8 at world 1 1.121 -> 1.288 ms).  FM_CHUNK_UNR32 overrides.
#ifndef FM_CHUNK_UNR32
#define FM_CHUNK_UNR32 12
#endif
// The EMIT-specialised kernel of the row-sharded step: 12 for fp8 rows (bf16 r1 rows: half the
// registers per row in flight); fp32 / bf16 rows spill 12 VGPRs at 12 under the 128-VGPR cap and
// keep 8.  FM_CHUNK_UNR32_EMIT overrides the fp8 value.
#ifndef FM_CHUNK_UNR32_EMIT
#define FM_CHUNK_UNR32_EMIT FM_CHUNK_UNR32
#endif
// The wide fp8 kernel (8 values per lane, below): 5 r1 rows in flight per lane (6 spills 6 VGPRs under
// the 128-VGPR cap, 4 one) -- about the bytes in flight of the 4-value kernel's 12.  FM_CHUNK_UNR_W8 overrides.
#ifndef FM_CHUNK_UNR_W8
#define FM_CHUNK_UNR_W8 5
#endif
template <int LPR, bool LOC, bool EMT, typename TV>
constexpr int chunk_unr() {
  return LOC && LPR == 32 ? FM_CHUNK_UNR32
         : EMT && LPR == 32 ? (R1Bf16<TV>::v ? FM_CHUNK_UNR32_EMIT : kChunkUnr)
                            : kChunkUnr;
}

struct BwdArgs {
  int mode;                 // BwdMode
  const int* counts;        // device [2]: U, #chunks
  const int* chunk_start;   // [#chunks+1] into the sorted occurrence arrays
  const int* chunk_seg;     // [#chunks] segment (row) id | kChunkFirst | kChunkSingle
  const int* chunk_key;     // [#chunks] key (= table row in LOCAL mode) of the chunk's segment
  const int* seg_start;     // [U+1]
  const int* seg_chunk;     // [U+1] first chunk of each segment
  const int* uniq;          // [U] table row of each segment (LOCAL)
  const int* sorted_ex;     // [nnz] example index of each sorted occurrence (<< ex_shift when packed)
  int ex_shift;             // > 0: sorted_ex holds packed codes (example << ex_shift | slot)
  const float* sorted_x;    // [nnz] value of each sorted occurrence or nullptr (=1)
  const float* dpred;       // [B]
  const void* r1;           // [B, Kp] fp32 (bf16 for fp8 tables: R1Bf16)
  int Kp;
  void* v;                  // LOCAL: table (read/write); EMIT: gathered rows (read)
  long long v_stride;
  float* w;
  long long w_stride;
  void* s0v;                // optimizer state, same row layout as v (fp32; bf16 for fp8 tables)
  void* s1v;
  long long s_stride;
  float* s0w;
  float* s1w;
  float reg_v, reg_w;       // lambda_f * reg_grad, lambda_b * reg_grad
  OptParams opt;
  float* grad_out;          // EMIT: [U, g_stride] 4-byte words; v-grad fp32 (or bf16), w-grad fp32 at word g_wcol
  long long g_stride;
  int g_wcol;               // word index of the w-grad in a gradient row
  int g_bf16;               // 1: v-grad stored as bf16 (the exchange's bf16 wire)
  const int* sr_counter;    // stochastic rounding of bf16 / fp8 row stores (null: round to nearest)
  int counters_ready;       // 1: counts[2] and *big_count are already 0 (fresh dedup)
  // split backward (row-sharded exchange): piece p >= 0 reduces only the segments in
  // [seg_bounds[2q + p], seg_bounds[2q + p + 1]) for every owner q < n_owners, so the
  // gradient rows of piece 0 can travel while piece 1 is computed; -1 = all segments
  const int* seg_bounds;    // [2 * n_owners + 1]
  int piece, n_owners;
  int big_blocks;           // (set by launch_bwd) fm_bwd_combine_kernel's hot-row workgroups (its first ones)
  float* partial;           // [#chunks, Kp + 4]
  int* big_list;            // [U] rows for the workgroup combine
  int* big_count;           // device scalar, zeroed by the launcher
  int* multi;               // [counts[2]] rows spanning more than one chunk (filled by the chunk kernel)
  int* counts_rw;           // == counts, writable (counts[2] = #multi, zeroed by the launcher)
  int nex;                  // examples in the batch (r1 rows)
  SelfRows self;            // EMIT (row-sharded step): segments that are this rank's own table rows
};

// Parameter row + optimizer slots of one segment, read before its gradient is
// known so that the loads overlap the occurrence reduction.
template <int EPL>
struct RowState {
  long long row;
  bool apply;               // optimizer step in place on table row `row` (else: gradient row out)
  float vv[EPL], st0[EPL], st1[EPL];
  float wv, q0, q1;
};

// Row base of `row` in a row-major array of T with `stride` elements per row: one 32 x 32 ->
// 64-bit multiply-add (rows are non-negative and < 2^31, a row's bytes < 2^32).
template <typename T>
__device__ inline T* row_ptr(T* base, long long row, long long stride) {
  using C = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return reinterpret_cast<T*>(reinterpret_cast<C*>(base) +
                              (uint64_t)(uint32_t)row * (uint32_t)(stride * (long long)sizeof(T)));
}
// Optimizer state row (fp32; bf16 for fp8 tables: StateBf16).
template <typename TV>
__device__ inline void* state_row(void* s, long long row, long long stride) {
  if constexpr (StateBf16<TV>::v) return row_ptr(reinterpret_cast<uint16_t*>(s), row, stride);
  return row_ptr(reinterpret_cast<float*>(s), row, stride);
}

// g_v of one element, A - Scx v + reg n_u v, and the occurrence sums, as fixed fma chains for the 16-bit
// and fp8 tables: the rounding is not left to the compiler's contraction, which differed between
// instantiations of different lane widths (1 ulp on rare elements: the wide fp8 kernel against the
// 4-value one) -- and the fused forms made the k = 128 bf16 FTRL step 1.025 -> 0.94 ms.  fp32 tables
// keep the plain expressions: pinned, the row-sharded step's k = 64 fp32 EMIT kernels ran 0.620 ->
// 0.666 ms (profiles/r6/fp8_wide_ab.txt); no wide fp32 kernel needs the pinned bits.
#ifndef FM_FMA_PIN
#define FM_FMA_PIN 1  // 0: plain expressions for every dtype (A/B build variant "nopin")
#endif
template <typename TV>
constexpr bool fma_pinned() { return FM_FMA_PIN && !std::is_same<TV, float>::value; }
template <typename TV>
__device__ __forceinline__ float row_grad(float A, float Scx, float nreg_v, float v) {
  if constexpr (fma_pinned<TV>()) return __builtin_fmaf(nreg_v, v, __builtin_fmaf(-Scx, v, A));
  return A - Scx * v + nreg_v * v;
}
template <typename TV>
__device__ __forceinline__ float fma_acc(float a, float b, float c) {
  if constexpr (fma_pinned<TV>()) return __builtin_fmaf(a, b, c);
  return c + a * b;
}

// LOCAL mode known at compile time (the chunk kernel's local instantiations): table row `key`,
// optimizer applied in place, 32 x 32-bit row addressing.
template <typename TV, int EPL>
__device__ inline void bwd_load_local(const BwdArgs& a, long long key, int tE, RowState<EPL>& r) {
  using F = Frag<TV>;
  r.apply = true;
  r.row = key;
  frag_load<TV, EPL>(row_ptr(reinterpret_cast<const TV*>(a.v), r.row, a.v_stride) + tE * EPL, r.vv);
  const float* wr = row_ptr(static_cast<const float*>(a.w), r.row, a.w_stride);
  r.wv = wr[0];
  if constexpr (F::kScaled) {
    const float s = wr[1];  // (row_scale)
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.vv[k] *= s;
  }
  load_state<TV, EPL>(state_row<TV>(a.s0v, r.row, a.s_stride), tE * EPL, r.st0);
  r.q0 = a.s0w[(uint32_t)r.row];
  if (a.s1v) {
    load_state<TV, EPL>(state_row<TV>(a.s1v, r.row, a.s_stride), tE * EPL, r.st1);
    r.q1 = a.s1w[(uint32_t)r.row];
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.st1[k] = 0.f;
    r.q1 = 0.f;
  }
}

template <int LPR, typename TV, int EPL>
__device__ inline void bwd_finish_local(const BwdArgs& a, int t, bool tact, RowState<EPL>& r, const float (&A)[EPL],
                                        float Scx, float Sc, int n_u, uint32_t sr) {
  const float nreg_v = a.reg_v * (float)n_u, nreg_w = a.reg_w * (float)n_u;
  float gr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) gr[k] = row_grad<TV>(A[k], Scx, nreg_v, r.vv[k]);
  const float gw = Sc + nreg_w * r.wv;
  TV* tv = reinterpret_cast<TV*>(a.v);
  opt_step_row<TV, EPL>(a.opt, gr, r.vv, r.st0, r.st1);
  store_row_e<LPR, TV, EPL>(row_ptr(tv, r.row, a.v_stride) + t * EPL, r.vv, a.w, r.row, a.w_stride, t, tact, sr);
  if (tact) {
    store_state<TV, EPL>(state_row<TV>(a.s0v, r.row, a.s_stride), t * EPL, r.st0, sr ? sr ^ kSrSalt0 : 0u,
                         (uint32_t)r.row, (uint32_t)(t * EPL));
    if (a.s1v)
      store_state<TV, EPL>(state_row<TV>(a.s1v, r.row, a.s_stride), t * EPL, r.st1, sr ? sr ^ kSrSalt1 : 0u,
                           (uint32_t)r.row, (uint32_t)(t * EPL));
  }
  if (t == 0) {
    opt_step_tv<TV>(a.opt, gw, r.wv, r.q0, r.q1);
    row_ptr(a.w, r.row, a.w_stride)[0] = r.wv;
    a.s0w[(uint32_t)r.row] = r.q0;
    if (a.s1w) a.s1w[(uint32_t)r.row] = r.q1;
  }
}

// EMIT mode known at compile time (the row-sharded step's specialised chunk kernel): segment u's
// parameters come from gathered wire row u or -- this rank's own rows -- from table row key - base,
// and an exclusive own row is updated in place; 32 x 32-bit row addressing throughout.
template <typename TV, int EPL>
__device__ inline void bwd_load_emit(const BwdArgs& a, int u, long long key, int tE, RowState<EPL>& r) {
  using F = Frag<TV>;
  const bool own = a.self.has(u);
  r.apply = own && a.self.exclusive(u);
  r.row = own ? key - a.self.base : (long long)u;
  const TV* vsrc = reinterpret_cast<const TV*>(own ? a.self.v : a.v);
  const float* wsrc = own ? a.self.w : a.w;
  frag_load<TV, EPL>(row_ptr(vsrc, r.row, own ? a.self.v_stride : a.v_stride) + tE * EPL, r.vv);
  const float* wr = row_ptr(wsrc, r.row, own ? a.self.w_stride : a.w_stride);
  r.wv = wr[0];
  if constexpr (F::kScaled) {
    const float s = wr[1];  // (row_scale)
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.vv[k] *= s;
  }
  if (!r.apply) return;
  load_state<TV, EPL>(state_row<TV>(a.s0v, r.row, a.s_stride), tE * EPL, r.st0);
  r.q0 = a.s0w[(uint32_t)r.row];
  if (a.s1v) {
    load_state<TV, EPL>(state_row<TV>(a.s1v, r.row, a.s_stride), tE * EPL, r.st1);
    r.q1 = a.s1w[(uint32_t)r.row];
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.st1[k] = 0.f;
    r.q1 = 0.f;
  }
}

template <int LPR, typename TV, int EPL>
__device__ inline void bwd_finish_emit(const BwdArgs& a, int u, int t, bool tact, RowState<EPL>& r,
                                       const float (&A)[EPL], float Scx, float Sc, int n_u, uint32_t sr) {
  const float nreg_v = a.reg_v * (float)n_u, nreg_w = a.reg_w * (float)n_u;
  float gr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) gr[k] = row_grad<TV>(A[k], Scx, nreg_v, r.vv[k]);
  const float gw = Sc + nreg_w * r.wv;
  if (!r.apply) {  // gradient row u for its owner's apply
    float* dst = row_ptr(a.grad_out, (long long)u, a.g_stride);
    if (tact) {
      if (a.g_bf16) {  // EPL bf16 values per lane (EPL * 2 bytes, 8-byte aligned)
        uint16_t* d16 = reinterpret_cast<uint16_t*>(dst) + t * EPL;
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          uint2 o;
          o.x = f32_to_bf16_bits(gr[k]) | (f32_to_bf16_bits(gr[k + 1]) << 16);
          o.y = f32_to_bf16_bits(gr[k + 2]) | (f32_to_bf16_bits(gr[k + 3]) << 16);
          *reinterpret_cast<uint2*>(d16 + k) = o;
        }
      } else {
#pragma unroll
        for (int k = 0; k < EPL; k += 4)
          *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(gr[k], gr[k + 1], gr[k + 2], gr[k + 3]);
      }
    }
    if (t == 0) dst[a.g_wcol] = gw;
    return;
  }
  // exclusive own row: the optimizer in place on this rank's table
  TV* tv = reinterpret_cast<TV*>(const_cast<void*>(a.self.v));
  opt_step_row<TV, EPL>(a.opt, gr, r.vv, r.st0, r.st1);
  store_row_e<LPR, TV, EPL>(row_ptr(tv, r.row, a.self.v_stride) + t * EPL, r.vv, a.self.w, r.row, a.self.w_stride, t,
                            tact, sr);
  if (tact) {
    store_state<TV, EPL>(state_row<TV>(a.s0v, r.row, a.s_stride), t * EPL, r.st0, sr ? sr ^ kSrSalt0 : 0u,
                         (uint32_t)r.row, (uint32_t)(t * EPL));
    if (a.s1v)
      store_state<TV, EPL>(state_row<TV>(a.s1v, r.row, a.s_stride), t * EPL, r.st1, sr ? sr ^ kSrSalt1 : 0u,
                           (uint32_t)r.row, (uint32_t)(t * EPL));
  }
  if (t == 0) {
    opt_step_tv<TV>(a.opt, gw, r.wv, r.q0, r.q1);
    row_ptr(a.self.w, r.row, a.self.w_stride)[0] = r.wv;
    a.s0w[(uint32_t)r.row] = r.q0;
    if (a.s1w) a.s1w[(uint32_t)r.row] = r.q1;
  }
}

// Parameters (and, when the row is updated here, optimizer state) of segment u with key
// `key`: LOCAL reads table row key; EMIT reads gathered row u, or -- a self row of the
// row-sharded step -- table row key - self.base, applied in place when exclusive;
// EMIT_TABLE reads table row key and scatters its gradient there.
template <typename TV, int EPL>
__device__ inline void bwd_load(const BwdArgs& a, int u, long long key, int tE, RowState<EPL>& r) {
  using F = Frag<TV>;
  const void* vsrc = a.v;
  const float* wsrc = a.w;
  long long vst = a.v_stride, wst = a.w_stride;
  r.apply = a.mode == kBwdLocal;
  r.row = a.mode == kBwdEmit ? (long long)u : key;
  if (a.mode == kBwdEmit && a.self.has(u)) {
    r.row = key - a.self.base;
    r.apply = a.self.exclusive(u);
    vsrc = a.self.v; wsrc = a.self.w; vst = a.self.v_stride; wst = a.self.w_stride;
  }
  frag_load<TV, EPL>(reinterpret_cast<const TV*>(vsrc) + r.row * vst + tE * EPL, r.vv);
  r.wv = wsrc[r.row * wst];
  if constexpr (F::kScaled) {
    const float s = row_scale<TV>(wsrc, r.row, wst);
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.vv[k] *= s;
  }
  if (!r.apply) return;
  load_state<TV, EPL>(a.s0v, r.row * a.s_stride + tE * EPL, r.st0);
  r.q0 = a.s0w[r.row];
  if (a.s1v) {
    load_state<TV, EPL>(a.s1v, r.row * a.s_stride + tE * EPL, r.st1);
    r.q1 = a.s1w[r.row];
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) r.st1[k] = 0.f;
    r.q1 = 0.f;
  }
}

template <int LPR, typename TV, int EPL>
__device__ inline void bwd_finish(const BwdArgs& a, int u, int t, bool tact, RowState<EPL>& r,
                                  const float (&A)[EPL], float Scx, float Sc, int n_u, uint32_t sr) {
  using F = Frag<TV>;
  const float nreg_v = a.reg_v * (float)n_u, nreg_w = a.reg_w * (float)n_u;
  float gr[EPL];
#pragma unroll
  for (int k = 0; k < EPL; ++k) gr[k] = row_grad<TV>(A[k], Scx, nreg_v, r.vv[k]);
  const float gw = Sc + nreg_w * r.wv;
  if (!r.apply) {
    float* dst = a.grad_out + (a.mode == kBwdEmitTable ? r.row : (long long)u) * a.g_stride;
    if (tact) {
      if (a.g_bf16) {  // EPL bf16 values per lane (EPL * 2 bytes, 8-byte aligned)
        uint16_t* d16 = reinterpret_cast<uint16_t*>(dst) + t * EPL;
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          uint2 o;
          o.x = f32_to_bf16_bits(gr[k]) | (f32_to_bf16_bits(gr[k + 1]) << 16);
          o.y = f32_to_bf16_bits(gr[k + 2]) | (f32_to_bf16_bits(gr[k + 3]) << 16);
          *reinterpret_cast<uint2*>(d16 + k) = o;
        }
      } else {
#pragma unroll
        for (int k = 0; k < EPL; k += 4)
          *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(gr[k], gr[k + 1], gr[k + 2], gr[k + 3]);
      }
    }
    if (t == 0) {
      dst[a.g_wcol] = gw;
      if (a.mode == kBwdEmitTable) dst[a.g_wcol + 1] = 1.f;  // touched (the dense apply scans for it)
    }
    return;
  }
  // in place: the table (LOCAL) or this rank's own table (EMIT self row)
  const bool own = a.mode != kBwdLocal;
  TV* tv = reinterpret_cast<TV*>(own ? const_cast<void*>(a.self.v) : a.v);
  float* tw = own ? a.self.w : a.w;
  const long long tvs = own ? a.self.v_stride : a.v_stride, tws = own ? a.self.w_stride : a.w_stride;
  opt_step_row<TV, EPL>(a.opt, gr, r.vv, r.st0, r.st1);
  store_row_e<LPR, TV, EPL>(tv + r.row * tvs + t * EPL, r.vv, tw, r.row, tws, t, tact, sr);
  if (tact) {
    const long long off = r.row * a.s_stride + t * EPL;
    store_state<TV, EPL>(a.s0v, off, r.st0, sr ? sr ^ kSrSalt0 : 0u, (uint32_t)r.row, (uint32_t)(t * EPL));
    if (a.s1v)
      store_state<TV, EPL>(a.s1v, off, r.st1, sr ? sr ^ kSrSalt1 : 0u, (uint32_t)r.row, (uint32_t)(t * EPL));
  }
  if (t == 0) {
    opt_step_tv<TV>(a.opt, gw, r.wv, r.q0, r.q1);
    tw[r.row * tws] = r.wv;
    a.s0w[r.row] = r.q0;
    if (a.s1w) a.s1w[r.row] = r.q1;
  }
}

template <int LPR, typename TV, int EPL>
__device__ inline void bwd_finalize(const BwdArgs& a, int u, int t, bool tact, int tE,
                                    const float (&A)[EPL], float Scx, float Sc, int n_u, uint32_t sr) {
  RowState<EPL> r;
  bwd_load<TV, EPL>(a, u, (long long)a.uniq[u], tE, r);
  bwd_finish<LPR, TV, EPL>(a, u, t, tact, r, A, Scx, Sc, n_u, sr);
}

// Minimum waves per SIMD the chunk kernel must keep (amdgpu_waves_per_eu): the fp8
// instantiations with 32 / 64 lanes per row sit a few VGPRs above the 128-VGPR step
// (129 -> 3 waves/SIMD instead of 4: +5% on the k128 fp8 FTRL step); capping them at
// 128 costs no spills.  1 = no constraint (the compiler's own choice).
template <int LPR, typename TV>
constexpr int chunk_min_waves() {
  // (bf16 LPR 32 -- k=128 bf16 -- crossed to 129 VGPRs with the short-chunk path: capped too; the
  // same cap on the fp32 k=64 kernel, 135 -> 128 VGPRs + 44 B/lane of spills, made the k=64 step
  // 10% slower: profiles/r1s3/chunk_vgpr_cap_ab.txt)
  return LPR == 32 ? 4 : 1;
}

// Chunk-kernel instantiations: kChunkAny runs every mode (split pieces, self rows, EMIT /
// EMIT_TABLE gradient rows, 64-bit r1 offsets); the others know the mode at compile time, with
// 32-bit row and r1 offsets (the launcher checks that r1 fits) and group-relative ds_bpermute
// sources: LOCAL (no piece walk, no self-row or gradient-row paths), EMIT (the row-sharded step:
// wire / own-table rows, gradient rows or in-place own-row updates; the piece walk of the split
// backward only in the *Pc kinds), and *NoX: the occurrences carry no values (x = 1: one
// ds_bpermute per occurrence less, Scx = Sc).
enum ChunkKind : int {
  kChunkAny = 0, kChunkLocal = 1, kChunkLocalNoX = 2,
  kChunkEmit = 3, kChunkEmitNoX = 4, kChunkEmitPc = 5, kChunkEmitPcNoX = 6
};
#ifndef FM_BWD_SPECIALIZE
#define FM_BWD_SPECIALIZE 1  // 0: every mode runs kChunkAny (the "bwdgen" build variant, A/B)
#endif

// One lane group per chunk of <= CH (<= kMaxCH) sorted occurrences of one row.
template <int LPR, typename TV, int KV, int EW = 0>
__device__ __forceinline__ void bwd_chunk_body(const BwdArgs& a) {
  constexpr bool FAST = KV != kChunkAny;                                   // 32-bit offsets, bpermute
  constexpr bool LOC = KV == kChunkLocal || KV == kChunkLocalNoX;          // local epilogue
  constexpr bool EMT = KV >= kChunkEmit;                                   // EMIT epilogue
  constexpr bool NOX = KV == kChunkLocalNoX || KV == kChunkEmitNoX || KV == kChunkEmitPcNoX;
  constexpr bool PCW = KV == kChunkAny || KV == kChunkEmitPc || KV == kChunkEmitPcNoX;  // piece walk
  const uint32_t sr = sr_step_seed(a.sr_counter);  // stochastic rounding seed (0: nearest)
  constexpr int EPL = EW ? EW : Frag<TV>::N;  // elements per lane: the table dtype's, or the wide kernel's 8
  static_assert(EW == 0 || LOC || EMT, "the wide kernels: local and EMIT kinds");
  constexpr int G = kWave / LPR;
  constexpr int PF = (kMaxCH + LPR - 1) / LPR;  // prefetched occurrences per lane
  constexpr int UNR0 = EW ? FM_CHUNK_UNR_W8 : chunk_unr<LPR, LOC, EMT, TV>();
  constexpr int UNR = LPR < UNR0 ? LPR : UNR0;  // r1 rows in flight
  constexpr bool kShortPath = LPR * EPL >= 128;                   // short-chunk block (below): k = 128 rows
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int gbase = g * LPR;
  const int gb4 = gbase << 2;  // (ds_bpermute byte address of the group's lane 0)
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int nchunks = a.counts[1];
  // r1 row of example ex, this lane's EPL columns (specialised kinds: 32-bit byte offsets, one mad)
  constexpr uint32_t kR1E = R1Bf16<TV>::v ? 2u : 4u;
  const char* r1b = reinterpret_cast<const char*>(a.r1);
  const uint32_t r1rb = (uint32_t)a.Kp * kR1E, r1cb = (uint32_t)(tE * EPL) * kR1E;
  auto r1_at = [&](int ex, float (&o)[EPL]) {
    if constexpr (FAST) load_r1<TV, EPL>(r1b + ((uint32_t)ex * r1rb + r1cb), 0, o);
    else load_r1<TV, EPL>(a.r1, (long long)ex * a.Kp + tE * EPL, o);
  };
  // the r1 row of an occurrence slot only where the slot holds one (its c is 0 otherwise): the unused
  // slots of the 4-slot short block -- 275k of a Criteo-shaped batch's 378k rows occur once -- issue no
  // load (FM_R1_MASK=0: every slot loads its lane's clamped row, the A/B).  Masking the UNR blocks'
  // tails too was much slower (k64 fp32 0.592-0.597 -> 0.701-0.704 ms, EMIT 0.624 -> 0.736: each masked
  // load became its own branch, so the block's loads no longer went out together; round 6).
  auto r1_at_if = [&](bool need, int ex, float (&o)[EPL]) {
    if (!FM_R1_MASK || need) {
      r1_at(ex, o);
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) o[k] = 0.f;
    }
  };
  // split-backward piece: this piece's chunk ranges (one per owner) and their prefix sums
  __shared__ int pr_start[PCW ? kMaxPieceOwners : 1], pr_pre[PCW ? kMaxPieceOwners + 1 : 1];
  const bool pieced = PCW && a.piece >= 0;
  if (pieced) {
    if (threadIdx.x == 0) {
      int acc = 0;
      for (int q = 0; q < a.n_owners; ++q) {
        const int c0 = a.seg_chunk[a.seg_bounds[2 * q + a.piece]];
        const int c1 = a.seg_chunk[a.seg_bounds[2 * q + a.piece + 1]];
        pr_start[q] = c0;
        pr_pre[q] = acc;
        acc += c1 - c0;
      }
      pr_pre[a.n_owners] = acc;
    }
    __syncthreads();
  }
  const int i1 = pieced ? pr_pre[a.n_owners] : nchunks;
  const int stride = gridDim.x * kWavesPerBlock * G;
  // Software pipeline over this lane group's chunks: the descriptor of the next
  // chunk (and the list entry of the one after) load while the current one is
  // reduced, so the dependent metadata chain is off the critical path.
  int ii = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g;
  auto chunk_at = [&](int i) {
    if (pieced) {
      int q = 0;
      while (q + 1 < a.n_owners && pr_pre[q + 1] <= i) ++q;
      return pr_start[q] + (i - pr_pre[q]);
    }
#if FM_CHUNK_PERM
    // (probe variant "chunkperm": the walk interleaves 8 far-apart streams of chunks -- lane groups
    // working together reduce rows ~n/8 apart instead of consecutive ones -- to measure what the
    // read-modify-write's page locality is worth: profiles/r6/rmw_locality.txt)
    const int q8 = nchunks / 8;
    if (i < 8 * q8) return (i & 7) * q8 + (i >> 3);
#endif
    return i;
  };
  int c = ii < i1 ? chunk_at(ii) : 0;
  int cn = ii + stride < i1 ? chunk_at(ii + stride) : 0;
  int d_j0 = 0, d_j1 = 0, d_seg = 0, d_key = 0;
  if (ii < i1) {
    d_j0 = a.chunk_start[c]; d_j1 = a.chunk_start[c + 1]; d_seg = a.chunk_seg[c]; d_key = a.chunk_key[c];
  }
  for (; ii < i1; ii += stride) {
    const int cc = c, j0 = d_j0, j1 = d_j1, key = d_key;
    const int u = d_seg & kChunkSegMask;
    const bool single = (unsigned)d_seg & kChunkSingle;
    const bool first = d_seg & kChunkFirst;
    if (ii + stride < i1) {
      c = cn;
      d_j0 = a.chunk_start[c]; d_j1 = a.chunk_start[c + 1]; d_seg = a.chunk_seg[c]; d_key = a.chunk_key[c];
      cn = ii + 2 * stride < i1 ? chunk_at(ii + 2 * stride) : 0;
    }
    const int len = j1 - j0;
    RowState<EPL> rs;
    if (single) {
      if constexpr (LOC) bwd_load_local<TV, EPL>(a, (long long)key, tE, rs);
      else if constexpr (EMT) bwd_load_emit<TV, EPL>(a, u, (long long)key, tE, rs);
      else bwd_load<TV, EPL>(a, u, (long long)key, tE, rs);
    }
    // lane-parallel prefetch of the chunk's (example, dpred*x, x)
    int pex[PF];
    float pc[PF], px[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int jj = j0 + q * LPR + t;
      const bool ok = jj < j1;
      const int jc = ok ? jj : j0;
      const int ex = a.sorted_ex[jc] >> a.ex_shift;
      const float x = !NOX && a.sorted_x ? a.sorted_x[jc] : 1.f;
      pex[q] = ex;
      px[q] = x;
      pc[q] = ok ? a.dpred[ex] * x : 0.f;
    }
    // (the sums below are explicit fma chains: contraction left to the compiler fused some multiply-adds
    // and not others depending on the instantiation -- 1-ulp differences between lane widths)
    float A[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) A[k] = 0.f;
    float Scx = 0.f, Sc = 0.f;
    // occurrence li of prefetch slot q: (example, c masked by ok, x).  General kernel: __shfl from
    // lane gbase + li (gbase when !ok); specialised: ds_bpermute from gb4 + 4 li (the constant folds into
    // the instruction's offset; an invalid slot reads its lane's clamped, valid example, c = 0)
    auto occ = [&](int q, int li, bool ok, int& ex, float& cs, float& xs) {
      if constexpr (FAST) {
        const int sb = gb4 + (li << 2);
        ex = __builtin_amdgcn_ds_bpermute(sb, pex[q]);
        const float c0 = __int_as_float(__builtin_amdgcn_ds_bpermute(sb, __float_as_int(pc[q])));
        cs = ok ? c0 : 0.f;
        xs = NOX ? 1.f : __int_as_float(__builtin_amdgcn_ds_bpermute(sb, __float_as_int(px[q])));
      } else {
        // shuffles are unconditional (every lane of the group takes part); mask after
        const int src = gbase + (ok ? li : 0);
        ex = __shfl(pex[q], src, kWave);
        const float c0 = __shfl(pc[q], src, kWave);
        cs = ok ? c0 : 0.f;
        xs = __shfl(px[q], src, kWave);
      }
    };
    if constexpr (LPR < kChunkUnr) {
      // narrow rows (k=16 bf16: LPR 2): flat walk over the chunk's occurrences with
      // kChunkUnr r1 rows in flight per lane (the q-major walk below keeps only LPR in
      // flight); same summation order.  k16 bf16 step 0.525 -> 0.497 ms; for LPR >= 8 the
      // flat walk measured slower (k64 0.652 -> 0.665, k128 fp8 0.989 -> 1.039 ms):
      // profiles/r1s4/chunk_flat_ab.txt
      constexpr int UNRF = kChunkUnr;
#pragma unroll
      for (int o0 = 0; o0 < PF * LPR; o0 += UNRF) {
        if (o0 >= len) break;
        float rr[UNRF][EPL], cc[UNRF], xx[UNRF];
#pragma unroll
        for (int uu = 0; uu < UNRF; ++uu) {
          const int oi = o0 + uu;
          const int q = oi / LPR < PF ? oi / LPR : PF - 1, li = oi % LPR;
          const bool ok = oi < PF * LPR && oi < len;
          int ex;
          occ(q, li, ok, ex, cc[uu], xx[uu]);
          r1_at(ex, rr[uu]);
        }
#pragma unroll
        for (int uu = 0; uu < UNRF; ++uu) {
#pragma unroll
          for (int k = 0; k < EPL; ++k) A[k] = fma_acc<TV>(cc[uu], rr[uu][k], A[k]);
          Scx = fma_acc<TV>(cc[uu], xx[uu], Scx);
          Sc += cc[uu];
        }
      }
    } else if (kShortPath && len <= 4) {
      // short chunks (275k of the 378k rows of a Criteo-shaped batch occur once, 341k of
      // the 510k chunks have <= 4 occurrences): one block of 4 r1 rows instead of UNR,
      // so the group issues no redundant loads for the occurrences it does not have.
      // Same-box A/B (profiles/r2/short_chunk_ab.txt): k128 bf16 FTRL 1.044 -> 0.976 ms;
      // k64 bf16 0.655 -> 0.695 ms (slower), k64 fp32 +-0: on for the 32-lane rows only
      constexpr int U4 = 4;
      float rr[U4][EPL], cc[U4], xx[U4];
#pragma unroll
      for (int uu = 0; uu < U4; ++uu) {
        int ex;
        occ(0, uu, uu < len, ex, cc[uu], xx[uu]);
        r1_at_if(uu == 0 || uu < len, ex, rr[uu]);
      }
#pragma unroll
      for (int uu = 0; uu < U4; ++uu) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) A[k] = fma_acc<TV>(cc[uu], rr[uu][k], A[k]);
        Scx = fma_acc<TV>(cc[uu], xx[uu], Scx);
        Sc += cc[uu];
      }
    } else {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        if (q * LPR < len) {
          for (int l = 0; l < LPR && q * LPR + l < len; l += UNR) {
            float rr[UNR][EPL], cc[UNR], xx[UNR];
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
              const int li = l + uu;
              const bool ok = li < LPR && q * LPR + li < len;
              int ex;
              occ(q, li < LPR ? li : 0, ok, ex, cc[uu], xx[uu]);
              r1_at(ex, rr[uu]);
            }
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
#pragma unroll
              for (int k = 0; k < EPL; ++k) A[k] = fma_acc<TV>(cc[uu], rr[uu][k], A[k]);
              Scx = fma_acc<TV>(cc[uu], xx[uu], Scx);
              Sc += cc[uu];
            }
          }
        }
      }
    }
    if (single) {
      if constexpr (LOC) bwd_finish_local<LPR, TV, EPL>(a, t, tact, rs, A, Scx, Sc, len, sr);
      else if constexpr (EMT) bwd_finish_emit<LPR, TV, EPL>(a, u, t, tact, rs, A, Scx, Sc, len, sr);
      else bwd_finish<LPR, TV, EPL>(a, u, t, tact, rs, A, Scx, Sc, len, sr);
    } else {
      float* dst = a.partial + (long long)cc * (a.Kp + 4);
      if (tact) {
#pragma unroll
        for (int k = 0; k < EPL; k += 4)
          *reinterpret_cast<float4*>(dst + t * EPL + k) = make_float4(A[k], A[k + 1], A[k + 2], A[k + 3]);
      }
      if (t == 0) {
        dst[a.Kp] = Scx;
        dst[a.Kp + 1] = Sc;
        // the row's first chunk registers the row for the combine: rows over <= kSmallChunks chunks
        // for a lane group, hotter rows for a workgroup (both lists complete when this kernel ends,
        // so the two combines run as one launch)
        if (first) {
          if (a.seg_chunk[u + 1] - a.seg_chunk[u] > kSmallChunks) a.big_list[atomicAdd(a.big_count, 1)] = u;
          else a.multi[atomicAdd(&a.counts_rw[2], 1)] = u;
        }
      }
    }
  }
}

template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(chunk_min_waves<LPR, TV>())))
void fm_bwd_chunk_kernel(BwdArgs a) { bwd_chunk_body<LPR, TV, kChunkAny>(a); }
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(chunk_min_waves<LPR, TV>())))
void fm_bwd_chunk_local_kernel(BwdArgs a) { bwd_chunk_body<LPR, TV, kChunkLocal>(a); }
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(chunk_min_waves<LPR, TV>())))
void fm_bwd_chunk_local_nox_kernel(BwdArgs a) { bwd_chunk_body<LPR, TV, kChunkLocalNoX>(a); }
#if FM_FP8_WIDE
// the wide fp8 kernels (8 values per lane; LPR = Kp / 8): 128-VGPR cap as the 32-lane fp8 kernels
template <int LPR>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void fm_bwd_chunk_local_w8_kernel(BwdArgs a) { bwd_chunk_body<LPR, fp8e4m3, kChunkLocal, 8>(a); }
template <int LPR>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void fm_bwd_chunk_local_nox_w8_kernel(BwdArgs a) { bwd_chunk_body<LPR, fp8e4m3, kChunkLocalNoX, 8>(a); }
#endif
#define FM_EMIT_CHUNK_KERNEL(NAME, KIND)                                                          \
  template <int LPR, typename TV>                                                                 \
  __global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(chunk_min_waves<LPR, TV>()))) \
  void NAME(BwdArgs a) { bwd_chunk_body<LPR, TV, KIND>(a); }
FM_EMIT_CHUNK_KERNEL(fm_bwd_chunk_emit_kernel, kChunkEmit)
FM_EMIT_CHUNK_KERNEL(fm_bwd_chunk_emit_nox_kernel, kChunkEmitNoX)
FM_EMIT_CHUNK_KERNEL(fm_bwd_chunk_emit_pc_kernel, kChunkEmitPc)
FM_EMIT_CHUNK_KERNEL(fm_bwd_chunk_emit_pc_nox_kernel, kChunkEmitPcNoX)
#undef FM_EMIT_CHUNK_KERNEL
#if FM_FP8_WIDE
// (the row-sharded step's wide fp8 kernels: wire / own-table rows, gradient rows or in-place own rows)
template <int KIND>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void fm_bwd_chunk_emit_w8_kernel(BwdArgs a) { bwd_chunk_body<16, fp8e4m3, KIND, 8>(a); }
#endif

// Rows split over 2..kSmallChunks chunks: one lane group, ordered sum of the partials (EW: the wide fp8
// form, 8 values per lane -- the same sums in the same order).
template <int LPR, typename TV, int EW = 0>
__device__ inline void bwd_combine_body(const BwdArgs& a, int blk, int nblk, uint32_t sr) {
  constexpr int EPL = EW ? EW : Frag<TV>::N;
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int nmulti = a.counts[2];  // rows spanning 2..kSmallChunks chunks, listed by the chunk kernel
  const int ngroups = nblk * kWavesPerBlock * G;
  for (int i = (blk * kWavesPerBlock + (threadIdx.x >> 6)) * G + g; i < nmulti; i += ngroups) {
    const int u = a.multi[i];
    const int c0 = a.seg_chunk[u], c1 = a.seg_chunk[u + 1];
    float A[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) A[k] = 0.f;
    float Scx = 0.f, Sc = 0.f;
    for (int c = c0; c < c1; c += 4) {
      float pr[4][EPL], ps[4], pt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = c + q < c1;
        const float* src = a.partial + (long long)(ok ? c + q : c0) * (a.Kp + 4);
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
          pr[q][k] = f.x; pr[q][k + 1] = f.y; pr[q][k + 2] = f.z; pr[q][k + 3] = f.w;
        }
        ps[q] = ok ? src[a.Kp] : 0.f;
        pt[q] = ok ? src[a.Kp + 1] : 0.f;
        if (!ok) {
#pragma unroll
          for (int k = 0; k < EPL; ++k) pr[q][k] = 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) A[k] += pr[q][k];
        Scx += ps[q];
        Sc += pt[q];
      }
    }
    bwd_finalize<LPR, TV, EPL>(a, u, t, tact, tE, A, Scx, Sc, a.seg_start[u + 1] - a.seg_start[u], sr);
  }
}

// Hot rows: one workgroup per row. Lane group q of the workgroup sums chunks
// c0+q, c0+q+NG, ... ; the NG group sums are reduced in LDS in group order.  (1024-thread workgroups
// for the 32-lane rows' hot-row launch measured slower: k128 fp8 FTRL 78 -> 116 us in-step, round 6.)
template <int LPR, typename TV, int WPB = kWavesPerBlock>
__device__ inline void bwd_big_body(const BwdArgs& a, int blk, int nblk, uint32_t sr) {
  constexpr int EPL = Frag<TV>::N;
  constexpr int G = kWave / LPR;
  constexpr int NG = WPB * G;
  constexpr int ROW = LPR * EPL + 4;  // LDS floats per group sum (>= Kp + 2)
  __shared__ float lds[NG * ROW];
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int grp = (threadIdx.x >> 6) * G + g;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;
  const int nbig = *a.big_count;
  for (int bi = blk; bi < nbig; bi += nblk) {
    const int u = a.big_list[bi];
    const int c0 = a.seg_chunk[u], c1 = a.seg_chunk[u + 1];
    float A[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) A[k] = 0.f;
    float Scx = 0.f, Sc = 0.f;
    // 4 partial rows in flight per group; fixed order (c0+grp, +NG, ...) keeps the sum deterministic
    for (int c = c0 + grp; c < c1; c += 4 * NG) {
      float pr[4][EPL], ps[4], pt[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cc = c + q * NG;
        const bool ok = cc < c1;
        const float* src = a.partial + (long long)(ok ? cc : c) * (a.Kp + 4);
#pragma unroll
        for (int k = 0; k < EPL; k += 4) {
          const float4 f = *reinterpret_cast<const float4*>(src + tE * EPL + k);
          pr[q][k] = f.x; pr[q][k + 1] = f.y; pr[q][k + 2] = f.z; pr[q][k + 3] = f.w;
        }
        const float m = ok ? 1.f : 0.f;
        ps[q] = m * src[a.Kp];
        pt[q] = m * src[a.Kp + 1];
#pragma unroll
        for (int k = 0; k < EPL; ++k) pr[q][k] *= m;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int k = 0; k < EPL; ++k) A[k] += pr[q][k];
        Scx += ps[q];
        Sc += pt[q];
      }
    }
    float* my = lds + grp * ROW;
#pragma unroll
    for (int k = 0; k < EPL; ++k) my[t * EPL + k] = A[k];
    if (t == 0) { my[LPR * EPL] = Scx; my[LPR * EPL + 1] = Sc; }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) A[k] = 0.f;
      Scx = Sc = 0.f;
      for (int q = 0; q < NG; ++q) {
        const float* o = lds + q * ROW;
#pragma unroll
        for (int k = 0; k < EPL; ++k) A[k] += o[t * EPL + k];
        Scx += o[LPR * EPL];
        Sc += o[LPR * EPL + 1];
      }
      bwd_finalize<LPR, TV, EPL>(a, u, t, tact, tE, A, Scx, Sc, a.seg_start[u + 1] - a.seg_start[u], sr);
    }
    __syncthreads();
  }
}

// Both combines in one launch (their row lists are disjoint and complete after the chunk kernel):
// the first a.big_blocks workgroups take the hot rows (the long poles, dispatched first), the rest the
// lane-group combine.  Two launches ran back to back (combine 35-43 us, then big 38-40 us in-step);
// one launch, same box: k64 fp32 0.605-0.608 -> 0.592-0.596 ms, EMIT k64 0.636 -> 0.623, k16 bf16 tied;
// 32-lane rows (k128) lost (fp8 FTRL 0.770 -> 0.778) and keep two launches of this kernel
// (big_blocks = 0: combine only; = grid: hot rows only).  (Placing the hot-row workgroups last, and
// 256-8192 of them, measured no better: the A/B knobs were removed in round 6.)
constexpr int kBigBlocks = 1024;
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) void fm_bwd_combine_kernel(BwdArgs a) {
  const uint32_t sr = sr_step_seed(a.sr_counter);  // stochastic rounding seed (0: nearest)
  if ((int)blockIdx.x < a.big_blocks) bwd_big_body<LPR, TV>(a, blockIdx.x, a.big_blocks, sr);
  else bwd_combine_body<LPR, TV>(a, blockIdx.x - a.big_blocks, gridDim.x - a.big_blocks, sr);
}
#if FM_FP8_WIDE
// the lane-group combine of the wide fp8 rows (the hot-row workgroup combine keeps 4 values per lane: its
// group count fixes the summation order)
template <int LPR>
__global__ __launch_bounds__(kBlock) void fm_bwd_combine_w8_kernel(BwdArgs a) {
  bwd_combine_body<LPR, fp8e4m3, 8>(a, blockIdx.x, gridDim.x, sr_step_seed(a.sr_counter));
}
#endif

// specialised kinds (local / EMIT) share the launch shape: EMIT runs the local step's kernel body
static bool fast_kind(int kind) { return kind != kChunkAny; }

static int chunk_wg_per_cu(int lpr, int kind) { return fast_kind(kind) && lpr <= 16 ? 3 : 0; }

static long long g_bwd_wide_launches = 0;  // (host counter: tests check the wide kernel ran)
long long bwd_wide_launches() { return g_bwd_wide_launches; }

int launch_bwd(const BwdArgs& a, int dtype, long long max_chunks, long long max_unique, hipStream_t st) {
  if (max_chunks <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  const int G = kWave / lpr;
  if (!a.counters_ready) {  // (a fresh dedup zeroed both on its own stream)
    (void)hipMemsetAsync(a.big_count, 0, sizeof(int), st);
    (void)hipMemsetAsync(a.counts_rw + 2, 0, sizeof(int), st);  // #multi-chunk rows, appended by the chunk kernel
  }
  int g1 = (fill_grid(max_chunks, kWavesPerBlock * G, 8192) + 7) / 8 * 8;
  // Cap on the chunk kernel's workgroups (the grid-stride walk covers every chunk either way).
  // Same-box sweeps (profiles/r2/chunk_grid_ab.txt): 16-lane rows (k=64 fp32 / bf16) 3456-4608
  // blocks beat the 8192 fill cap by 2.5-3% (k64 fp32 0.677-0.685 -> 0.661-0.662 ms), 4-lane
  // rows (k=16 bf16) 512-576 by 5.5% (0.519-0.522 -> 0.491-0.495 ms); for 32-lane rows (k=128)
  // every cap tried was slower.  The local step only: the row-sharded step at world 1 runs
  // steadiest without a cap (0.701-0.702 ms vs 0.68-0.73 with 3840; chunk_grid_ab.txt).  Re-swept with
  // 3 workgroups per CU (profiles/r4/chunk_grid_wg3.txt): 16-lane rows 3072 (0.616-0.618 ms) over 3840
  // (0.620-0.624), 2304 / 5120 slower; 4-lane rows 512 still best; 32-lane rows uncapped.
  if (a.piece >= 0 && a.n_owners > kMaxPieceOwners) return -6;
  // (a software-pipelined variant that issued the next chunk's occurrence and row loads before
  // reducing the current one ran 367 -> 316 us alone but made the step slower twice:
  // profiles/r2/chunk_pipe_ab.txt, profiles/r3/fwd_prefetch_ab.txt; removed)
  // (workgroup counts: a 2048 cap / 1024 measured best among 512-8192, profiles/r2/combine_grid_ab.txt)
  const int g2 = fill_grid(max_unique, kWavesPerBlock * G, 2048);
  // (a split walk -- the chunks of multi-chunk rows first, their combine beside the single-chunk
  // rows' launch, or both launches concurrent -- measured slower: k64 0.669 -> 0.72-0.78 ms, each
  // launch as long as the whole walk; profiles/r3/bwd_split_ab.txt)
  // specialised chunk kernels (see ChunkKind) when r1 fits 32-bit offsets: LOCAL mode, and EMIT mode
  // (the row-sharded step; the "bwdgen" build variant keeps every mode on the general kernel, A/B)
  const long long r1_bytes = (long long)a.nex * a.Kp * (dtype == kFP8 ? 2 : 4);
  const bool fits = FM_BWD_SPECIALIZE && lpr >= 4 && r1_bytes < (1LL << 32);
  int kind = kChunkAny;
  if (fits && a.mode == kBwdLocal && a.piece < 0) {
    kind = a.sorted_x ? kChunkLocal : kChunkLocalNoX;
  } else if (fits && a.mode == kBwdEmit) {
    kind = a.piece >= 0 ? (a.sorted_x ? kChunkEmitPc : kChunkEmitPcNoX) : (a.sorted_x ? kChunkEmit : kChunkEmitNoX);
  }
  const int cap = !fast_kind(kind) ? -1 : (lpr == 16 ? 3072 : lpr == 4 ? 512 : -1);
  if (cap > 0 && g1 > cap) g1 = (cap + 7) / 8 * 8;
  // Chunk workgroups resident per CU, capped through dynamic LDS the kernel does not use (a CU holds
  // floor(LDS / bytes) of them).  The side stream's radix-sort blocks then find LDS on every CU and
  // the capped grid spreads over more CUs: same-box, 3 per CU took k64 fp32 0.648 -> 0.621 ms and
  // k16 bf16 0.511 -> 0.487; 32-lane rows (k128, uncapped grid) lose (fp8 FTRL 0.887 -> 0.978)
  // (profiles/r4/wg_per_cu_ab.txt).  An earlier build's 130-VGPR k16 kernel (3 waves / SIMD) had
  // the same effect by accident.
  const int wg_cu = chunk_wg_per_cu(lpr, kind);
  const bool pcw = kind == kChunkAny || kind == kChunkEmitPc || kind == kChunkEmitPcNoX;
  const int chunk_static_lds = pcw ? (int)sizeof(int) * (2 * kMaxPieceOwners + 1) : 0;  // piece walk
  const int chunk_lds = wg_cu > 0 ? lds_for_wg_per_cu(wg_cu, chunk_static_lds) : 0;
  // wide fp8 rows (k = 128, 16 lanes x 8 values): rows, r1 rows and state rows 16-byte aligned
  // (EMIT: wire rows and own table rows 8-byte aligned too)
  const bool emit_kind = kind >= kChunkEmit;
  const bool wide = FM_FP8_WIDE && dtype == kFP8 && lpr == 32 && a.Kp % 8 == 0 && fast_kind(kind) &&
                    a.v_stride % 8 == 0 && a.s_stride % 8 == 0 && ((uintptr_t)a.v % 8 == 0) &&
                    ((uintptr_t)a.r1 % 16 == 0) && ((uintptr_t)a.s0v % 16 == 0) && ((uintptr_t)a.s1v % 16 == 0) &&
                    (!emit_kind || (a.self.v_stride % 8 == 0 && (uintptr_t)a.self.v % 8 == 0));
  (void)wide;
#if FM_FP8_WIDE
  if (wide) {
    ++g_bwd_wide_launches;
    const int gw = (fill_grid(max_chunks, kWavesPerBlock * (kWave / 16), 8192) + 7) / 8 * 8;
    switch (kind) {
      case kChunkLocalNoX:
        hipLaunchKernelGGL(fm_bwd_chunk_local_nox_w8_kernel<16>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
      case kChunkLocal:
        hipLaunchKernelGGL(fm_bwd_chunk_local_w8_kernel<16>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
      case kChunkEmit:
        hipLaunchKernelGGL(fm_bwd_chunk_emit_w8_kernel<kChunkEmit>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
      case kChunkEmitNoX:
        hipLaunchKernelGGL(fm_bwd_chunk_emit_w8_kernel<kChunkEmitNoX>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
      case kChunkEmitPc:
        hipLaunchKernelGGL(fm_bwd_chunk_emit_w8_kernel<kChunkEmitPc>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
      default:
        hipLaunchKernelGGL(fm_bwd_chunk_emit_w8_kernel<kChunkEmitPcNoX>, dim3(gw), dim3(kBlock), chunk_lds, st, a);
        break;
    }
  } else
#endif
  if (kind == kChunkLocalNoX) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_local_nox_kernel, g1, chunk_lds, st, a);
  } else if (kind == kChunkLocal) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_local_kernel, g1, chunk_lds, st, a);
  } else if (kind == kChunkEmit) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_emit_kernel, g1, chunk_lds, st, a);
  } else if (kind == kChunkEmitNoX) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_emit_nox_kernel, g1, chunk_lds, st, a);
  } else if (kind == kChunkEmitPc) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_emit_pc_kernel, g1, chunk_lds, st, a);
  } else if (kind == kChunkEmitPcNoX) {
    FM_DISPATCH_WIDE(dtype, lpr, fm_bwd_chunk_emit_pc_nox_kernel, g1, chunk_lds, st, a);
  } else {
    FM_DISPATCH_SHM(dtype, lpr, fm_bwd_chunk_kernel, g1, chunk_lds, st, a);
  }
  BwdArgs b = a;
  if (lpr >= 32) {  // (one launch lost for 32-lane rows: above)
    b.big_blocks = 0;
#ifndef FM_FP8_WIDE_COMBINE
#define FM_FP8_WIDE_COMBINE 1  // (0: the 4-value lane-group combine beside the wide chunk kernel, A/B)
#endif
#if FM_FP8_WIDE
    if (wide && FM_FP8_WIDE_COMBINE)
      hipLaunchKernelGGL(fm_bwd_combine_w8_kernel<16>, dim3(fill_grid(max_unique, kWavesPerBlock * (kWave / 16), 2048)),
                         dim3(kBlock), 0, st, b);
    else
#endif
    FM_DISPATCH(dtype, lpr, fm_bwd_combine_kernel, g2, st, b);
    b.big_blocks = kBigBlocks;
    FM_DISPATCH(dtype, lpr, fm_bwd_combine_kernel, kBigBlocks, st, b);
  } else {
    b.big_blocks = kBigBlocks;
    FM_DISPATCH(dtype, lpr, fm_bwd_combine_kernel, kBigBlocks + g2, st, b);
  }
  return (int)hipGetLastError();
}

}  // namespace fm
