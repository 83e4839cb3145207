// Fused FM forward + loss on gfx950 (see the design notes below).
//
// Parity: reference FmScorer (cc/fm_scorer_op.h:8-140: BiasGenerator,
// FeatureRankGenerator, pred/reg reductions) fused with the loss ops of
// tffm/fm_model.py:311-333.
//
// Design: one wave64 per example; the example's (row, value) pairs are loaded
// once, lane-parallel, and broadcast with ds_bpermute; factor rows are fetched
// 16 B per lane, G = 64/LPR rows per wave instruction, UNR row groups in flight
// per lane; r1 = sum x*v is cached for the backward (the reference recomputes
// it, G5) and the loss gradient dpred is emitted by the same kernel (T6).
#include "fm_common.h"

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
  void* r1;             // [B, Kp] fp32 (bf16 for fp8 tables: R1Bf16) or nullptr
  float* dpred;         // [B] or nullptr
  float* loss_partial;  // [gridDim.x] or nullptr
  float* reg_partial;   // [2*gridDim.x] (sum |v|^2, sum w^2) or nullptr
  const float* bias;    // [1] global bias (optional model extension) or nullptr
  SelfRows self;           // row-sharded step: segments read from this rank's own table rows
  // Segment lookup (row-sharded step, dedup.hip seg_index_kernel): rows[] hold the shard keys
  // and each occurrence's segment is found through the bucket index instead of an inverse map.
  const int* seg_idx;      // [nb + 1] first segment of each key bucket, or null (rows are segment ids)
  const int* seg_keys;     // [U] sorted unique keys
  int seg_shift;           // bucket = key >> seg_shift
  int max_feats;           // host-known max occurrences per example (-1: unknown); the MFMA fp8 path needs it
};

// Segment of key k (present in the batch): the bucket's first candidate, then a scan over the
// bucket's other keys (the last candidate needs no compare).  ~0.4 keys per bucket at the
// default sizing, so usually the idx reads only.
__device__ inline int seg_lookup(const FwdArgs& a, int k) {
  const int b = (int)((uint32_t)k >> a.seg_shift);
  int s = a.seg_idx[b];
  const int e = a.seg_idx[b + 1];
  while (s + 1 < e && a.seg_keys[s] != k) ++s;
  return s;
}

#ifndef FM_FWD_PREFETCH
#define FM_FWD_PREFETCH 1
#endif
#ifndef FM_FWD_SPECIALIZE  // 0: every step runs the general (sharded) forward (A/B build variant "fwdgen")
#define FM_FWD_SPECIALIZE 1
#endif
constexpr int kSelfBit = (int)0x80000000u;   // row index tag: this rank's own table row (SelfRows)
// Rows of one example kept in flight per lane group: enough to cover a
// Criteo-shaped example (39 features) in one round for K=64 (G=4 -> 10 row
// loads per lane) while bounding VGPRs for large K.
// ceil(40 / G): G = 32 (k=16 bf16) keeps both of an example's row groups in flight
// (floor gave 1: k16 bf16 step 0.532 -> 0.522 ms, profiles/r1s4/fwd_unroll_ceil_ab.txt).
template <int G>
struct FwdUnroll {
  static constexpr int v = ((40 + G - 1) / G) > 12 ? 12 : ((40 + G - 1) / G);
};

// Minimum waves per SIMD of the forward (amdgpu_waves_per_eu; 1 = compiler's choice): the
// 32/64-lane instantiations (k>=128) need 132-136 VGPRs -> 3 waves/SIMD uncapped; capped at
// 4 the k=128 FTRL step runs 1.038 -> 0.992 ms (fp32) and 1.033 -> 0.987 ms (fp8)
// (profiles/r1s3/fwd_cap_ab.txt).  A floor of 5 or 6 on the k=64 (16-lane) instantiations spills:
// 0.65 -> 0.73 / 0.86 ms (round 1 A/B variants, since removed).
template <int LPR, typename TV>
constexpr int fwd_min_waves() {
  return LPR >= 32 ? 4 : 1;
}
// The local forward's 16-lane instantiations (k=64): 2 row groups in flight per lane at 7 waves per
// SIMD (72 VGPRs) instead of 10 at 4 (115): k64 fp32 0.618 -> 0.607 ms same-box; 3 at 6 waves ties,
// 4 at 5 / 6 at 4 lose (profiles/r4/fwd_occupancy_ab.txt).  Latency-bound gathers: more waves hide
// more than more loads per wave.  (A variant of the register accumulation needed 136 VGPRs
// uncapped -- 3 waves -- and the 4-wave floor then bought 0.674 -> 0.643 ms: specialize_ab.txt.)
#ifndef FM_FWD_LOCAL_W16
#define FM_FWD_LOCAL_W16 7
#endif
#ifndef FM_FWD_UNR16
#define FM_FWD_UNR16 2
#endif
// The same pair for the 32-lane instantiations (k = 128): fp8 rows 4 at 7 waves (72 VGPRs):
// k128 fp8 FTRL 0.806 -> 0.784 ms; bf16 / fp32 rows keep 12 at 4 (lower pairs spill there: k128
// bf16 FTRL 0.95 -> 1.07-1.21 ms; profiles/r4/fwd_occupancy_ab.txt).  FM_FWD_UNR32[_FP8] /
// FM_FWD_LOCAL_W32[_FP8]: A/B knobs.
#ifndef FM_FWD_LOCAL_W32
#define FM_FWD_LOCAL_W32 4
#endif
#ifndef FM_FWD_UNR32
#define FM_FWD_UNR32 12
#endif
#ifndef FM_FWD_LOCAL_W32_FP8
#define FM_FWD_LOCAL_W32_FP8 7
#endif
#ifndef FM_FWD_UNR32_FP8
#define FM_FWD_UNR32_FP8 4
#endif
// The 4-lane bf16 instantiation (k = 16 bf16): 5 row groups in flight at >= 4 waves per SIMD instead
// of 3 at the compiler's choice: k16 bf16 0.490-0.491 -> 0.485-0.488 ms over four same-box reps; 8 waves
// lose 4-36%, 6 at 4 / 8 at 3 / 4 at 5 tie or lose (profiles/r4/fwd_occupancy_ab.txt).  Other dtypes
// of 4-lane rows keep the generic choice.  FM_FWD_LOCAL_W4 / FM_FWD_UNR4: A/B knobs (0 = generic).
#ifndef FM_FWD_LOCAL_W4
#define FM_FWD_LOCAL_W4 4
#endif
#ifndef FM_FWD_UNR4
#define FM_FWD_UNR4 5
#endif
// The sharded forward's 16-lane rows (k = 64): its row address takes two broadcasts and a 64-bit
// add (the local kernel's: one broadcast and a mad), a longer per-row-group chain, and 2 row groups
// at 7 waves ran 0.70 ms EMIT (fwd 228-244 us vs the local kernel's 175): 10 in flight at 4 waves
// instead (FM_FWD_UNR16_SH / FM_FWD_SH_W16, A/B build variants).
#ifndef FM_FWD_UNR16_SH
#define FM_FWD_UNR16_SH 10
#endif
#ifndef FM_FWD_SH_W16
#define FM_FWD_SH_W16 4
#endif
template <typename TV>
constexpr bool fwd_is_bf16() { return std::is_same<TV, __hip_bfloat16>::value; }
template <int LPR, typename TV, bool SH = false>
constexpr int fwd_local_min_waves() {
  return LPR == 4 && fwd_is_bf16<TV>() && FM_FWD_LOCAL_W4 > 0 ? FM_FWD_LOCAL_W4
         : LPR == 16 ? (SH && !Frag<TV>::kScaled ? FM_FWD_SH_W16 : FM_FWD_LOCAL_W16)
         : LPR == 32 ? (Frag<TV>::kScaled ? FM_FWD_LOCAL_W32_FP8 : FM_FWD_LOCAL_W32)
                     : fwd_min_waves<LPR, TV>();
}
template <int LPR, typename TV, bool SH = false>
constexpr int fwd_unroll() {
  return LPR == 16 && SH && !Frag<TV>::kScaled ? FM_FWD_UNR16_SH
         : LPR == 4 && fwd_is_bf16<TV>() && FM_FWD_UNR4 > 0 ? FM_FWD_UNR4
         : LPR == 16 ? FM_FWD_UNR16
         : LPR == 32 ? (Frag<TV>::kScaled ? FM_FWD_UNR32_FP8 : FM_FWD_UNR32)
                     : FwdUnroll<kWave / LPR>::v;
}

// SH: the row-sharded step's features -- rows[] may be keys (segment lookup), an occurrence's row
// lives either in the gathered wire buffer (segment u) or, for this rank's own rows, in the table
// (SelfRows).  Both instantiations share the mechanics measured on the local step: the example's
// (row, value) pairs are loaded lane-parallel and broadcast with precomputed ds_bpermute offsets,
// fp8 rows arrive raw and are converted with their power-of-two row scale (v_cvt_scalef32), s2 /
// reg come from the stored row norms, and the occupancy / rows-in-flight pair is the local one.
// The local kernel addresses a row as base + row * stride (one 32 x 32 -> 64-bit mad per row
// group); the sharded one resolves each occurrence's row to a byte address once, lane-parallel
// (source select, segment lookup, tail loads), and broadcasts the 64-bit address (two ds_bpermute
// and one 64-bit add per row group) -- no per-row-group tag test or base / stride select.
template <int LPR, typename TV, bool SH>
__device__ __forceinline__ void fwd_body(const FwdArgs& a) {
  using F = Frag<TV>;
  constexpr int EPL = F::N;
  constexpr int G = kWave / LPR;
  constexpr int UNR = fwd_unroll<LPR, TV, SH>();
  // fp8: raw 4-byte fragments converted with the row scale; s2 / reg from the stored norms
  constexpr bool kRaw = F::kScaled;
  constexpr bool kNorm = F::kScaled;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, t = lane % LPR;
  const int nv = a.Kp / EPL;
  const bool tact = t < nv;
  const int tE = tact ? t : nv - 1;        // clamped: loads never leave the row
  const float tmask = tact ? 1.f : 0.f;
  const uint32_t coff = (uint32_t)(tE * EPL * (int)sizeof(TV));  // this lane's column byte offset
  // (local step) byte base of this lane's fragment and the row stride in bytes (< 2^32: host-checked)
  const char* vbytes = reinterpret_cast<const char*>(a.v) + coff;
  const uint32_t vsb = (uint32_t)(a.v_stride * (long long)sizeof(TV));
  const bool self_on = SH && a.self.u1 > a.self.u0;  // (uniform)
  const uint32_t tsb = self_on ? (uint32_t)(a.self.v_stride * (long long)sizeof(TV)) : vsb;
  // (SH) byte bases of this lane's fragment in the wire rows and in the own table rows
  const uint64_t wbase = reinterpret_cast<uint64_t>(a.v) + coff;
  const uint64_t sbase = self_on ? reinterpret_cast<uint64_t>(a.self.v) + coff : wbase;
  const int wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * kWavesPerBlock;
  const bool want_reg = a.reg_partial != nullptr;
  // (segment lookup + self rows: the key range of the own segments, read once)
  const bool self_key = SH && self_on && a.seg_idx != nullptr;
  const int self_kmin = self_key ? a.self.keys[a.self.u0] : 0;
  const int self_kmax = self_key ? a.self.keys[a.self.u1 - 1] : -1;
  const int wv = threadIdx.x >> 6;

  float loss_acc = 0.f, regv_acc = 0.f, regw_acc = 0.f;
  // Software pipeline over the wave's examples i, i + nwaves, ...: an example's chain is CSR
  // offsets -> its (row, value) pairs -> its rows (and w); without the pipeline each example paid
  // the three dependent latencies in turn (the forward ran latency-bound: 4 waves / SIMD, one
  // example each).  Here the offsets are loaded two examples ahead and the first 64 (row, value)
  // pairs one example ahead, so while example i's rows are in flight the next example's pairs
  // are too, and example i starts with its pairs already in registers: one latency per example.
  // (Longer examples load their further 64-wide pieces in place.)
  constexpr bool kPrefetch = FM_FWD_PREFETCH;  // (A/B build variant "fwdnopf": 0)
  auto pairs = [&](int base, int m, int& row, float& x) {
    row = 0;
    x = 0.f;
    if (lane < m) {
      row = a.rows[base + lane];
      x = a.vals ? a.vals[base + lane] : 1.f;
    }
  };
  int s = 0, e = 0, sn = 0, en = 0;
  int p_row = 0;
  float p_x = 0.f;
  if (wave < a.B) {
    s = a.offsets[wave];
    e = a.offsets[wave + 1];
    if (kPrefetch) pairs(s, min(kWave, e - s), p_row, p_x);
  }
  if (wave + nwaves < a.B) {
    sn = a.offsets[wave + nwaves];
    en = a.offsets[wave + nwaves + 1];
  }
  for (int i = wave; i < a.B; i += nwaves) {
    // next example's first pairs (its offsets arrived an example ago), the offsets after it
    int n_row = 0;
    float n_x = 0.f;
    if (kPrefetch) pairs(sn, i + nwaves < a.B ? min(kWave, en - sn) : 0, n_row, n_x);
    int snn = 0, enn = 0;
    if (i + 2 * nwaves < a.B) {
      snn = a.offsets[i + 2 * nwaves];
      enn = a.offsets[i + 2 * nwaves + 1];
    }
    // label / weight of example i: needed after the reduction, loaded now
    float y_pre = 0.f, wt_pre = 1.f;
    if (kPrefetch && a.loss_type != kLossNone && lane == 0) {
      y_pre = a.labels[i];
      if (a.weights) wt_pre = a.weights[i];
    }
    float s1[EPL], s2[EPL];
#pragma unroll
    for (int k = 0; k < EPL; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
    float lin = 0.f, rv = 0.f, rw = 0.f;
    float s2n = 0.f;  // (kNorm) sum_j x_j^2 |v_j|^2, one occurrence per lane
    for (int base = s; base < e; base += kWave) {
      const int m = min(kWave, e - base);
      int my_row = 0;
      float my_x = 0.f, my_w = 0.f, my_s = 1.f, my_n2 = 0.f;
      uint32_t my_t = 0;  // (SH) the occurrence's row in its source, bit 31: an own (table) row
      if (kPrefetch && base == s) {
        my_row = p_row;
        my_x = p_x;
      } else {
        pairs(base, m, my_row, my_x);
      }
      if constexpr (!SH) {
        if (lane < m) {
          if constexpr (kNorm) {  // [w, scale, |v|^2, pad]: one 16-byte load (w_stride 4, host-checked)
            const float4 wr = *reinterpret_cast<const float4*>(a.w + (uint64_t)(uint32_t)my_row * 4u);
            my_w = wr.x;
            my_s = wr.y;
            my_n2 = wr.z;
          } else {
            my_w = a.w[(long long)my_row * a.w_stride];
          }
        }
      } else {
        if (lane < m) {
          // segment lookup mode: rows[] are keys; an own row is known by its key alone (the self
          // segments are exactly the batch's keys in [self_kmin, self_kmax]), so it needs neither
          // the lookup nor the segment's key load -- at world 1 every row
          const int key = my_row;
          const bool own_key = self_key && key >= self_kmin && key <= self_kmax;
          if (a.seg_idx && !own_key) my_row = seg_lookup(a, key);
          // the linear weight (fp8: with scale and norm, one 16-byte tail) of occurrence `lane`,
          // one lane-parallel load per 64 occurrences instead of one per row group
          const bool own = own_key || (self_on && !self_key && a.self.has(my_row));
          const long long r = own ? (own_key ? (long long)key - a.self.base : a.self.row(my_row)) : my_row;
          my_t = (uint32_t)r | (own ? 0x80000000u : 0u);  // (rows < 2^31: host-checked strides / counts)
          const uint64_t wp = reinterpret_cast<uint64_t>(own ? a.self.w + r * a.self.w_stride : a.w + r * a.w_stride);
          if constexpr (kNorm) {  // [w, scale, |v|^2, tag] wire tails / [w, scale, |v|^2, pad] table rows
            const gf4 wr = *gptr<gf4>(wp);
            my_w = wr.x;
            my_s = wr.y;
            my_n2 = wr.z;
          } else {
            my_w = *gptr<float>(wp);
          }
        }
        // lanes past the example take lane 0's row: the wrapped slots of a round read a valid row
        const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)my_t);
        if (lane >= m) my_t = t0;
      }

      for (int q = 0; q < m; q += G * UNR) {
        float fr[UNR][EPL], fx[UNR], fs[UNR];
        int fraw[kRaw ? UNR : 1];
        // Issue every row load of the round before the first use.  Loads are unconditional (slots
        // past the example read a valid row -- lanes past it hold row 0 / lane 0's row -- and are
        // masked to zero afterwards), so hipcc keeps all UNR loads in flight.  Lanes past the round
        // wrap around the wave (ds_bpermute takes the lane modulo 64).
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int f = q + u * G + g;
          const int fb = (f & (kWave - 1)) << 2;
          const float x = __int_as_float(__builtin_amdgcn_ds_bpermute(fb, __float_as_int(my_x)));
          fx[u] = f < m ? x : 0.f;
          if constexpr (SH) {
            // one broadcast per row group: the tagged row, then its source's base and stride (the
            // 64-bit address in two broadcasts: k16 bf16 0.525 -> 0.518 ms, k128 fp8 0.864 -> 0.857,
            // k64 tied; profiles/r5/emit_ab.txt)
            const uint32_t tr = (uint32_t)__builtin_amdgcn_ds_bpermute(fb, (int)my_t);
            const bool own = (tr >> 31) != 0;
            const uint64_t pr = (own ? sbase : wbase) + (uint64_t)(tr & 0x7fffffffu) * (own ? tsb : vsb);
            if constexpr (kRaw) fraw[u] = *gptr<int>(pr);
            else F::load_g(pr, fr[u]);
          } else {
            const int row = __builtin_amdgcn_ds_bpermute(fb, my_row);
            const char* rp = vbytes + (uint64_t)(uint32_t)row * vsb;
            if constexpr (kRaw) fraw[u] = *reinterpret_cast<const int*>(rp);
            else F::load(reinterpret_cast<const TV*>(rp), fr[u]);
          }
          if constexpr (F::kScaled) fs[u] = __int_as_float(__builtin_amdgcn_ds_bpermute(fb, __float_as_int(my_s)));
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          float (&fv)[EPL] = fr[u];
          // (folding the fp8 row scale into the occurrence's x instead of every element, with the
          // reg term as a per-occurrence sum times scale^2 -- fewer VALU ops -- made the k128 fp8
          // FTRL step slower, 0.888 -> 1.014 ms same-box: profiles/r4/specialize_ab.txt)
          if constexpr (kRaw) F::cvt_scaled(fraw[u], fs[u], fv);
          const float xm = fx[u] * tmask;
#pragma unroll
          for (int k = 0; k < EPL; ++k) {
            const float xv = xm * fv[k];
            s1[k] += xv;
            if constexpr (!kNorm) s2[k] += xv * xv;
          }
          if (!kNorm && want_reg) {
            const float ok = (q + u * G + g) < m ? 1.f : 0.f;
#pragma unroll
            for (int k = 0; k < EPL; ++k) rv += ok * tmask * fv[k] * fv[k];
          }
        }
      }
      // (w is used after the row loads were issued: its load latency hides under theirs)
      lin += my_x * my_w;
      if (want_reg) rw += my_w * my_w;
      if constexpr (kNorm) {  // (lanes past the example: x = 0; their norm is not summed)
        s2n += my_x * my_x * my_n2;
        if (want_reg && lane < m) rv += my_n2;
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
    if constexpr (kNorm) part -= group_sum<kWave>(s2n);
    lin = group_sum<kWave>(lin);
    const float pred = lin + 0.5f * part + (a.bias ? a.bias[0] : 0.f);
    if (a.r1 != nullptr && g == 0 && tact) store_r1<TV, EPL>(a.r1, (long long)i * a.Kp + t * EPL, s1);
    if (want_reg) {
      rv = group_sum<kWave>(rv);
      rw = group_sum<kWave>(rw);
      regv_acc += rv;
      regw_acc += rw;
    }
    // loss and dL/dpred (every lane holds the same pred: butterfly sums are lane-symmetric)
    float l = 0.f, d = 0.f;
    if (a.loss_type != kLossNone && lane == 0) {
      const float y = kPrefetch ? y_pre : a.labels[i];
      const float wt = kPrefetch ? wt_pre : (a.weights ? a.weights[i] : 1.f);
      if (a.loss_type == kLossMse) {
        const float diff = pred - y;
        l = wt * diff * diff;
        d = 2.f * wt * diff;
      } else {
        // sigmoid_cross_entropy_with_logits, numerically stable form
        l = wt * (fmaxf(pred, 0.f) - pred * y + softplus_neg_abs(pred));
        d = wt * (sigmoidf(pred) - y);
      }
    }
    if (lane == 0) {
      a.pred[i] = pred;
      if (a.loss_type != kLossNone) {
        loss_acc += l;
        if (a.dpred) a.dpred[i] = d * a.grad_scale;
      }
    }
    s = sn; e = en; sn = snn; en = enn;
    p_row = n_row; p_x = n_x;
  }
  if (a.loss_partial == nullptr && a.reg_partial == nullptr) return;
  __shared__ float red[3][kWavesPerBlock];
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

template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(fwd_local_min_waves<LPR, TV>())))
void fm_fwd_kernel(FwdArgs a) {
  fwd_body<LPR, TV, false>(a);
}

// The row-sharded step's forward (self rows, segment lookup).
template <int LPR, typename TV>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(fwd_local_min_waves<LPR, TV, true>())))
void fm_fwd_shard_kernel(FwdArgs a) {
  fwd_body<LPR, TV, true>(a);
}

// The matrix-core form of the fp8 k=128 forward is a build variant ("mfma": -DFM_WITH_MFMA=1), not part
// of the default module: built, correct, and slower than the VALU kernel twice over -- the forward is
// bound by its random row gathers, not by its arithmetic (profiles/r5/fwd_mfma_ab.txt).
#ifndef FM_WITH_MFMA
#define FM_WITH_MFMA 0
#endif
#if FM_WITH_MFMA
#include "fm_fwd_mfma.hip"
#endif

// Expand CSR offsets into the example index of every occurrence.
// Example of every CSR occurrence; with slot_bits > 0 the packed occurrence code
// (example << slot_bits) | (position inside the example), which the dedup sort
// carries as its payload: the example and, through offsets, the occurrence
// index both decode from it without a gather.
// One wave per 64 consecutive examples: lane l holds offsets[i0 + l]; the wave then
// walks the group's occurrences 64 at a time (one fully coalesced 256-B store per
// step) and each lane finds its example by a 6-step binary search over the lanes'
// offsets (ds_bpermute, no LDS).  (The earlier wave-per-example form left 25 of 64
// lanes idle per store and paid two dependent offset loads per 39 writes: 63-106 us
// for 5.1M occurrences next to the forward.)
__global__ __launch_bounds__(kBlock) void csr_rows_kernel(int B, const int* offsets, int* ex_of_occ, int slot_bits) {
  const int lane = threadIdx.x & (kWave - 1);
  const int ngroups = (B + kWave - 1) / kWave;
  const int nwaves = gridDim.x * kWavesPerBlock;
  for (int g = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
    const int i0 = g * kWave;
    const int n = min(kWave, B - i0);
    const int o = offsets[i0 + min(lane, n)];  // lanes >= n hold the group's end
    const int s = __shfl(o, 0);
    const int e = offsets[i0 + n];
    for (int base = s; base < e; base += kWave) {  // wave-uniform trip count: every lane shuffles
      const int p = base + lane;
      int k = 0;
#pragma unroll
      for (int step = kWave / 2; step > 0; step >>= 1) {
        const int c = k + step;
        if (__shfl(o, c) <= p) k = c;
      }
      const int ok = __shfl(o, k);  // (all lanes active: shuffles stay outside the store guard)
      if (p < e) {
        const int ex = i0 + k;
        ex_of_occ[p] = slot_bits > 0 ? (ex << slot_bits) | (p - ok) : ex;
      }
    }
  }
}

// "mfma" build variant: fp8 k=128 batches of binary features take the matrix-core kernel
// (fm_fwd_mfma.hip) while set_fwd_mfma(true) (its default); the default module has no such kernel.
static bool g_fwd_mfma = FM_WITH_MFMA;
bool fwd_mfma_enabled() { return g_fwd_mfma; }
void set_fwd_mfma(bool on) { g_fwd_mfma = FM_WITH_MFMA && on; }

int fwd_grid(int B) { return fill_grid(B, kWavesPerBlock, 4096); }

int launch_fwd(const FwdArgs& a, int dtype, int grid, hipStream_t st) {
  if (a.B <= 0) return 0;
  const int lpr = lanes_per_row(a.Kp, dtype);
  // (capping the forward's workgroups per CU through dynamic LDS, as the chunk backward does, tied
  // on k64 fp32: profiles/r4/wg_per_cu_ab.txt)
  // fp8 rows: [w, scale, |v|^2, .] tails read as one 16-byte load (table rows: w_stride 4; wire
  // rows: the 16-byte tail after the factor bytes) -- for the wire / self sources as well
  if (dtype == kFP8) {
    auto aligned = [](const float* w, long long ws) { return ((uintptr_t)w & 15) == 0 && ws % 4 == 0; };
    if (!aligned(a.w, a.w_stride) || (a.self.u1 > a.self.u0 && !aligned(a.self.w, a.self.w_stride))) return -7;
  }
  const bool table_rows = dtype != kFP8 || a.w_stride == 4;  // (the local kernel's fp8 tails: w + 4 row)
#if FM_WITH_MFMA
  // fp8 rows on the matrix cores (fm_fwd_mfma.hip): binary features, Kp = 128, table rows, tiles of 16
  // examples within the kernel's LDS row capacity.
  if (fwd_mfma_enabled() && dtype == kFP8 && a.Kp == kMfRowB && a.v_stride == kMfRowB && !a.vals && table_rows &&
      a.self.u1 <= a.self.u0 && !a.seg_idx && a.max_feats > 0 && a.max_feats * kMfT <= kMfMaxRows) {
    hipLaunchKernelGGL(fm_fwd_mfma_fp8_kernel, dim3(grid), dim3(kBlock), 0, st, a);
    return (int)hipGetLastError();
  }
#endif

  if (a.self.u1 > a.self.u0 || a.seg_idx || !FM_FWD_SPECIALIZE || !table_rows) {
    FM_DISPATCH(dtype, lpr, fm_fwd_shard_kernel, grid, st, a);
  } else {
    FM_DISPATCH(dtype, lpr, fm_fwd_kernel, grid, st, a);
  }
  return (int)hipGetLastError();
}

int launch_csr_rows(int B, const int* offsets, int* ex_of_occ, int slot_bits, hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(csr_rows_kernel, dim3(fill_grid((B + kWave - 1) / kWave, kWavesPerBlock, 4096)), dim3(kBlock), 0, st, B,
                     offsets, ex_of_occ, slot_bits);
  return (int)hipGetLastError();
}

}  // namespace fm
