// Shared device helpers for the gfx950 FM kernels.
//
// Conventions used by every kernel in this directory
//  * wave64: lane = threadIdx.x & 63, 256-thread workgroups (4 waves).
//  * Factor rows are stored "v-first": a row of the V table holds Kp factor
//    values (Kp = K rounded up so that one lane moves exactly 16 bytes), the
//    linear weight w lives in a separate fp32 array (or at column Kp of a packed
//    exchange row).  The reference keeps w at column 0 of a [V, K+1] block
//    (fm_model.py:270-284); the checkpoint exporter restores that layout.
//  * A row is read by LPR lanes ("lanes per row", a power of two) with one
//    16-byte load each, so one wave instruction moves G = 64/LPR whole rows.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdint>

namespace fm {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

// Chunk descriptor word (dedup.hip emit -> fm_bwd.hip): segment id | flags.
constexpr int kChunkSegMask = (1 << 30) - 1;
constexpr int kChunkFirst = 1 << 30;         // first chunk of its segment
constexpr unsigned kChunkSingle = 1u << 31;  // the segment's only chunk

// Sticky device error word (one per device; bits below), set by kernels that detect an invalid result
// they cannot signal otherwise without a host sync; read and cleared by the host
// (module device_errors(), ops/kernels.py check_device_errors).
constexpr int kDevErrSort = 1;  // in-tree radix sort: a look-back spin bound was hit (dedup plan invalid)
__device__ int g_fm_dev_error = 0;

enum LossType : int { kLossNone = 0, kLossMse = 1, kLossLogistic = 2 };
enum OptType : int { kOptAdagrad = 0, kOptFtrl = 1, kOptSgd = 2 };
enum DType : int { kF32 = 0, kBF16 = 1, kFP8 = 2 };

// fp8 table storage: OCP e4m3 (gfx950 v_cvt_pk_*_fp8) with one fp32 scale per
// row, stored next to the row's linear weight (w[row * w_stride + 1], w_stride
// = 2), so the scale arrives with the w load.  A row is quantised as
// q = v / s with s = max|v| / kFp8Max (round to nearest even).
struct fp8e4m3 { uint8_t bits; };
constexpr float kFp8Max = 448.f;

// ---- stochastic rounding -----------------------------------------------------
// Low-precision tables (bf16 / fp8) store updated rows with stochastic rounding
// when a step seed is given (0 = round to nearest even): small Adagrad / FTRL
// steps then survive in expectation instead of being rounded away.  The random
// bits are a hash of (step seed, table row, column): deterministic run to run.
__device__ inline uint32_t sr_hash(uint32_t seed, uint32_t row, uint32_t col) {
  uint32_t h = seed ^ (row * 0x9E3779B1u) ^ (col * 0x85EBCA77u);
  h ^= h >> 16; h *= 0x7feb352du;
  h ^= h >> 15; h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

// Next random word of a lane's stream (xorshift32: one hash per lane, not per element).
__device__ inline uint32_t sr_next(uint32_t r) {
  r ^= r << 13; r ^= r >> 17; r ^= r << 5;
  return r;
}

// fp8 tables (factors with 3 mantissa bits, bf16 optimizer state) take a cheaper row-update
// epilogue: FTRL's square roots and divides on v_sqrt / v_rcp (1 ulp) instead of the correctly
// rounded expansions, and the stochastic-rounding words of a lane's 4 values as rotations of ONE
// hash instead of a hash plus a 3-step xorshift chain (each rotation's bits are uniform on their
// own, which is all an unbiased rounding needs).  The k128 fp8 FTRL chunk backward is VALU-bound
// with its per-row epilogue as large as its occurrence loop (profiles/r6/fp8_epilogue_ab.txt).
// FM_FP8_FAST_EPI=0 (build variant "fp8slow") keeps the exact forms: the A/B.
#ifndef FM_FP8_FAST_EPI
#define FM_FP8_FAST_EPI 1
#endif
__device__ inline uint32_t sr_rot(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, s); }
// random word i (0..3) of a lane's 4 values from one hash
__device__ inline uint32_t sr_word(uint32_t r0, int i) {
  if (!FM_FP8_FAST_EPI) {
    for (int k = 0; k < i; ++k) r0 = sr_next(r0);
    return r0;
  }
  return i == 0 ? r0 : sr_rot(r0, i == 1 ? 16 : i == 2 ? 8 : 24);
}

// A computed address (e.g. broadcast between lanes) as a global-memory pointer: without the
// address space hipcc emits flat loads, which count against both vmcnt and lgkmcnt and make every
// wait a full drain (the sharded forward's row loads: profiles/r5).
template <typename T>
__device__ inline const __attribute__((address_space(1))) T* gptr(uint64_t addr) {
  return reinterpret_cast<const __attribute__((address_space(1))) T*>(addr);
}
typedef float gf4 __attribute__((ext_vector_type(4)));      // (HIP's float4 / uint2 have no copy
typedef uint32_t gu2 __attribute__((ext_vector_type(2)));   //  constructor from address_space(1))

// ---- 16-byte row fragments ------------------------------------------------
template <typename T> struct Frag;

template <> struct Frag<float> {
  static constexpr int N = 4;  // elements per lane
  static constexpr bool kScaled = false;
  __device__ static inline void load(const float* p, float (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static inline void load_g(uint64_t a, float (&o)[4]) {
    const gf4 v = *gptr<gf4>(a);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static inline void store(float* p, const float (&o)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
  __device__ static inline void store_sr(float* p, const float (&o)[4], uint32_t, uint32_t, uint32_t) { store(p, o); }
};

__device__ inline float bf16_bits_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
// Round-to-nearest-even f32 -> bf16 bits (NaN stays NaN: quiet bit forced).
__device__ inline uint32_t f32_to_bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (u >> 16) | 0x40u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// Stochastically rounded f32 -> bf16 bits: add 16 random bits below the kept
// mantissa, truncate (Inf / NaN pass through).
__device__ inline uint32_t f32_to_bf16_bits_sr(float f, uint32_t r) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0x7fffffu) ? 0x40u : 0u);
  return (u + (r & 0xffffu)) >> 16;
}

// 4 bf16 per lane (an 8-byte load): the same lane mapping and fp32 register
// footprint as an fp32 row (a K=64 row is one 16-lane instruction).  With 16-byte
// fragments (8 values per lane) the backward chunk kernel needed 185 VGPRs (2
// waves/SIMD) and the k=64 bf16 step was slower than the fp32 one.
template <> struct Frag<__hip_bfloat16> {
  static constexpr int N = 4;
  static constexpr bool kScaled = false;
  __device__ static inline void load(const __hip_bfloat16* p, float (&o)[4]) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    o[0] = bf16_bits_to_f32(v.x & 0xffffu);
    o[1] = bf16_bits_to_f32(v.x >> 16);
    o[2] = bf16_bits_to_f32(v.y & 0xffffu);
    o[3] = bf16_bits_to_f32(v.y >> 16);
  }
  __device__ static inline void load_g(uint64_t a, float (&o)[4]) {
    const gu2 v = *gptr<gu2>(a);
    o[0] = bf16_bits_to_f32(v.x & 0xffffu);
    o[1] = bf16_bits_to_f32(v.x >> 16);
    o[2] = bf16_bits_to_f32(v.y & 0xffffu);
    o[3] = bf16_bits_to_f32(v.y >> 16);
  }
  __device__ static inline void store(__hip_bfloat16* p, const float (&o)[4]) {
    uint2 v;
    v.x = f32_to_bf16_bits(o[0]) | (f32_to_bf16_bits(o[1]) << 16);
    v.y = f32_to_bf16_bits(o[2]) | (f32_to_bf16_bits(o[3]) << 16);
    *reinterpret_cast<uint2*>(p) = v;
  }
  __device__ static inline void store_sr(__hip_bfloat16* p, const float (&o)[4], uint32_t seed, uint32_t row,
                                         uint32_t col) {
    uint32_t b[4];
    uint32_t r = sr_hash(seed, row, col);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      b[k] = f32_to_bf16_bits_sr(o[k], r);
      r = sr_next(r);
    }
    *reinterpret_cast<uint2*>(p) = make_uint2(b[0] | (b[1] << 16), b[2] | (b[3] << 16));
  }
};

// Scale of an fp8 row whose largest |value| is m: the power of two s with m / s in (224, 448] -- an
// E8M0 exponent, as the OCP MX formats use.  fp8 keeps 3 mantissa bits at any binade, so a power of
// two costs no precision against s = m / 448 (one binade of subnormal range at most), and it makes
// quantising (v * (1 / s)) and dequantising (q * s) exact scalings; gfx950's scaled conversion
// v_cvt_scalef32_pk_f32_fp8 applies only the scale's exponent, so it dequantises in the conversion.
__host__ __device__ inline float fp8_row_scale(float m) {
  if (!(m > 0.f)) return 1.f;
  const float t = m / kFp8Max;
  if (t < 1.17549435e-38f) return 1.17549435e-38f;  // (2^-126: m / s < 448 still)
  const uint32_t b = __builtin_bit_cast(uint32_t, t);
  return (b & 0x7fffffu) ? __builtin_bit_cast(float, (b & 0x7f800000u) + 0x00800000u) : t;
}

// 4 fp8 per lane (a 4-byte load: a K=128 row is one 32-lane instruction, the
// same lane mapping and register footprint as fp32); values are unscaled here.
template <> struct Frag<fp8e4m3> {
  static constexpr int N = 4;
  static constexpr bool kScaled = true;
  __device__ static inline void cvt(int u, float (&o)[4]) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(u, false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(u, true);
    o[0] = lo[0]; o[1] = lo[1]; o[2] = hi[0]; o[3] = hi[1];
  }
  __device__ static inline void load(const fp8e4m3* p, float (&o)[4]) { cvt(*reinterpret_cast<const int*>(p), o); }
  __device__ static inline void load_g(uint64_t a, float (&o)[4]) { cvt(*gptr<int>(a), o); }
  // q * s for a power-of-two row scale s (fp8_row_scale) in the conversion instruction itself
  __device__ static inline void cvt_scaled(int u, float s, float (&o)[4]) {
    const auto lo = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(u, s, false);
    const auto hi = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(u, s, true);
    o[0] = lo[0]; o[1] = lo[1]; o[2] = hi[0]; o[3] = hi[1];
  }
  // the 4 bytes of 4 values (round to nearest even)
  __device__ static inline int pack(const float (&o)[4]) {
    int u = __builtin_amdgcn_cvt_pk_fp8_f32(o[0], o[1], 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(o[2], o[3], u, true);
  }
  // gfx950 v_cvt_sr_fp8_f32: hardware stochastic rounding with the given random bits (values of
  // columns col .. col + 3 of `row`)
  __device__ static inline int pack_sr(const float (&o)[4], uint32_t seed, uint32_t row, uint32_t col) {
    const uint32_t r0 = sr_hash(seed, row, col);
    int u = __builtin_amdgcn_cvt_sr_fp8_f32(o[0], (int)r0, 0, 0);
    u = __builtin_amdgcn_cvt_sr_fp8_f32(o[1], (int)sr_word(r0, 1), u, 1);
    u = __builtin_amdgcn_cvt_sr_fp8_f32(o[2], (int)sr_word(r0, 2), u, 2);
    return __builtin_amdgcn_cvt_sr_fp8_f32(o[3], (int)sr_word(r0, 3), u, 3);
  }
  // (store / store_sr return the 4 stored bytes: the row norm is taken from them)
  __device__ static inline int store(fp8e4m3* p, const float (&o)[4]) {
    const int u = pack(o);
    *reinterpret_cast<int*>(p) = u;
    return u;
  }
  __device__ static inline int store_sr(fp8e4m3* p, const float (&o)[4], uint32_t seed, uint32_t row,
                                        uint32_t col) {
    const int u = pack_sr(o, seed, row, col);
    *reinterpret_cast<int*>(p) = u;
    return u;
  }
};

// ---- wave reductions (xor butterfly inside a lane group) -------------------
template <int WIDTH>
__device__ inline float group_sum(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

template <int WIDTH>
__device__ inline float group_max(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// r1 = sum_j x_j v_j of every example, written by the forward and gathered once per
// occurrence by the backward (its largest stream: 5.1M rows of a Criteo-shaped batch).
// fp32 for fp32 / bf16 tables; bf16 for fp8 tables, whose factors carry 3 mantissa bits:
// r1's rounding (2^-9 relative) stays far below the table's own quantisation step (2^-4)
// and the gather halves (k=128: 512 -> 256 B per occurrence).
template <typename TV> struct R1Bf16 { static constexpr bool v = false; };
template <> struct R1Bf16<fp8e4m3> { static constexpr bool v = true; };

// EPL bf16 values (8-byte aligned; 16-byte loads when EPL is a multiple of 8 -- the wide fp8 chunk kernel,
// whose rows and r1 rows are then 16-byte aligned: half the address work per byte of the 8-byte form)
template <int EPL>
__device__ inline void load_bf16x(const uint16_t* p, float (&o)[EPL]) {
  if constexpr (EPL % 8 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 8) {
      const uint4 h = *reinterpret_cast<const uint4*>(p + k);
      o[k] = bf16_bits_to_f32(h.x & 0xffffu); o[k + 1] = bf16_bits_to_f32(h.x >> 16);
      o[k + 2] = bf16_bits_to_f32(h.y & 0xffffu); o[k + 3] = bf16_bits_to_f32(h.y >> 16);
      o[k + 4] = bf16_bits_to_f32(h.z & 0xffffu); o[k + 5] = bf16_bits_to_f32(h.z >> 16);
      o[k + 6] = bf16_bits_to_f32(h.w & 0xffffu); o[k + 7] = bf16_bits_to_f32(h.w >> 16);
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const uint2 h = *reinterpret_cast<const uint2*>(p + k);
      o[k] = bf16_bits_to_f32(h.x & 0xffffu); o[k + 1] = bf16_bits_to_f32(h.x >> 16);
      o[k + 2] = bf16_bits_to_f32(h.y & 0xffffu); o[k + 3] = bf16_bits_to_f32(h.y >> 16);
    }
  }
}

template <typename TV, int EPL>
__device__ inline void load_r1(const void* r1, long long off, float (&o)[EPL]) {
  if constexpr (R1Bf16<TV>::v) {
    load_bf16x<EPL>(reinterpret_cast<const uint16_t*>(r1) + off, o);
  } else {
    const float* p = reinterpret_cast<const float*>(r1) + off;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 f = *reinterpret_cast<const float4*>(p + k);
      o[k] = f.x; o[k + 1] = f.y; o[k + 2] = f.z; o[k + 3] = f.w;
    }
  }
}

template <typename TV, int EPL>
__device__ inline void store_r1(void* r1, long long off, const float (&s)[EPL]) {
  if constexpr (R1Bf16<TV>::v) {
    uint16_t* p = reinterpret_cast<uint16_t*>(r1) + off;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      uint2 h;
      h.x = f32_to_bf16_bits(s[k]) | (f32_to_bf16_bits(s[k + 1]) << 16);
      h.y = f32_to_bf16_bits(s[k + 2]) | (f32_to_bf16_bits(s[k + 3]) << 16);
      *reinterpret_cast<uint2*>(p + k) = h;
    }
  } else {
    float* p = reinterpret_cast<float*>(r1) + off;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) *reinterpret_cast<float4*>(p + k) = make_float4(s[k], s[k + 1], s[k + 2], s[k + 3]);
  }
}

// Optimizer state rows (Adagrad accumulator / FTRL n; FTRL z): fp32, except for fp8 tables.
// Their factors carry 3 mantissa bits, so the state is kept in bf16 (8 bits), stored with
// stochastic rounding when a step seed is given -- sums of small squared gradients survive in
// expectation -- which halves the state's share of the row read-modify-write (k=128 FTRL:
// 1032 -> 516 of 1.17 KB per row).  The bias state (s0w / s1w) stays fp32.
template <typename TV> struct StateBf16 { static constexpr bool v = false; };
template <> struct StateBf16<fp8e4m3> { static constexpr bool v = true; };

template <typename TV, int EPL>
__device__ inline void load_state(const void* s, long long off, float (&o)[EPL]) {
  if constexpr (StateBf16<TV>::v) {
    load_bf16x<EPL>(reinterpret_cast<const uint16_t*>(s) + off, o);
  } else {
    const float* p = reinterpret_cast<const float*>(s) + off;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const float4 f = *reinterpret_cast<const float4*>(p + k);
      o[k] = f.x; o[k + 1] = f.y; o[k + 2] = f.z; o[k + 3] = f.w;
    }
  }
}

// seed: the step's stochastic-rounding seed (0: round to nearest even), salted per state slot
template <typename TV, int EPL>
__device__ inline void store_state(void* s, long long off, const float (&o)[EPL], uint32_t seed, uint32_t row,
                                   uint32_t col) {
  if constexpr (StateBf16<TV>::v) {
    uint16_t* p = reinterpret_cast<uint16_t*>(s) + off;
    // (random bits per 4 values, salted by their first column: the same bits for any EPL)
    uint32_t b[EPL];
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      if (seed) {
        const uint32_t r = sr_hash(seed, row, col + (uint32_t)k);
#pragma unroll
        for (int i = 0; i < 4; ++i) b[k + i] = f32_to_bf16_bits_sr(o[k + i], sr_word(r, i));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) b[k + i] = f32_to_bf16_bits(o[k + i]);
      }
    }
    if constexpr (EPL % 8 == 0) {
#pragma unroll
      for (int k = 0; k < EPL; k += 8)
        *reinterpret_cast<uint4*>(p + k) = make_uint4(b[k] | (b[k + 1] << 16), b[k + 2] | (b[k + 3] << 16),
                                                      b[k + 4] | (b[k + 5] << 16), b[k + 6] | (b[k + 7] << 16));
    } else {
#pragma unroll
      for (int k = 0; k < EPL; k += 4)
        *reinterpret_cast<uint2*>(p + k) = make_uint2(b[k] | (b[k + 1] << 16), b[k + 2] | (b[k + 3] << 16));
    }
  } else {
    float* p = reinterpret_cast<float*>(s) + off;
#pragma unroll
    for (int k = 0; k < EPL; k += 4) *reinterpret_cast<float4*>(p + k) = make_float4(o[k], o[k + 1], o[k + 2], o[k + 3]);
  }
}
constexpr uint32_t kSrSalt0 = 0x68e31da4u, kSrSalt1 = 0xb5297a4du;  // per state slot

// Dequantisation factor of a table row (1 for unscaled dtypes).
template <typename TV>
__device__ inline float row_scale(const float* w, long long row, long long w_stride) {
  if constexpr (Frag<TV>::kScaled) return w[row * w_stride + 1];
  return 1.f;
}

// fp8 rows keep their squared L2 norm next to [w, scale] (w_row[2], kFp8Norm): the local
// forward's s2 and reg terms are then one scalar per occurrence (sum_j x_j^2 |v_j|^2, sum_j |v_j|^2)
// instead of two multiply-adds per element.  The norm is a function of the stored bytes only:
// exact squares of the unscaled values, summed in a fixed order per lane and a butterfly over the
// row's LPR lanes, times scale^2 (a power of two: exact) -- every writer (store_row, the init /
// refresh kernels) calls this, so they agree bitwise.  `u`: the lane's 4 stored fp8 values.
constexpr int kFp8Norm = 2;  // word of the norm in an fp8 table's w row [w, scale, |v|^2, pad]
template <int LPR>
__device__ inline float fp8_norm2(int u, float s, bool tact) {
  float q[4];
  Frag<fp8e4m3>::cvt(u, q);
  float p = tact ? __fmaf_rn(q[0], q[0], __fmaf_rn(q[1], q[1], __fmaf_rn(q[2], q[2], q[3] * q[3]))) : 0.f;
  p = group_sum<LPR>(p);
  return p * (s * s);
}

// Store this lane's EPL fp32 values of a row (every lane of the LPR group must
// call: scaled dtypes reduce the row's max |v| over the group first).
template <int LPR, typename TV>
__device__ inline void store_row(TV* lane_ptr, const float (&o)[Frag<TV>::N], float* w, long long row,
                                 long long w_stride, int t, bool tact, uint32_t sr_seed = 0) {
  using F = Frag<TV>;
  const uint32_t col = (uint32_t)(t * F::N);
  if constexpr (F::kScaled) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < F::N; ++k) m = fmaxf(m, fabsf(o[k]));
    m = group_max<LPR>(m);
    const float s = fp8_row_scale(m);
    const float inv = 1.f / s;  // (exact: s is a power of two)
    float q[F::N];
#pragma unroll
    for (int k = 0; k < F::N; ++k) q[k] = fminf(fmaxf(o[k] * inv, -kFp8Max), kFp8Max);
    int u = 0;
    if (tact) u = sr_seed ? F::store_sr(lane_ptr, q, sr_seed, (uint32_t)row, col) : F::store(lane_ptr, q);
    const float n2 = fp8_norm2<LPR>(u, s, tact);
    if (t == 0) {
      w[row * w_stride + 1] = s;
      w[row * w_stride + kFp8Norm] = n2;
    }
  } else {
    if (tact) {
      if (sr_seed) F::store_sr(lane_ptr, o, sr_seed, (uint32_t)row, col);
      else F::store(lane_ptr, o);
    }
  }
}

// store_row for fp8 rows held 8 values per lane (the wide chunk kernel, LPR = Kp / 8): the same bytes,
// row scale and norm as store_row<2 LPR, fp8> over 4-value lanes -- lane t's halves are the 4-value
// lanes 2t and 2t + 1 (their stochastic-rounding columns), and the norm's butterfly is theirs: over the
// halves' partner lanes first, the two halves added last (the 4-value butterfly's last step).
template <int LPR>
__device__ inline void store_row_fp8x8(fp8e4m3* lane_ptr, const float (&o)[8], float* w, long long row,
                                       long long w_stride, int t, bool tact, uint32_t sr_seed) {
  using F = Frag<fp8e4m3>;
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(o[k]));
  m = group_max<LPR>(m);
  const float s = fp8_row_scale(m);
  const float inv = 1.f / s;  // (exact: s is a power of two)
  float qa[4], qb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    qa[k] = fminf(fmaxf(o[k] * inv, -kFp8Max), kFp8Max);
    qb[k] = fminf(fmaxf(o[k + 4] * inv, -kFp8Max), kFp8Max);
  }
  const uint32_t col = (uint32_t)(t * 8);
  int ua = 0, ub = 0;
  if (tact) {
    ua = sr_seed ? F::pack_sr(qa, sr_seed, (uint32_t)row, col) : F::pack(qa);
    ub = sr_seed ? F::pack_sr(qb, sr_seed, (uint32_t)row, col + 4) : F::pack(qb);
    *reinterpret_cast<uint2*>(lane_ptr) = make_uint2((uint32_t)ua, (uint32_t)ub);
  }
  float pa[4], pb[4];
  F::cvt(ua, pa);
  F::cvt(ub, pb);
  float na = tact ? __fmaf_rn(pa[0], pa[0], __fmaf_rn(pa[1], pa[1], __fmaf_rn(pa[2], pa[2], pa[3] * pa[3]))) : 0.f;
  float nb = tact ? __fmaf_rn(pb[0], pb[0], __fmaf_rn(pb[1], pb[1], __fmaf_rn(pb[2], pb[2], pb[3] * pb[3]))) : 0.f;
  na = group_sum<LPR>(na);
  nb = group_sum<LPR>(nb);
  const float n2 = (na + nb) * (s * s);
  if (t == 0) {
    w[row * w_stride + 1] = s;
    w[row * w_stride + kFp8Norm] = n2;
  }
}

// Wide fp8 kernels (FM_FP8_WIDE=1, default): k = 128 fp8 rows reduced / updated with 8 values per lane --
// 8-byte row loads, 16-byte r1 / optimizer-state / bf16-gradient accesses, LPR = Kp / 8 -- instead of 4
// (4-, 8- and 8-byte accesses): the same bytes with half the per-lane addresses, which the gather-bound
// kernels spend their texture-address time on, and twice the rows per wave.  The chunk backward (local and
// EMIT kinds) and the owner apply; bitwise the same results (store_row_fp8x8).  0 keeps the 4-value kernels
// (the "fp8narrow" build variant, A/B).
#ifndef FM_FP8_WIDE
#define FM_FP8_WIDE 1
#endif

// EPL values of a table row for this lane: one Frag, or -- the wide fp8 kernel -- 8 fp8 values in
// one 8-byte load.
template <typename TV, int EPL>
__device__ inline void frag_load(const TV* p, float (&o)[EPL]) {
  if constexpr (EPL == Frag<TV>::N) {
    Frag<TV>::load(p, o);
  } else {
    static_assert(std::is_same<TV, fp8e4m3>::value && EPL == 8, "wide rows: fp8, 8 values per lane");
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    float lo[4], hi[4];
    Frag<TV>::cvt((int)u.x, lo);
    Frag<TV>::cvt((int)u.y, hi);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = lo[k];
      o[k + 4] = hi[k];
    }
  }
}
template <int LPR, typename TV, int EPL>
__device__ inline void store_row_e(TV* lane_ptr, const float (&o)[EPL], float* w, long long row, long long w_stride,
                                   int t, bool tact, uint32_t sr) {
  if constexpr (EPL == Frag<TV>::N) store_row<LPR, TV>(lane_ptr, o, w, row, w_stride, t, tact, sr);
  else store_row_fp8x8<LPR>(lane_ptr, o, w, row, w_stride, t, tact, sr);
}

// Per-step seed of the stochastic rounding (device counter ticked once per training
// step, so hipGraph replays draw fresh bits); 0 = round to nearest even.
__device__ inline uint32_t sr_step_seed(const int* counter) {
  return counter ? (sr_hash((uint32_t)*counter, 0x5bd1e995u, 0x1b873593u) | 1u) : 0u;
}

// Sum over the row groups of a wave: lanes t, t+LPR, t+2*LPR, ...
template <int LPR>
__device__ inline float across_groups_sum(float v) {
#pragma unroll
  for (int o = LPR; o < kWave; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ inline float softplus_neg_abs(float p) {  // log(1 + exp(-|p|))
  return log1pf(__expf(-fabsf(p)));
}

__device__ inline float sigmoidf(float p) { return 1.f / (1.f + __expf(-p)); }

// Optimizer hyper-parameters, passed by value in kernargs.
struct OptParams {
  int type;          // OptType
  float lr;          // learning rate (adagrad / sgd) or alpha (ftrl)
  float l1, l2;      // ftrl regularisers
  float beta;        // ftrl beta
};

// Row-sharded step, the rows this rank owns ("self rows", parallel/exchange.py): segments
// [u0, u1) of the batch's sorted unique keys are this rank's own table rows (row = key -
// base).  The forward and the backward read them straight from the table instead of the
// gathered wire buffer (no owner gather, no early copy to patch), and the backward applies
// the optimizer in place to the exclusive ones -- rows no other rank requested this step,
// whose whole gradient is this rank's -- instead of emitting a gradient row for the owner's
// apply.  Empty range: off.
struct SelfRows {
  int u0, u1;
  long long base;           // key of local row 0 (rank * rows per shard)
  const int* keys;          // [U] segment keys
  const int* excl;          // [u1 - u0] 1 = exclusive (applied in place); null = all exclusive
  const void* v; long long v_stride;   // table rows (elements of the table dtype)
  float* w; long long w_stride;        // table linear weights (fp8: scale at w + 1)
  __device__ inline bool has(int u) const { return u >= u0 && u < u1; }
  __device__ inline bool exclusive(int u) const { return excl == nullptr || excl[u - u0] != 0; }
  __device__ inline long long row(int u) const { return (long long)keys[u] - base; }
};

// In-place per-element optimizer step on fp32 registers. `s0`/`s1` are the
// optimizer state values (adagrad: s0 = accumulator; ftrl: s0 = n, s1 = z).
__device__ inline void opt_step(const OptParams& o, float g, float& p, float& s0, float& s1) {
  if (o.type == kOptAdagrad) {
    // TF SparseApplyAdagrad: accum += g^2; var -= lr * g * rsqrt(accum)
    s0 += g * g;
    p -= o.lr * g * rsqrtf(s0);
  } else if (o.type == kOptFtrl) {
    // TF ApplyFtrl with lr_power = -0.5 (plus optional beta).
    const float n_new = s0 + g * g;
    const float sq_old = sqrtf(s0), sq_new = sqrtf(n_new);
    s1 += g - (sq_new - sq_old) / o.lr * p;
    s0 = n_new;
    const float quad = (o.beta + sq_new) / o.lr + 2.f * o.l2;
    p = fabsf(s1) > o.l1 ? (copysignf(o.l1, s1) - s1) / quad : 0.f;
  } else {
    p -= o.lr * g;
  }
}

// The same step for a table of dtype TV: fp8 tables on the hardware square root / reciprocal
// (FM_FP8_FAST_EPI, above).  Every writer of a table row (in-place backward, owner apply, dense
// apply) goes through this, so a row gets the same bits whichever path updates it.
template <typename TV>
__device__ inline void opt_step_tv(const OptParams& o, float g, float& p, float& s0, float& s1) {
  if constexpr (FM_FP8_FAST_EPI && StateBf16<TV>::v) {
    if (o.type == kOptFtrl) {
      const float ilr = __builtin_amdgcn_rcpf(o.lr);  // (wave-uniform: hoisted by the compiler)
      const float n_new = __builtin_fmaf(g, g, s0);
      const float sq_old = __builtin_amdgcn_sqrtf(s0), sq_new = __builtin_amdgcn_sqrtf(n_new);
      // (explicit fma / mul order: the rounding is fixed, not left to contraction, so every writer and
      // every lane width -- the wide fp8 chunk kernel -- produces the same bits)
      s1 += __builtin_fmaf(-((sq_new - sq_old) * ilr), p, g);
      s0 = n_new;
      const float quad = __builtin_fmaf(o.beta + sq_new, ilr, 2.f * o.l2);
      p = fabsf(s1) > o.l1 ? (copysignf(o.l1, s1) - s1) * __builtin_amdgcn_rcpf(quad) : 0.f;
      return;
    }
    if (o.type == kOptAdagrad) {
      s0 = __builtin_fmaf(g, g, s0);
      p = __builtin_fmaf(-(o.lr * g), __builtin_amdgcn_rsqf(s0), p);
      return;
    }
  }
  opt_step(o, g, p, s0, s1);
}

// A lane's N elements of one row: the optimizer switch taken once per row, not per element, so the
// elements' dependency chains interleave (the per-element form compiled to a scalar branch ladder per
// element).  Same per-element arithmetic as opt_step_tv: bitwise the same results.
template <typename TV, int N>
__device__ inline void opt_step_row(const OptParams& o, const float (&g)[N], float (&p)[N], float (&s0)[N],
                                    float (&s1)[N]) {
  if (o.type == kOptFtrl) {
    OptParams f = o;
    f.type = kOptFtrl;
#pragma unroll
    for (int k = 0; k < N; ++k) opt_step_tv<TV>(f, g[k], p[k], s0[k], s1[k]);
  } else if (o.type == kOptAdagrad) {
    OptParams f = o;
    f.type = kOptAdagrad;
#pragma unroll
    for (int k = 0; k < N; ++k) opt_step_tv<TV>(f, g[k], p[k], s0[k], s1[k]);
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) p[k] -= o.lr * g[k];
  }
}

// ---- host-side launch helpers ----------------------------------------------
inline int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }

inline int lanes_per_row(int Kp, int dtype) {
  const int epl = 4;  // fp32: 16 B, bf16: 8 B, fp8: 4 B per lane
  return next_pow2((Kp + epl - 1) / epl);
}

// Dynamic LDS bytes that let at most n workgroups (with `static_lds` bytes of their own) share a CU.
inline int lds_for_wg_per_cu(int n, int static_lds) {
  static const int cu_lds = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || v <= 0)
      v = 160 * 1024;
    return v;
  }();
  const int per = cu_lds / (n + 1) + 1024 - static_lds;  // n + 1 do not fit (margin: allocation granules)
  return per > 0 && (per + static_lds) * n <= cu_lds ? per : 0;
}

inline int fill_grid(long long work_groups, int groups_per_block, int cap = 8192) {
  long long blocks = (work_groups + groups_per_block - 1) / groups_per_block;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  return (int)blocks;
}

// SHM: dynamic LDS bytes per workgroup (0 for all but the occupancy-limited chunk kernel launch)
#define FM_DISPATCH_LPR(LPR_VAL, KERNEL, TV, GRID, SHM, STREAM, ARGS)                                   \
  switch (LPR_VAL) {                                                                                     \
    case 1: hipLaunchKernelGGL((KERNEL<1, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 2: hipLaunchKernelGGL((KERNEL<2, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 4: hipLaunchKernelGGL((KERNEL<4, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 8: hipLaunchKernelGGL((KERNEL<8, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 16: hipLaunchKernelGGL((KERNEL<16, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    case 32: hipLaunchKernelGGL((KERNEL<32, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    case 64: hipLaunchKernelGGL((KERNEL<64, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    default: return -1;                                                                                  \
  }

// rows of >= 4 lanes only (kernels without narrow-row instantiations)
#define FM_DISPATCH_WIDE_LPR(LPR_VAL, KERNEL, TV, GRID, SHM, STREAM, ARGS)                              \
  switch (LPR_VAL) {                                                                                     \
    case 4: hipLaunchKernelGGL((KERNEL<4, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 8: hipLaunchKernelGGL((KERNEL<8, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;     \
    case 16: hipLaunchKernelGGL((KERNEL<16, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    case 32: hipLaunchKernelGGL((KERNEL<32, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    case 64: hipLaunchKernelGGL((KERNEL<64, TV>), dim3(GRID), dim3(kBlock), SHM, STREAM, ARGS); break;   \
    default: return -1;                                                                                  \
  }

#define FM_DISPATCH_TV(DTYPE, M, LPR_VAL, KERNEL, GRID, SHM, STREAM, ARGS)   \
  if ((DTYPE) == kBF16) {                                                   \
    M(LPR_VAL, KERNEL, __hip_bfloat16, GRID, SHM, STREAM, ARGS)             \
  } else if ((DTYPE) == kFP8) {                                             \
    M(LPR_VAL, KERNEL, fp8e4m3, GRID, SHM, STREAM, ARGS)                    \
  } else {                                                                  \
    M(LPR_VAL, KERNEL, float, GRID, SHM, STREAM, ARGS)                      \
  }
#define FM_DISPATCH_WIDE(DTYPE, LPR_VAL, KERNEL, GRID, SHM, STREAM, ARGS) \
  FM_DISPATCH_TV(DTYPE, FM_DISPATCH_WIDE_LPR, LPR_VAL, KERNEL, GRID, SHM, STREAM, ARGS)
#define FM_DISPATCH_SHM(DTYPE, LPR_VAL, KERNEL, GRID, SHM, STREAM, ARGS) \
  FM_DISPATCH_TV(DTYPE, FM_DISPATCH_LPR, LPR_VAL, KERNEL, GRID, SHM, STREAM, ARGS)
#define FM_DISPATCH(DTYPE, LPR_VAL, KERNEL, GRID, STREAM, ARGS) \
  FM_DISPATCH_SHM(DTYPE, LPR_VAL, KERNEL, GRID, 0, STREAM, ARGS)

}  // namespace fm
