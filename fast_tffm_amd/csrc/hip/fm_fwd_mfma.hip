// fp8 FM forward on the CDNA4 matrix cores (BASELINE config 5: k = 128 fp8 table, binary features).
//
// Parity: reference FeatureRankGenerator / BiasGenerator / FmScorer (cc/fm_scorer_op.h:8-44, 46-94,
// 101-140) fused with the loss ops (tffm/fm_model.py:311-333), like fm_fwd.hip's VALU kernel.
//
// Formulation.  A tile is 16 consecutive examples and their R rows (contiguous in CSR order).  The
// factor sums of the tile are one matrix product
//     S1[16 x 128] = X[16 x R] . Q[R x 128]
// where Q holds the rows' raw e4m3 bytes and X is block-diagonal: X[m][r] = x_r s_r if row r belongs
// to example m (s_r: the row's power-of-two scale), else 0.  With binary features x_r s_r is a power
// of two, exact in e5m2 after one exponent offset per tile (2^c, undone in fp32 at the end), so the
// product runs on v_mfma_f32_16x16x32_bf8_fp8 (A = e5m2 X, B = e4m3 Q, fp32 accumulation) with the
// rows' bytes as they are stored.  The block-diagonal zeros cost 15/16 of the matrix work, which at
// the fp8 rate is a few microseconds per batch; what it removes is the VALU kernel's per-element
// conversion and FMA work (the k128 fp8 forward ran at 60% VALU busy, profiles/r4).  s2 / reg come
// from the stored row norms, lin from the rows' w (one 16-byte tail per row), as in the VALU kernel.
//
// Per wave (no cross-wave sharing; one __shared__ array, per-wave regions):
//  1. the tile's row indices -> LDS (global_load_lds, 4 B per lane), then the rows' [w, scale, |v|^2,
//     pad] tails -> LDS (16 B per lane, per-lane source addresses);
//  2. per row, lane-parallel: its example (a search over the tile's 17 CSR offsets), lin / s2n
//     accumulated per example in LDS, the scale exponent; the tile's largest exponent sets 2^c; the
//     A byte of every row (e5m2 2^(e + c)) and its example byte go to LDS;
//  3. K-steps of 32 rows: the rows' 128 bytes stream into a 3-slot LDS ring by global_load_lds (4
//     wave-instructions per step, per-lane source = row base + 16-byte chunk, chunks XOR-swizzled by
//     row so the transposed reads are conflict-free) two steps ahead, each step retired by a counted
//     vmcnt; B fragments come out of the ring with ds_read_b64_tr_b8 (8 rows x 1 column per lane),
//     A fragments from the example / A bytes by a byte-SIMD select; 8 MFMAs (one per 16 columns);
//  4. epilogue: S1 scaled by 2^-c, sum of squares per example (16-lane butterflies), r1 (bf16)
//     transposed through LDS into coalesced 16-byte stores, pred / loss / dpred by 16 lanes.
// Host conditions (launch_fwd): fp8 rows, Kp = 128, no per-occurrence values, table rows (w_stride 4,
// no self rows / segment lookup), 16 * max_feats <= kMfMaxRows.
// (Included by fm_fwd.hip inside namespace fm.)

typedef float mf_v4f __attribute__((ext_vector_type(4)));
typedef int mf_i32x2 __attribute__((__vector_size__(2 * sizeof(int))));

constexpr int kMfT = 16;                 // examples per tile (MFMA M)
constexpr int kMfKS = 32;                // rows per K-step (MFMA K)
constexpr int kMfRing = 3;               // K-step slots per wave (two steps in flight)
constexpr int kMfRowB = 128;             // bytes per fp8 row (Kp = 128)
constexpr int kMfSlot = kMfKS * kMfRowB; // 4096
constexpr int kMfMaxRows = 768;          // rows per tile (16 examples x 48 features)
// per-wave LDS: ring (aliased by the tails during the row pass) | idx | example bytes | A bytes | sums
constexpr int kMfOffIdx = kMfRing * kMfSlot;          // 12288
constexpr int kMfOffEx = kMfOffIdx + 4 * kMfMaxRows;  // 15360
constexpr int kMfOffXs = kMfOffEx + kMfMaxRows;       // 16128
constexpr int kMfOffSum = kMfOffXs + kMfMaxRows;      // 16896: lin[16] s2n[16] sq[16] (floats)
constexpr int kMfWaveB = kMfOffSum + 64 * 4;          // 17152
static_assert(kMfMaxRows * 16 <= kMfOffIdx, "row tails alias the ring");
static_assert(kMfMaxRows % 64 == 0, "row passes cover whole 64-row groups");

typedef __attribute__((address_space(3))) uint8_t lds_u8;

// FM_MF_PROF=1 (build variant "mfprof"): per-phase shader-clock totals of the kernel's waves
// (tile start -> indices -> tails -> row pass -> K-loop -> epilogue; [5] = tiles), read and
// cleared by the module's mf_prof()
#ifndef FM_MF_PROF
#define FM_MF_PROF 0
#endif
#if FM_MF_PROF
__device__ unsigned long long g_mf_prof[8];
#define MF_T(i)                                                                         \
  do {                                                                                  \
    const long long t_ = clock64();                                                     \
    if (lane == 0) atomicAdd(&g_mf_prof[i], (unsigned long long)(t_ - t_last));        \
    t_last = t_;                                                                        \
  } while (0)
#else
#define MF_T(i) \
  do {          \
  } while (0)
#endif

// global_load_lds in inline asm (LDS destination: M0 = the wave-uniform LDS byte address, + 16 B x lane):
// the compiler does not track these, so it inserts no vmcnt waits of its own for the LDS they write (with
// the builtin it drains vmcnt to 0 before every LDS read of the same array, which serialises the ring);
// every read of DMA-written LDS below is ordered by an explicit, counted s_waitcnt instead.
__device__ inline void mf_glds16(const void* src, uint32_t lds) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}
__device__ inline void mf_glds4(const void* src, uint32_t lds) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}

// s_waitcnt vmcnt(n) for the ring (n = 4 x steps left in flight: 0, 4 or 8)
__device__ inline void mf_wait_vm(int n) {
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// chunk position of 16-byte chunk c of tile row q inside the ring slot (XOR swizzle: the 16 rows a
// 32-lane half reads transposed land in 16 distinct 16-byte bank groups)
__device__ inline int mf_chunk_pos(int q, int c) { return c ^ ((q >> 1) & 7); }

__global__ __launch_bounds__(kBlock) void fm_fwd_mfma_fp8_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kWavesPerBlock * kMfWaveB];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  const uint32_t W = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((lds_u8*)smem) + wv * kMfWaveB);
  int* idx_l = reinterpret_cast<int*>(smem + wv * kMfWaveB + kMfOffIdx);
  uint8_t* ex_l = smem + wv * kMfWaveB + kMfOffEx;
  uint8_t* xs_l = smem + wv * kMfWaveB + kMfOffXs;
  float* sum_l = reinterpret_cast<float*>(smem + wv * kMfWaveB + kMfOffSum);  // lin | s2n | sq
  const float4* tail_l = reinterpret_cast<const float4*>(smem + wv * kMfWaveB);  // (row pass: ring bytes)
  const uint8_t* ring = smem + wv * kMfWaveB;
  const int g = lane >> 4, li = lane & 15;
  const bool want_reg = a.reg_partial != nullptr;
  float loss_acc = 0.f, regv_acc = 0.f, regw_acc = 0.f;
  const int ntile = (a.B + kMfT - 1) / kMfT;
  for (int tile = blockIdx.x * kWavesPerBlock + wv; tile < ntile; tile += gridDim.x * kWavesPerBlock) {
#if FM_MF_PROF
    long long t_last = clock64();
    if (lane == 0) atomicAdd(&g_mf_prof[5], 1ull);
#endif
    const int e0 = tile * kMfT;
    const int ne = min(kMfT, a.B - e0);
    // tile-relative CSR offsets of its examples: lane m <= ne holds offsets[e0 + m] (lanes past ne: the end)
    const int ob = a.offsets[e0 + min(lane, ne)];
    const int R0 = __shfl(ob, 0), R1 = __shfl(ob, ne);
    const int R = R1 - R0;
    const int o_rel = ob - R0;
    if (R > kMfMaxRows) {  // (max_feats understated by the caller: NaN scores and loss, no LDS overrun)
      if (lane < ne) {
        a.pred[e0 + lane] = __builtin_nanf("");
        if (a.dpred) a.dpred[e0 + lane] = __builtin_nanf("");
        loss_acc = __builtin_nanf("");
      }
      continue;
    }
    // label / weight of example li (lanes < ne), used after the K-loop
    float y = 0.f, wt = 1.f;
    if (lane < ne && a.loss_type != kLossNone) {
      y = a.labels[e0 + lane];
      if (a.weights) wt = a.weights[e0 + lane];
    }
    if (lane < 3 * kMfT) sum_l[lane] = 0.f;
    const int nI = (R + kWave - 1) / kWave;  // 64-row groups of the row pass
    // 1. row indices, then the rows' tails, into LDS
    for (int p = 0; p < nI; ++p) mf_glds4(a.rows + R0 + min(p * kWave + lane, R - 1), W + kMfOffIdx + p * 256);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    MF_T(0);
    for (int p = 0; p < nI; ++p) {
      const int id = idx_l[min(p * kWave + lane, R - 1)];
      mf_glds16(a.w + (uint64_t)(uint32_t)id * 4u, W + p * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    MF_T(1);
    // 2. per row: example, lin / s2n sums, scale exponent
    int maxE = 0;
    for (int p = 0; p < nI; ++p) {
      const int r = p * kWave + lane;
      const bool valid = r < R;
      const float4 t4 = tail_l[r];
      int m = 0;  // largest m < ne with o_rel[m] <= r (binary search over lanes 0..15)
#pragma unroll
      for (int step = 8; step > 0; step >>= 1) {
        const int c = m + step;
        if (__shfl(o_rel, c < ne ? c : 0) <= r && c < ne) m = c;
      }
      const uint32_t sb = __float_as_uint(t4.y);
      const int E = (int)((sb >> 23) & 0xffu);
      const bool live = valid && t4.z > 0.f;  // (all-zero rows: A byte 0, no say in the exponent)
      if (valid) {
        atomicAdd(&sum_l[m], t4.x);
        atomicAdd(&sum_l[kMfT + m], t4.z);
        if (want_reg) { regw_acc += t4.x * t4.x; regv_acc += t4.z; }
      }
      if (live) maxE = max(maxE, E);
      ex_l[r] = valid ? (uint8_t)m : (uint8_t)0xff;
      xs_l[r] = live ? (uint8_t)E : (uint8_t)0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxE = max(maxE, __shfl_xor(maxE, o));
    // A bytes: e5m2 2^(E - maxE + 14) (biased exponent E - maxE + 29); two subnormal steps below,
    // then 0 (a row 2^-30 below the tile's largest scale: dropped)
    for (int p = 0; p < nI; ++p) {
      const int r = p * kWave + lane;
      const int E = xs_l[r];
      const int be = E - maxE + 29;
      xs_l[r] = E == 0 ? 0 : be >= 1 ? (uint8_t)(be << 2) : be == 0 ? 2 : be == -1 ? 1 : 0;
    }
    MF_T(2);
    // 3. K-steps
    const int S = (R + kMfKS - 1) / kMfKS;
    mf_v4f acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = mf_v4f{0.f, 0.f, 0.f, 0.f};
    auto issue = [&](int s) {
      const uint32_t slot = W + (s % kMfRing) * kMfSlot;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 8 * i + (lane >> 3);
        const int id = idx_l[min(s * kMfKS + q, R - 1)];
        const int c = mf_chunk_pos(q, lane & 7);
        mf_glds16(reinterpret_cast<const char*>(a.v) + (uint64_t)(uint32_t)id * (uint32_t)a.v_stride + 16 * c,
                  slot + i * 1024);
      }
    };
    if (S > 0) issue(0);
    if (S > 1) issue(1);
    const uint64_t mrep = 0x0101010101010101ull * (uint64_t)li;
    const int q_rd = 8 * g + (li >> 1);                     // this lane's row of the transposed reads
    const int rd_off = q_rd * kMfRowB + 8 * (li & 1);
    const int sw = (q_rd >> 1) & 7;
    for (int s = 0; s < S; ++s) {
      if (s + 2 < S) issue(s + 2);
      mf_wait_vm(4 * min(2, S - 1 - s));
      const uint8_t* slot = ring + (s % kMfRing) * kMfSlot;
      // A: rows 32 s + 8 g .. + 7 of example li: the A byte where the row's example byte == li
      const uint64_t exb = *reinterpret_cast<const uint64_t*>(ex_l + s * kMfKS + 8 * g);
      const uint64_t xsb = *reinterpret_cast<const uint64_t*>(xs_l + s * kMfKS + 8 * g);
      const uint64_t x = exb ^ mrep;
      const uint64_t y = (x | 0x8080808080808080ull) - 0x0101010101010101ull;
      const uint64_t z = ~y & 0x8080808080808080ull;
      const long afrag = (long)(xsb & ((z >> 7) * 0xffull));
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const lds_u8* p = (const lds_u8*)(slot + rd_off + 16 * (t ^ sw));
        const mf_i32x2 b = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) mf_i32x2*)p);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(afrag, __builtin_bit_cast(long, b), acc[t], 0, 0, 0);
      }
    }
    MF_T(3);
    // 4. epilogue: lane (g, li) holds S1[4 g + i][16 t + li] * 2^c
    const float unscale = __uint_as_float((uint32_t)max(1, maxE - 14) << 23);  // 2^(maxE - 141)
    float sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[t][i] *= unscale;
        sq[i] += acc[t][i] * acc[t][i];
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) sq[i] = group_sum<16>(sq[i]);
    if (li == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sum_l[2 * kMfT + 4 * g + i] = sq[i];
    }
    if (a.r1 != nullptr) {  // r1 rows (bf16) through the ring slot 0 image: [16][128] bf16, then 16-byte stores
      uint16_t* t16 = reinterpret_cast<uint16_t*>(smem + wv * kMfWaveB);
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) t16[(4 * g + i) * 128 + 16 * t + li] = (uint16_t)f32_to_bf16_bits(acc[t][i]);
      const int e = lane >> 2, part = lane & 3;
      if (e < ne) {
        const uint4* src = reinterpret_cast<const uint4*>(t16 + e * 128 + part * 32);
        uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.r1) + (long long)(e0 + e) * a.Kp + part * 32);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = src[k];
      }
    }
    if (lane < ne) {
      const float pred = sum_l[lane] + 0.5f * (sum_l[2 * kMfT + lane] - sum_l[kMfT + lane]) + (a.bias ? a.bias[0] : 0.f);
      a.pred[e0 + lane] = pred;
      if (a.loss_type != kLossNone) {
        float l, d;
        if (a.loss_type == kLossMse) {
          const float diff = pred - y;
          l = wt * diff * diff;
          d = 2.f * wt * diff;
        } else {
          l = wt * (fmaxf(pred, 0.f) - pred * y + softplus_neg_abs(pred));
          d = wt * (sigmoidf(pred) - y);
        }
        loss_acc += l;
        if (a.dpred) a.dpred[e0 + lane] = d * a.grad_scale;
      }
    }
    MF_T(4);
  }
  if (a.loss_partial == nullptr && a.reg_partial == nullptr) return;
  loss_acc = group_sum<kWave>(loss_acc);
  regv_acc = group_sum<kWave>(regv_acc);
  regw_acc = group_sum<kWave>(regw_acc);
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

