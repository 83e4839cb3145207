#include "fm_common.h"
#include "../hash64.h"

namespace fm {

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

// fp8 rows: one thread per row (the row's scale needs its max |v| first, so
// the values are generated twice; init runs once).
__global__ __launch_bounds__(kBlock) void init_rows_fp8_kernel(InitArgs a) {
  for (long long r = (long long)blockIdx.x * kBlock + threadIdx.x; r < a.rows; r += (long long)gridDim.x * kBlock) {
    const long long gid = r * a.gid_mul + a.gid_add;
    float m = 0.f;
    for (int c = 0; c < a.K; ++c) m = fmaxf(m, fabsf(init_uniform(a.seed, gid, c + 1, a.range)));
    const float s = fp8_row_scale(m);
    int* dst = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(a.v) + r * a.v_stride);
    for (int c = 0; c < a.Kp; c += 4) {
      float q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        q[k] = c + k < a.K ? fminf(fmaxf(init_uniform(a.seed, gid, c + k + 1, a.range) / s, -kFp8Max), kFp8Max) : 0.f;
      int u = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
      dst[c / 4] = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], u, true);
    }
    a.w[r * a.w_stride] = init_uniform(a.seed, gid, 0, a.range);
    a.w[r * a.w_stride + 1] = s;
  }
}

// |v|^2 of fp8 rows (w_row[kFp8Norm], fm_common.h fp8_norm2) from their stored bytes and scales:
// one LPR-lane group per row, the same reduction as store_row's.  After init and after any write
// of rows / scales from the host side (checkpoint restore, Table.set_v).  ``idx`` (optional): the
// rows to refresh (``rows`` of them), else rows 0 .. rows - 1.
template <int LPR>
__global__ __launch_bounds__(kBlock) void fp8_norms_kernel(const uint8_t* v, long long v_stride, float* w,
                                                           long long w_stride, long long rows, int Kp,
                                                           const long long* idx) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1), t = lane % LPR;
  const bool tact = t < Kp / 4;
  const long long gid = ((long long)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + lane / LPR;
  const long long stride = (long long)gridDim.x * kWavesPerBlock * G;
  for (long long i = gid; i < rows; i += stride) {  // (uniform per group: the butterfly stays in it)
    const long long r = idx ? idx[i] : i;
    const int u = tact ? *reinterpret_cast<const int*>(v + r * v_stride + 4 * t) : 0;
    const float n2 = fp8_norm2<LPR>(u, w[r * w_stride + 1], tact);
    if (t == 0) w[r * w_stride + kFp8Norm] = n2;
  }
}

// v_stride in bytes (= elements of an fp8 table)
int launch_fp8_norms(const uint8_t* v, long long v_stride, float* w, long long w_stride, long long rows, int Kp,
                     hipStream_t st, const long long* idx) {
  if (rows <= 0) return 0;
  if (Kp % 4 != 0 || w_stride <= kFp8Norm) return -1;
  const int lpr = lanes_per_row(Kp, kFP8);
  const long long per_block = (long long)kWavesPerBlock * (kWave / lpr);
  long long blocks = (rows + per_block - 1) / per_block;
  if (blocks > 16384) blocks = 16384;
  switch (lpr) {
#define FM_NORMS(L) \
  case L: hipLaunchKernelGGL(fp8_norms_kernel<L>, dim3((int)blocks), dim3(kBlock), 0, st, v, v_stride, w, w_stride, rows, Kp, idx); break;
    FM_NORMS(1) FM_NORMS(2) FM_NORMS(4) FM_NORMS(8) FM_NORMS(16) FM_NORMS(32) FM_NORMS(64)
#undef FM_NORMS
    default: return -1;
  }
  return (int)hipGetLastError();
}

int launch_init_rows(const InitArgs& a, hipStream_t st) {
  if (a.rows <= 0) return 0;
  if (a.dtype == kFP8) {
    if (a.Kp % 4 != 0 || a.w_stride <= kFp8Norm) return -1;
    long long blocks = (a.rows + kBlock - 1) / kBlock;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(init_rows_fp8_kernel, dim3((int)blocks), dim3(kBlock), 0, st, a);
    if (hipGetLastError() != hipSuccess) return -2;
    return launch_fp8_norms(reinterpret_cast<const uint8_t*>(a.v), a.v_stride, a.w, a.w_stride, a.rows, a.Kp, st,
                            nullptr);
  }
  const long long total = a.rows * (long long)(a.Kp + 1);
  long long blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(init_rows_kernel, dim3((int)blocks), dim3(kBlock), 0, st, a);
  return (int)hipGetLastError();
}

}  // namespace fm

