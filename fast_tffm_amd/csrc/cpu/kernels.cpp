#include "kernels.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include <omp.h>

#include "../hash64.h"

namespace fm {
namespace cpu {

namespace {

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return static_cast<uint16_t>((u >> 16) | 0x40u);
  return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

inline void load_row(const void* v, long long off, int Kp, int dtype, float* dst) {
  if (dtype == 1) {
    const uint16_t* p = static_cast<const uint16_t*>(v) + off;
    for (int k = 0; k < Kp; ++k) dst[k] = bf16_to_f32(p[k]);
  } else {
    std::memcpy(dst, static_cast<const float*>(v) + off, sizeof(float) * Kp);
  }
}

inline void store_row(void* v, long long off, int Kp, int dtype, const float* src) {
  if (dtype == 1) {
    uint16_t* p = static_cast<uint16_t*>(v) + off;
    for (int k = 0; k < Kp; ++k) p[k] = f32_to_bf16(src[k]);
  } else {
    std::memcpy(static_cast<float*>(v) + off, src, sizeof(float) * Kp);
  }
}

inline void opt_step(const OptParams& o, float g, float& p, float& s0, float& s1) {
  if (o.type == 0) {
    s0 += g * g;
    p -= o.lr * g / std::sqrt(s0);
  } else if (o.type == 1) {
    const float n_new = s0 + g * g;
    const float sq_old = std::sqrt(s0), sq_new = std::sqrt(n_new);
    s1 += g - (sq_new - sq_old) / o.lr * p;
    s0 = n_new;
    const float quad = (o.beta + sq_new) / o.lr + 2.f * o.l2;
    p = std::fabs(s1) > o.l1 ? (std::copysign(o.l1, s1) - s1) / quad : 0.f;
  } else {
    p -= o.lr * g;
  }
}

inline void set_threads(int threads) {
  if (threads > 0) omp_set_num_threads(threads);
}

void update_row(const OptParams& opt, long long row, const float* g, float gw, int Kp, void* v, long long v_stride,
                float* w, long long w_stride, float* s0v, float* s1v, long long s_stride, float* s0w, float* s1w,
                int dtype, float* scratch) {
  load_row(v, row * v_stride, Kp, dtype, scratch);
  float* a0 = s0v + row * s_stride;
  float* a1 = s1v ? s1v + row * s_stride : nullptr;
  for (int k = 0; k < Kp; ++k) {
    float z = a1 ? a1[k] : 0.f;
    opt_step(opt, g[k], scratch[k], a0[k], z);
    if (a1) a1[k] = z;
  }
  store_row(v, row * v_stride, Kp, dtype, scratch);
  float& pw = w[row * w_stride];
  float z = s1w ? s1w[row] : 0.f;
  opt_step(opt, gw, pw, s0w[row], z);
  if (s1w) s1w[row] = z;
}

}  // namespace

FwdResult fwd(int B, const int* offsets, const int* rows, const float* vals, const void* v, long long v_stride,
              const float* w, long long w_stride, int Kp, int dtype, const float* labels, const float* weights,
              int loss_type, float grad_scale, float* pred, float* r1, float* dpred, int threads,
              const float* bias) {
  set_threads(threads);
  double loss_sum = 0, regv_sum = 0, regw_sum = 0;
#pragma omp parallel reduction(+ : loss_sum, regv_sum, regw_sum)
  {
    std::vector<float> s1(Kp), s2(Kp), row(Kp);
#pragma omp for schedule(static)
    for (int i = 0; i < B; ++i) {
      std::fill(s1.begin(), s1.end(), 0.f);
      std::fill(s2.begin(), s2.end(), 0.f);
      float lin = 0.f, rv = 0.f, rw = 0.f;
      for (int j = offsets[i]; j < offsets[i + 1]; ++j) {
        const long long r = rows[j];
        const float x = vals ? vals[j] : 1.f;
        load_row(v, r * v_stride, Kp, dtype, row.data());
        const float wv = w[r * w_stride];
        for (int k = 0; k < Kp; ++k) {
          const float xv = x * row[k];
          s1[k] += xv;
          s2[k] += xv * xv;
          rv += row[k] * row[k];
        }
        lin += x * wv;
        rw += wv * wv;
      }
      float part = 0.f;
      for (int k = 0; k < Kp; ++k) part += s1[k] * s1[k] - s2[k];
      const float p = lin + 0.5f * part + (bias ? bias[0] : 0.f);
      pred[i] = p;
      if (r1) std::memcpy(r1 + (long long)i * Kp, s1.data(), sizeof(float) * Kp);
      regv_sum += rv;
      regw_sum += rw;
      if (loss_type != 0) {
        const float y = labels[i];
        const float wt = weights ? weights[i] : 1.f;
        float l, d;
        if (loss_type == 1) {
          const float diff = p - y;
          l = wt * diff * diff;
          d = 2.f * wt * diff;
        } else {
          l = wt * (std::max(p, 0.f) - p * y + std::log1p(std::exp(-std::fabs(p))));
          d = wt * (1.f / (1.f + std::exp(-p)) - y);
        }
        loss_sum += l;
        if (dpred) dpred[i] = d * grad_scale;
      }
    }
  }
  return FwdResult{loss_sum, regv_sum, regw_sum};
}

int dedup(int n, const uint32_t* keys, uint32_t* skeys, int* perm, uint32_t* uniq, int* seg_start, int* inv,
          const int* ex_of_occ, int* sorted_ex, const float* vals, float* sorted_x) {
  if (n <= 0) {
    seg_start[0] = 0;
    return 0;
  }
  std::vector<uint64_t> kv(n);
  for (int j = 0; j < n; ++j) kv[j] = (static_cast<uint64_t>(keys[j]) << 32) | static_cast<uint32_t>(j);
  std::sort(kv.begin(), kv.end());  // (key, index) order == stable sort by key
  int U = 0;
  for (int j = 0; j < n; ++j) {
    const uint32_t key = static_cast<uint32_t>(kv[j] >> 32);
    const int p = static_cast<int>(kv[j] & 0xffffffffu);
    skeys[j] = key;
    perm[j] = p;
    if (j == 0 || key != skeys[j - 1]) {
      uniq[U] = key;
      seg_start[U] = j;
      ++U;
    }
    if (inv) inv[p] = U - 1;
    if (sorted_ex) sorted_ex[j] = ex_of_occ[p];
    if (sorted_x) sorted_x[j] = vals[p];
  }
  seg_start[U] = n;
  return U;
}

void bwd(int mode, int U, const int* seg_start, const int* uniq, const int* sorted_ex, const float* sorted_x,
         const float* dpred, const float* r1, int Kp, void* v, long long v_stride, float* w, long long w_stride,
         float* s0v, float* s1v, long long s_stride, float* s0w, float* s1w, float reg_v, float reg_w,
         OptParams opt, float* grad_out, long long g_stride, int dtype, int threads) {
  set_threads(threads);
#pragma omp parallel
  {
    std::vector<float> A(Kp), vv(Kp), g(Kp), scratch(Kp);
#pragma omp for schedule(dynamic, 256)
    for (int u = 0; u < U; ++u) {
      std::fill(A.begin(), A.end(), 0.f);
      float Scx = 0.f, Sc = 0.f;
      const int sa = seg_start[u], sb = seg_start[u + 1];
      for (int j = sa; j < sb; ++j) {
        const int ex = sorted_ex[j];
        const float x = sorted_x ? sorted_x[j] : 1.f;
        const float c = dpred[ex] * x;
        const float* rr = r1 + (long long)ex * Kp;
        for (int k = 0; k < Kp; ++k) A[k] += c * rr[k];
        Scx += c * x;
        Sc += c;
      }
      const long long row = mode == 0 ? (long long)uniq[u] : (long long)u;
      load_row(v, row * v_stride, Kp, mode == 0 ? dtype : 0, vv.data());
      const float wv = w[row * w_stride];
      const float n_u = static_cast<float>(sb - sa);
      for (int k = 0; k < Kp; ++k) g[k] = A[k] - Scx * vv[k] + reg_v * n_u * vv[k];
      const float gw = Sc + reg_w * n_u * wv;
      if (mode == 1) {
        float* dst = grad_out + (long long)u * g_stride;
        std::memcpy(dst, g.data(), sizeof(float) * Kp);
        dst[Kp] = gw;
      } else {
        update_row(opt, row, g.data(), gw, Kp, v, v_stride, w, w_stride, s0v, s1v, s_stride, s0w, s1w, dtype,
                   scratch.data());
      }
    }
  }
}

void gather_rows(int R, const int* req, const void* v, long long v_stride, const float* w, long long w_stride,
                 int Kp, int dtype, float* out, long long o_stride, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(static)
  for (int p = 0; p < R; ++p) {
    const long long row = req[p];
    float* dst = out + (long long)p * o_stride;
    load_row(v, row * v_stride, Kp, dtype, dst);
    dst[Kp] = w[row * w_stride];
    for (long long k = Kp + 1; k < o_stride; ++k) dst[k] = 0.f;
  }
}

void apply_rows(int U, const int* seg_start, const int* uniq, const int* perm, const float* grad_in,
                long long g_stride, int Kp, void* v, long long v_stride, float* w, long long w_stride, float* s0v,
                float* s1v, long long s_stride, float* s0w, float* s1w, OptParams opt, int dtype, int threads) {
  set_threads(threads);
#pragma omp parallel
  {
    std::vector<float> g(Kp), scratch(Kp);
#pragma omp for schedule(dynamic, 256)
    for (int u = 0; u < U; ++u) {
      std::fill(g.begin(), g.end(), 0.f);
      float gw = 0.f;
      for (int j = seg_start[u]; j < seg_start[u + 1]; ++j) {
        const float* src = grad_in + (long long)perm[j] * g_stride;
        for (int k = 0; k < Kp; ++k) g[k] += src[k];
        gw += src[Kp];
      }
      update_row(opt, uniq[u], g.data(), gw, Kp, v, v_stride, w, w_stride, s0v, s1v, s_stride, s0w, s1w, dtype,
                 scratch.data());
    }
  }
}

void csr_rows(int B, const int* offsets, int* ex_of_occ) {
  for (int i = 0; i < B; ++i)
    for (int j = offsets[i]; j < offsets[i + 1]; ++j) ex_of_occ[j] = i;
}

namespace {
inline float init_uniform(unsigned long long seed, long long gid, int col, float range) {
  const unsigned long long h =
      mix64(seed ^ mix64(static_cast<unsigned long long>(gid) * 0x100000001b3ull + static_cast<unsigned long long>(col)));
  const float u = static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
  return range * (2.f * u - 1.f);
}
}  // namespace

void init_rows(void* v, long long v_stride, float* w, long long w_stride, long long rows, int K, int Kp, int dtype,
               long long gid_mul, long long gid_add, unsigned long long seed, float range, int threads) {
  set_threads(threads);
#pragma omp parallel for schedule(static)
  for (long long r = 0; r < rows; ++r) {
    const long long gid = r * gid_mul + gid_add;
    for (int c = 0; c < Kp; ++c) {
      const float val = c < K ? init_uniform(seed, gid, c + 1, range) : 0.f;
      if (dtype == 1)
        static_cast<uint16_t*>(v)[r * v_stride + c] = f32_to_bf16(val);
      else
        static_cast<float*>(v)[r * v_stride + c] = val;
    }
    w[r * w_stride] = init_uniform(seed, gid, 0, range);
  }
}

}  // namespace cpu
}  // namespace fm
