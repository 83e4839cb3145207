// Host (CPU) implementations of the FM step kernels. They follow the same
// contracts as the gfx950 kernels in csrc/hip/ (same argument meaning, same
// row layouts) and back the world_size=1 CPU configuration and the gloo
// multi-process tests. They mirror the reference's CPU Eigen path
// (cc/fm_scorer_op.cc:79, cc/fm_grad_op.cc:88), but group occurrences per
// row instead of the CAS-loop float atomics of cc/fm_grad_op.h:4-15.
#pragma once
#include <cstdint>

namespace fm {
namespace cpu {

struct OptParams {
  int type;  // 0 adagrad, 1 ftrl, 2 sgd
  float lr, l1, l2, beta;
};

struct FwdResult {
  double loss_sum, regv_sum, regw_sum;
};

FwdResult fwd(int B, const int* offsets, const int* rows, const float* vals, const void* v, long long v_stride,
              const float* w, long long w_stride, int Kp, int dtype, const float* labels, const float* weights,
              int loss_type, float grad_scale, float* pred, float* r1, float* dpred, int threads,
              const float* bias = nullptr);

// Stable sort of (key, occurrence) + run-length encoding. Returns U.
int dedup(int n, const uint32_t* keys, uint32_t* skeys, int* perm, uint32_t* uniq, int* seg_start, int* inv,
          const int* ex_of_occ, int* sorted_ex, const float* vals, float* sorted_x);

void bwd(int mode, int U, const int* seg_start, const int* uniq, const int* sorted_ex, const float* sorted_x,
         const float* dpred, const float* r1, int Kp, void* v, long long v_stride, float* w, long long w_stride,
         float* s0v, float* s1v, long long s_stride, float* s0w, float* s1w, float reg_v, float reg_w,
         OptParams opt, float* grad_out, long long g_stride, int dtype, int threads);

void gather_rows(int R, const int* req, const void* v, long long v_stride, const float* w, long long w_stride,
                 int Kp, int dtype, float* out, long long o_stride, int threads);

void apply_rows(int U, const int* seg_start, const int* uniq, const int* perm, const float* grad_in,
                long long g_stride, int Kp, void* v, long long v_stride, float* w, long long w_stride, float* s0v,
                float* s1v, long long s_stride, float* s0w, float* s1w, OptParams opt, int dtype, int threads);

void csr_rows(int B, const int* offsets, int* ex_of_occ);

// Counter-based U(-range, range) init, identical to the gfx950 init_rows kernel.
void init_rows(void* v, long long v_stride, float* w, long long w_stride, long long rows, int K, int Kp, int dtype,
               long long gid_mul, long long gid_add, unsigned long long seed, float range, int threads);

}  // namespace cpu
}  // namespace fm
