// rc_generic.hip -- batched fp32 GEMM for the generic (non-fused) REDCLIFF-S path.
//
// The published configuration (DGCNN embedder, one simulation step, weights applied after
// the simulation) runs the fused step kernels.  The other configurations the reference
// supports -- cEmbedder / Vanilla embedders (models/redcliff_factor_score_embedders.py:51-331),
// num_sims > 1 roll-outs and the per-step factor weighting mode
// (...withStateSmoothing.py:253-323) -- are composed on the host from this one contraction
// (cMLP layers, graph convolutions, Chebyshev powers, fc layers, the Vanilla convolutions
// as im2col products) with autograd supplying the backward products.
//
//   C[b] = alpha * op(A[b]) op(B[b]) + beta * C[b]      row-major, op(X) = X or X^T
//
// 64x64 output tile per 256-thread workgroup, 4x4 outputs per thread, K staged through LDS
// in steps of 16; each output is an in-order fmaf chain over k (deterministic).
#include "rc_common.h"

namespace {

#define GT 64
#define GK 16

__global__ __launch_bounds__(RC_BLOCK) void k_gemm(int ta, int tb, int M, int N, int K, float alpha,
                                                   const float* A, int64_t lda, int64_t sA, const float* B,
                                                   int64_t ldb, int64_t sB, float beta, float* C, int64_t ldc,
                                                   int64_t sC) {
  const int bz = blockIdx.z;
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;
  const int n0 = blockIdx.x * GT, m0 = blockIdx.y * GT;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  __shared__ float As[GK][GT + 4];  // As[k][m]
  __shared__ float Bs[GK][GT + 4];  // Bs[k][n]
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += GK) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + r * RC_BLOCK;  // 1024 elements of each 16x64 tile
      // A tile: element (k, m); lanes walk the contiguous index of the operand's storage
      int kk, mm;
      if (ta) { kk = e >> 6; mm = e & 63; } else { mm = e >> 4; kk = e & 15; }
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? (ta ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk]) : 0.f;
      int kb, nb;
      if (tb) { nb = e >> 4; kb = e & 15; } else { kb = e >> 6; nb = e & 63; }
      const int gn = n0 + nb, gk2 = k0 + kb;
      Bs[kb][nb] = (gn < N && gk2 < K) ? (tb ? B[(int64_t)gn * ldb + gk2] : B[(int64_t)gk2 * ldb + gn]) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + ty * 4 + i;
    if (gm >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gn = n0 + tx * 4 + j;
      if (gn >= N) continue;
      float* cp = C + (int64_t)gm * ldc + gn;
      *cp = beta == 0.f ? alpha * acc[i][j] : alpha * acc[i][j] + beta * *cp;
    }
  }
}

}  // namespace

extern "C" int redcliff_gemm(int32_t trans_a, int32_t trans_b, int32_t M, int32_t N, int32_t K, float alpha,
                             const float* A, int64_t lda, int64_t stride_a, const float* B, int64_t ldb,
                             int64_t stride_b, float beta, float* C, int64_t ldc, int64_t stride_c, int32_t batch,
                             void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 0 || !C || (K > 0 && (!A || !B))) {
    rc_set_error("gemm: bad arguments (M=%d N=%d K=%d batch=%d)", M, N, K, batch);
    return REDCLIFF_EINVAL;
  }
  if (M == 0 || N == 0 || batch == 0) return 0;
  if (batch > 65535) { rc_set_error("gemm: batch %d > 65535", batch); return REDCLIFF_ELIMIT; }
  dim3 grid((N + GT - 1) / GT, (M + GT - 1) / GT, batch);
  hipLaunchKernelGGL(k_gemm, grid, dim3(RC_BLOCK), 0, (hipStream_t)stream, trans_a, trans_b, M, N, K, alpha, A, lda,
                     stride_a, B, ldb, stride_b, beta, C, ldc, stride_c);
  return rc_check(hipGetLastError(), "k_gemm");
}
