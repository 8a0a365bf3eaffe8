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
// The kernel is the shared GEMM core of rc_gemm.h.
#include "rc_gemm.h"

extern "C" int redcliff_gemm(int32_t trans_a, int32_t trans_b, int32_t M, int32_t N, int32_t K, float alpha,
                             const float* A, int64_t lda, int64_t stride_a, const float* B, int64_t ldb,
                             int64_t stride_b, float beta, float* C, int64_t ldc, int64_t stride_c, int32_t batch,
                             void* stream) {
  if (M < 0 || N < 0 || K < 0 || batch < 0 || !C || (K > 0 && (!A || !B))) {
    rc_set_error("gemm: bad arguments (M=%d N=%d K=%d batch=%d)", M, N, K, batch);
    return REDCLIFF_EINVAL;
  }
  if (M == 0 || N == 0 || batch == 0) return 0;
  RcGemm g = rc_gemm_args(trans_a, trans_b, M, N, K, A, lda, stride_a, B, ldb, stride_b, C, ldc, stride_c);
  g.alpha = alpha;
  g.beta = beta;
  return rc_gemm_launch(g, batch, (hipStream_t)stream, "redcliff_gemm");
}
