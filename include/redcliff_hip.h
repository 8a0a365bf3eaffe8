/*
 * redcliff_hip.h -- C-ABI of libredcliff_hip.so, the MI355X (gfx950) implementation of the
 * REDCLIFF-S cMLP factor-model fitting hot path.
 *
 * The reference (carlson-lab/redcliff-s-hypothesizing-dynamic-causal-graphs) is pure
 * Python/PyTorch: it has no FFI of its own.  Each entry point below replaces one piece
 * of the reference's Python hot path (citations relative to the reference tree); the
 * Python host package binds them with ctypes.
 *
 * Conventions
 *  - All pointers are device pointers owned by the caller (PyTorch caching allocator).
 *    Nothing here allocates or frees device memory; scratch is a caller-supplied
 *    workspace of redcliff_workspace_bytes() bytes.
 *  - Every call is stream-ordered on the given hipStream_t (passed as void*) and does
 *    not synchronise the host.  Calls are stateless and re-entrant.
 *  - Return value: 0 on success, a negative argument-validation code, or a positive
 *    hipError_t.  redcliff_last_error() returns a thread-local message.
 *  - R "replicas" (independent fits with identical shapes, e.g. grid-search points)
 *    may be packed into one call; every per-replica buffer has an explicit stride.
 *  - fp32 throughout (the reference calls .float() on every model,
 *    general_utils/model_utils.py:392,417).
 */
#ifndef REDCLIFF_HIP_H
#define REDCLIFF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 8: the workspace region y is laid out network-major, y[nU][K][p][Bmax] (was y[nU][Bmax][K][p])
 * 9: redcliff_factor_forward writes finished predictions y_out[r][B][K][p] (callers no longer decode
 *    the kernel-private workspace); redcliff_factor_forward_workspace_floats sizes its workspace;
 *    redcliff_step_predictions reads a step's predictions back the same way; RedcliffAdamHyper.t_offset
 *    (was padding) offsets a replica's Adam step number from the launch's */
#define REDCLIFF_ABI_VERSION 9

/* error codes (negative) */
#define REDCLIFF_EINVAL (-1)  /* bad dimension / pointer                        */
#define REDCLIFF_ELIMIT (-2)  /* dimension outside what the kernels support     */
#define REDCLIFF_EWORKSPACE (-3)

/* step flags: which parts of one batch_update run (...withStateSmoothing.py:741-881) */
#define RC_BN_TRAIN      (1 << 0)  /* embedder BatchNorm in train mode (batch statistics)        */
#define RC_LOSS_FORECAST (1 << 1)  /* forecast MSE term (:629)                                   */
#define RC_LOSS_FACTOR   (1 << 2)  /* supervised factor-score MSE (:633-663)                     */
#define RC_LOSS_FWL1     (1 << 3)  /* factor-weight L1 (:666)                                    */
#define RC_LOSS_ADJ      (1 << 4)  /* lag-weighted adjacency L1 of conditional GC (:696-715)     */
#define RC_STEP_A        (1 << 5)  /* Adam step on the embedder (optimizerA)                     */
#define RC_STEP_B        (1 << 6)  /* Adam step on the factors  (optimizerB)                     */
#define RC_VALUES        (1 << 7)  /* compute loss values (validate_training, :1650-1790)        */
#define RC_CONFUSION     (1 << 8)  /* accumulate the factor-score confusion matrix (:786-803)    */
#define RC_STORE_OUTPUTS (1 << 9)  /* run the factor forward even without a loss (model.forward)  */
#define RC_REFRESH_SUPPORTS (1 << 10) /* recompute the DGCNN Chebyshev supports before the step  */
#define RC_GRAD_ONLY     (1 << 11) /* data-parallel shard: write the gradients of the RC_STEP_*
                                      groups to grad_emb / grad_fac instead of applying Adam
                                      (redcliff_adam_apply runs after the all-reduce)            */

/* Shapes shared by every call. */
typedef struct RedcliffDims {
  int32_t R;      /* replicas packed in one launch                                   */
  int32_t Bmax;   /* largest batch the workspace is sized for                         */
  int32_t T;      /* recorded time steps per window in the dataset buffer             */
  int32_t p;      /* channels (num_chans)                                            */
  int32_t L;      /* gen_lag: factor Conv1d kernel width                             */
  int32_t K;      /* num_factors                                                     */
  int32_t h;      /* factor hidden width (gen_hidden == [h])                          */
  int32_t F;      /* embed_lag == DGCNN num_features_per_node                        */
  int32_t n;      /* DGCNN Chebyshev layers                                          */
  int32_t H;      /* DGCNN hidden channels per node                                   */
  int32_t M1;     /* DGCNN fc1 width (64 in torcheeg)                                */
  int32_t nsup;   /* num_supervised_factors                                          */
  int32_t use_sigmoid;   /* use_sigmoid_restriction                                  */
  float sigmoid_ecc;     /* sigmoid_eccentricity_coeff                               */
} RedcliffDims;

/* torch.optim.Adam hyper-parameters of one parameter group.  Doubles are what torch's
 * Python side computes the bias corrections with; the fp32 copies are the scalars torch
 * applies element-wise (_single_tensor_adam / _multi_tensor_adam). */
typedef struct RedcliffAdamHyper {
  double lr, beta1, beta2;
  float eps, weight_decay;
  float beta2_f;            /* (float)beta2                                  */
  float one_minus_beta1_f;  /* (float)(1 - beta1): lerp weight               */
  float one_minus_beta2_f;  /* (float)(1 - beta2): addcmul value             */
  int32_t t_offset;         /* this replica's Adam step number minus the launch's tA / tB (packed
                               fits whose replicas stepped this group different numbers of times:
                               mixed phase schedules, ...withStateSmoothing.py:741-759); 0 otherwise */
} RedcliffAdamHyper;

/* Per-replica hyper-parameters, stored as a device array of R entries. */
typedef struct RedcliffReplicaHyper {
  float c_forecast, c_factor, c_cos, c_fwl1, c_smooth, c_adj; /* coeff_dict          */
  double bn_eps, bn_momentum;                                 /* BatchNorm1d         */
  RedcliffAdamHyper A;                                        /* optimizerA: embedder */
  RedcliffAdamHyper B;                                        /* optimizerB: factors  */
} RedcliffReplicaHyper;

/* Packed parameter layouts (floats, per replica):
 *  embedder (DGCNN): A[p][p] | gcW[n][F][H] | bn_w[F] | bn_b[F] | fc1W[M1][p*H] | fc1b[M1]
 *                    | fc2W[K][M1] | fc2b[K]
 *  factors:          W0[K][p][h][p][L] | b0[K][p][h] | W1[K][p][h] | b1[K][p]
 * (W0[k][j] is the Conv1d(p,h,L) weight of network j of factor k, models/cmlp.py:19.) */

typedef struct RedcliffStepArgs {
  RedcliffDims d;
  int32_t B;            /* windows in this batch (<= Bmax)                          */
  int32_t flags;        /* RC_* bitmask                                             */
  int32_t n_bn_updates; /* BatchNorm running-stat updates this step (3 in train phases) */
  int32_t tA, tB;       /* Adam step numbers (1-based) used for bias correction      */
  /* data: X[N][T][p] windows, labels[N][K] (already selected time index)            */
  const float* X; int64_t x_rstride; int64_t row0;
  const float* labels; int64_t lab_rstride;
  const double* bn_stats; int64_t bn_stats_rstride; /* [2][F] batch mean / biased var */
  /* parameters and Adam state                                                      */
  float* emb; float* emb_m; float* emb_v; int64_t emb_stride;
  float* fac; float* fac_m; float* fac_v; int64_t fac_stride;
  float* bn_rm; float* bn_rv;                      /* [R][F]                           */
  const RedcliffReplicaHyper* hyper;               /* device [R]                       */
  void* ws; size_t ws_bytes;                       /* workspace                        */
  double* acc;        /* [R][8] validation accumulators (may be NULL without RC_VALUES) */
  int32_t* confusion; /* [R][nsup][nsup] (may be NULL without RC_CONFUSION)              */
  /* data-parallel shards: this call processes B of the B_global windows of
   * the global batch.  Batch-mean terms (forecast MSE :629, factor MSE :638-661) and the
   * BatchNorm running-variance correction use B_global; batch sums (fw-L1, adj-L1) do not
   * scale, so the shard gradients of all ranks sum to the full-batch gradient.  bn_stats
   * must be the statistics of the GLOBAL batch.  B_global == 0 means B_global = B.       */
  int32_t B_global;
  int32_t pad_;
  float* grad_emb; float* grad_fac;  /* RC_GRAD_ONLY outputs, same layout/stride as emb / fac */
  /* Packed grid-search fits (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:125-160,
   * one fit per grid point): the replicas this call steps, a strictly increasing HOST array of
   * n_replicas indices < R (at most 256).  A replica that stopped early (the per-fit rule of
   * ...withStateSmoothing.py:1483-1559) is left out: its parameters, Adam state, BatchNorm
   * statistics and accumulators are not touched and its workgroups are not launched.
   * NULL = all R replicas.  n_replicas == 0 launches nothing. */
  const int32_t* replicas; int32_t n_replicas;
  int32_t pad2_;
} RedcliffStepArgs;

int redcliff_abi_version(void);
const char* redcliff_last_error(void);
/* Source hash this library was compiled from: the first 16 hex digits of the SHA-256 over
 * the .hip / .h files of csrc/ and the .h files of include/ (path-sorted, name + contents) and the compile defines
 * (redcliff_amd/build.py source_hash).  Ties a pushed binary to the committed sources. */
const char* redcliff_build_id(void);

/* Workspace bytes for one launch of R replicas (all kernels share one layout). */
size_t redcliff_workspace_bytes(const RedcliffDims* d);
size_t redcliff_emb_param_count(const RedcliffDims* d);
size_t redcliff_fac_param_count(const RedcliffDims* d);

/* BatchNorm batch statistics of the embedder window X[row][Lmax-F:Lmax] for n_batches
 * consecutive batches of size B (last one may be ragged; N total windows).
 * stats[r][batch][2][F] (mean, biased variance).  Replaces the statistics half of
 * torch.nn.BatchNorm1d.forward in train mode (torcheeg DGCNN.BN1, models/dgcnn.py:37). */
int redcliff_bn_batch_stats(const RedcliffDims* d, const float* X, int64_t x_rstride, int64_t N, int32_t B,
                            double* stats, int64_t stats_rstride, void* stream);

/* normalize_A + Chebyshev supports [I, L, L^2, ...] of the DGCNN adjacency into the
 * workspace (torcheeg normalize_A / generate_cheby_adj).  Must run after any change
 * of the embedder parameters made outside redcliff_train_step. */
int redcliff_dgcnn_supports(const RedcliffDims* d, const float* emb, int64_t emb_stride, void* ws, void* stream);

/* One REDCLIFF-S batch_update (...withStateSmoothing.py:734-933) for the published
 * configuration: DGCNN embedder, conditional_factor_fixed_embedder GC, factor weights
 * applied after simulation, num_sims == 1.  With RC_VALUES and no RC_STEP_* it is the
 * per-batch body of validate_training.  Launches the fused kernel chain on `stream`. */
int redcliff_train_step(const RedcliffStepArgs* a, void* stream);

/* nsteps consecutive batch_updates of one epoch without returning to the host:
 * step i uses rows[i] / sizes[i] (host arrays) as row0 / B, bn_stats advanced by
 * i*bn_stats_step doubles, and Adam step numbers a->tA + i (a->tB + i) when the
 * corresponding RC_STEP_* flag is set.  RC_REFRESH_SUPPORTS applies to the first step. */
int redcliff_train_steps(const RedcliffStepArgs* a, int32_t nsteps, const int64_t* rows, const int32_t* sizes,
                         int32_t bn_stats_step, void* stream);

/* Offsets (floats, per replica) of the workspace regions: T R f1 w a y G G0 w1 dwp dAadj dWi dS
 * dgb S dZ amat lossp xsim gfc total.  Returns the number of offsets available.  The host reads
 * w (raw embedder output, [B][K]), xsim (mixed forecast, [B][p]) and G / G0 (group norms) back
 * from a step run with RC_STORE_OUTPUTS; the per-factor predictions through
 * redcliff_step_predictions (the y region itself is kernel-private partial sums). */
int redcliff_workspace_layout(const RedcliffDims* d, int64_t* out, int32_t n_out);

/* Per-factor predictions of the last RC_STORE_OUTPUTS step of the R replicas of workspace ws (sized
 * for d): y_out[r][b][k][j] (y_rstride floats between replicas), b < B.  The models' per-factor
 * outputs of forward (...withStateSmoothing.py:326-385). */
int redcliff_step_predictions(const RedcliffDims* d, int32_t B, const void* ws, float* y_out, int64_t y_rstride,
                              void* stream);

/* Device status of the R replica slices of a workspace (no reference counterpart: the
 * reference has no device code).  out[r] (host array of R u32) receives replica r's count of
 * merged-backward hand-off waits that ran out of polls since the last call (the consumer then
 * proceeded without its producers' records, so that step's results are invalid); the words are
 * cleared.  Synchronises `stream`.  Returns the number of replicas with a non-zero count (0 =
 * healthy) or a negative error code.  Callers check it where they already synchronise. */
int redcliff_device_status(const RedcliffDims* d, void* ws, uint32_t* out, void* stream);

/* Verification mode (tests only; no reference counterpart): with floats > 0 every workspace
 * region laid out afterwards is followed by a guard band of that many floats, the last band
 * also closing replica R-1's slice.  A test fills the bands with a NaN pattern; a write past
 * a region's end changes a band, a read past it puts NaN into the results.  0 = production
 * layout.  Returns the previous setting.  Process-wide: set it before sizing workspaces. */
int redcliff_debug_guard_bands(int32_t floats);
/* (start, size) pairs, in floats, of the regions of one replica's workspace slice in layout
 * order (out[2i], out[2i+1]); returns the region count. */
int redcliff_workspace_regions(const RedcliffDims* d, int64_t* out, int32_t n_pairs);

/* Stand-alone forward of K cMLPs (models/cmlp.py:90-101, MLP.forward :29-35) on B windows
 * Xwin[r][B][L][p] (x_rstride floats between the R = d->R replicas): y_out[r][b][k][j]
 * (y_rstride floats between replicas) receives the prediction of network j of factor k for
 * window b.  ws: scratch of redcliff_factor_forward_workspace_floats(d, B) floats per replica
 * (ws_rstride floats between replicas; its contents are private to the kernels). */
size_t redcliff_factor_forward_workspace_floats(const RedcliffDims* d, int32_t B);
int redcliff_factor_forward(const RedcliffDims* d, int32_t B, const float* Xwin, int64_t x_rstride, const float* fac,
                            int64_t fac_stride, float* ws, int64_t ws_rstride, float* y_out, int64_t y_rstride,
                            void* stream);

/* G[r][k][j][c][t] = ||W0[k][j][:, c, t]||_2, G0[r][k][j][c] = ||W0[k][j][:, c, :]||_F (models/cmlp.py:147-167) */
int redcliff_gc_norms(const RedcliffDims* d, const float* fac, int64_t fac_stride, float* G, float* G0, void* stream);
/* In-place proximal step on layer-0 weights, penalty 0=GL 1=GSGL 2=H (models/cmlp.py:117-144). */
int redcliff_prox(const RedcliffDims* d, float* fac, int64_t fac_stride, float lam, float lr, int32_t penalty,
                  void* stream);

/* Adam (torch.optim.Adam, coupled L2, general_utils/model_utils.py:747-762) of one
 * parameter group from a gradient buffer: group 0 = embedder (hyper[r].A), 1 = factors
 * (hyper[r].B); n floats per replica at `stride`; t = 1-based step number.  The
 * data-parallel step is  train_step(RC_GRAD_ONLY) -> all-reduce(grad) -> adam_apply. */
int redcliff_adam_apply(const RedcliffDims* d, float* params, float* exp_avg, float* exp_avg_sq, const float* grad,
                        int64_t n, int64_t stride, const RedcliffReplicaHyper* hyper, int32_t group, int32_t t,
                        void* stream);

/* The data-parallel update in one launch: with the step arguments of the RC_GRAD_ONLY shard step
 * that just ran (after grad_emb / grad_fac were all-reduced), Adam of the RC_STEP_A group
 * (n_emb floats) and the RC_STEP_B group (n_fac floats), exactly as redcliff_adam_apply with
 * t = tA / tB, plus the DGCNN Chebyshev supports of the updated A in the workspace, so the next
 * step needs no RC_REFRESH_SUPPORTS.  Replaces the optimizer steps of batch_update
 * (models/redcliff_s_cmlp_withStateSmoothing.py:741-759) for summed gradients. */
int redcliff_dp_update(const RedcliffStepArgs* a, int64_t n_emb, int64_t n_fac, void* stream);

/* Batched fp32 GEMM, row-major: C[b] = alpha * op(A[b]) op(B[b]) + beta * C[b], op = X or X^T
 * (trans flag), A/B/C of batch b at X + b * stride_x.  The contraction of the generic
 * (non-fused) path: cEmbedder / Vanilla embedders (models/redcliff_factor_score_embedders.py:
 * 51-331), num_sims > 1 roll-outs and the per-step weighting forward mode
 * (models/redcliff_s_cmlp_withStateSmoothing.py:253-323), composed on the host with autograd. */
int redcliff_gemm(int32_t trans_a, int32_t trans_b, int32_t M, int32_t N, int32_t K, float alpha, const float* A,
                  int64_t lda, int64_t stride_a, const float* B, int64_t ldb, int64_t stride_b, float beta, float* C,
                  int64_t ldc, int64_t stride_c, int32_t batch, void* stream);

/* Per-epoch GC-progress metrics of fit() for S samples x G graphs (replaces the host loops of
 * general_utils/model_utils.py:18-160 over general_utils/metrics.py:111-252, 396-430 and
 * sklearn's roc_auc_score).  One workgroup per (sample, graph), 2 <= p <= 64, Lt <= 128:
 *   est      float32 [S][nE][p][p][Lt]  GC estimates (the first G of each sample are scored)
 *   truth    float64 [2][G][p][p]       true graphs summed over lags and max-normalised,
 *                                       [0] as is, [1] with self-connections removed first
 *   eps_pow  float64 [p]                eps_pow[k] = deltaConEps ** k (host pow)
 *   out      float64 [S][G][6 + p]      f1, roc_auc, f1 (off-diagonal), roc_auc (off-diagonal),
 *                                       deltacon0, deltacon0 with directed degrees, deltaffinity,
 *                                       path-length MSE for k = 1 .. p-1
 * roc_auc is NaN where sklearn would raise (truth without negatives, NaN scores). */
int redcliff_gc_progress(int32_t S, int32_t nE, int32_t G, int32_t p, int32_t Lt, const float* est,
                         const double* truth, const double* eps_pow, double in_degree_coeff, double out_degree_coeff,
                         double* out, void* stream);
/* The same with one truth block per group of spt consecutive samples: sample s is scored against
 * truth[s / spt] ([S / spt][2][G][p][p]) -- a packed grid whose replicas fit different data sets
 * (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:66-72: one model over many
 * datasets, each with its own true graphs).  redcliff_gc_progress is spt = S. */
int redcliff_gc_progress_grouped(int32_t S, int32_t spt, int32_t nE, int32_t G, int32_t p, int32_t Lt,
                                 const float* est, const double* truth, const double* eps_pow, double in_degree_coeff,
                                 double out_degree_coeff, double* out, void* stream);

/* Per-epoch tracker statistics of fit() (replaces the host reductions of
 * general_utils/model_utils.py:163-188 (L1 tracker) and :191-209 (cosine tracker), which the
 * reference runs on float64 copies of every estimate):
 *   est      float32 [n_l1_rows][l1_len]     lagged estimates, one (sample, factor) per row
 *   l1_out   float64 [n_l1_rows]             sum |e / max(e)|
 *   nolag    float32 [n_samples][K][row_len] lag-free estimates
 *   dots_out float64 [n_samples][K][K]       upper triangle (i1 <= i2): sum (a / max a)(b / max b)
 *                                            over rows i1, i2 (the diagonal: squared norms)
 * One workgroup per row / pair, reductions in a fixed order independent of the launch size. */
int redcliff_gc_track_stats(int32_t n_l1_rows, int64_t l1_len, const float* est, double* l1_out, int32_t n_samples,
                            int32_t K, int64_t row_len, const float* nolag, double* dots_out, void* stream);

/* Per-kernel HIP-event timing for benchmarking: redcliff_kernel_timing(1) brackets every
 * kernel launched by redcliff_train_step with events on its stream; redcliff_kernel_times()
 * synchronises them and returns per-kernel totals (ids 0..7: supports, emb_fwd, fac_fwd,
 * fac_bwd, emb_bwd, emb_final, fac_mix, emb_combine, fac_lead).  Returns the number of kernel ids.
 * When a single fit (R == 1) splits into two kernel chains (GEMM-shaped embedder and / or
 * matrix-core factor path), the factor chain runs on an internal second stream (one per host
 * thread and device) forked from and joined back into `stream` with events, so stream
 * ordering for the caller is unchanged.  Packed replicas run on `stream` only. */
int redcliff_kernel_timing(int32_t enable);
int redcliff_kernel_times(double* total_ms, int64_t* counts, int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* REDCLIFF_HIP_H */
