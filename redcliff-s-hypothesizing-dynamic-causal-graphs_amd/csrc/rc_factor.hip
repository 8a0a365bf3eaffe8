// rc_factor.hip -- the K factors x p channel networks of REDCLIFF-S as one grouped,
// batched contraction on gfx950.
//
// Reference: models/cmlp.py:12-35 (MLP: Conv1d(p, h, L) -> ReLU -> Conv1d(h, 1, 1)),
// models/cmlp.py:90-101 (cMLP.forward), models/cmlp.py:147-167 (GC group norms),
// models/redcliff_s_cmlp_withStateSmoothing.py:326-385 (x_sim = sum_k w_k * pred_k),
// :629 (forecast MSE) and :696-715 (lag-weighted adjacency L1 of the conditional GC
// estimate w_bk * G_k[..., -min(L,F):] + A^T).
//
// With num_sims == 1 every network sees one window of L steps, so network (k, j) is the
// GEMM  Z[b][u] = sum_q Xw[b][q] W0[k][j][u][q]  (q = c*L + t, B x pL x h).  One workgroup
// owns one network for the whole batch: its weights, their Adam state and the whole
// gradient reduction over the batch stay inside the workgroup (no atomics, fixed order).
#include <cstring>

#include "rc_common.h"
#include "rc_fac_bwd.h"

namespace {

__global__ __launch_bounds__(RC_BLOCK) void k_fac_bwd(StepCtx c, int nUl, int nQ, int role) {
  // nUl x nQ workgroups per network (1 x 1 when there is no factor update or only the records)
  extern __shared__ float sm[];
  // (one workgroup per network -- the split-lead step's records launch -- needs no division)
  const int per = nUl * nQ;
  const int kj = per == 1 ? (int)blockIdx.x : (int)blockIdx.x / per;
  const int rem0 = blockIdx.x - kj * per;
  const int uc = nQ == 1 ? rem0 : rem0 / nQ, qc = rem0 - uc * nQ;
  fac_bwd_wg(c, nUl, nQ, kj, uc, qc, rc_rep(c, blockIdx.y), sm, nullptr, role);
}

// Finished predictions of the stand-alone forward: out[r][b][k][j] = sum over the nU hidden-chunk
// partials y[u][k][j][b] (u ascending from 0, the order every consumer in the training step uses;
// the output bias sits in chunk 0), one thread per output, windows fastest in the reads.
// bstride: the window stride of the slots (B for the stand-alone forward, Bmax in a step workspace)
__global__ __launch_bounds__(256) void k_fac_pred(const float* __restrict__ ws, int64_t wss, int64_t yoff, int B,
                                                  int bstride, int kp, int nU, float* __restrict__ out,
                                                  int64_t out_rs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)kp * B) return;
  const int kj = (int)(i / B), b = (int)(i - (int64_t)kj * B);
  const float* y = ws + (int64_t)blockIdx.y * wss + yoff;
  float s = y[(int64_t)kj * bstride + b];
  for (int u = 1; u < nU; ++u) s += y[((int64_t)u * kp + kj) * bstride + b];
  out[(int64_t)blockIdx.y * out_rs + (int64_t)b * kp + kj] = s;
}

}  // namespace

// The vector factor backward stages per-window terms of the whole batch in LDS; past the
// 64 KiB budget (large K * Bmax) the matrix-core path, which tiles the windows, takes over.
bool rc_fac_vector_fits(const RedcliffDims& d) {
  return (size_t)fac_bwd_lds_floats(d) <= (size_t)RC_LDS_LIMIT_FLOATS;
}

int rc_fac_bwd_grid(const StepCtx& c) {
  const RedcliffDims& d = c.d;
  if (!(c.flags & RC_STEP_B)) return d.K * d.p;
  return d.K * d.p * rc_nuchunk(d) * ((d.p * d.L + FB_QT - 1) / FB_QT);
}

// role: RC_FB_ALL (one launch), or the split-lead pair RC_FB_RECORDS (K*p lead workgroups: dL/dw,
// dL/dA, group norms, x_sim, loss values) + RC_FB_UPDATE (every workgroup's dW0 / bias / Adam part),
// which depend only on the forward and so run concurrently (rc_capi.hip redcliff_train_step)
int rc_launch_fac_bwd(const StepCtx& c, hipStream_t s, int role, hipEvent_t stop) {
  const RedcliffDims& d = c.d;
  const int Q = d.p * d.L;
  const bool upd = (c.flags & RC_STEP_B) && role != RC_FB_RECORDS;
  if (role == RC_FB_UPDATE && !(c.flags & RC_STEP_B)) { rc_set_error("factor update launch without a factor step"); return REDCLIFF_EINVAL; }
  const int nQ = upd ? (Q + FB_QT - 1) / FB_QT : 1;
  const size_t lds = sizeof(float) * (size_t)fac_bwd_lds_floats(d);
  if (lds > RC_LDS_LIMIT_FLOATS * sizeof(float)) {
    // only reached when the matrix-core path cannot take over (h > 128) or is overridden
    // (REDCLIFF_FAC_PATH=vector): name the batch limit instead of a bare launch failure
    RedcliffDims e = d;
    while (e.Bmax > 1 && (size_t)fac_bwd_lds_floats(e) > (size_t)RC_LDS_LIMIT_FLOATS) --e.Bmax;
    const char* why = d.h > 128 ? "the matrix-core factor path supports h <= 128" : "REDCLIFF_FAC_PATH=vector is set";
    rc_set_error("vector factor backward: batches of %d windows with K=%d, h=%d need %zu KiB of LDS (64 KiB budget): "
                 "use batches of at most %d windows (%s)", d.Bmax, d.K, d.h, lds / 1024, e.Bmax, why);
    return REDCLIFF_ELIMIT;
  }
  // without a factor update only the lead workgroup of each network has work
  const int nUl = upd ? rc_nuchunk(d) : 1;
  if (stop)
    hipExtLaunchKernelGGL(k_fac_bwd, dim3(d.K * d.p * nUl * nQ, c.nrep), dim3(RC_BLOCK), lds, s, nullptr, stop, 0, c, nUl,
                          nQ, role);
  else
    hipLaunchKernelGGL(k_fac_bwd, dim3(d.K * d.p * nUl * nQ, c.nrep), dim3(RC_BLOCK), lds, s, c, nUl, nQ, role);
  return rc_check(hipGetLastError(), "k_fac_bwd");
}

// Stand-alone forward of K cMLPs on B windows Xwin[B][L][p] (cMLP.forward, models/cmlp.py:90-101,
// and the per-factor predictions of REDCLIFF forward).  Per replica the (kernel-private) workspace
// holds a[K][p][B][h] | y[nU][K][p][B] (partials over hidden chunks, network-major: rc_y_idx with
// Bmax = B) | G[K][p][p][L] | G0[K][p][p] | w1[K][p][h] | gq[nU][K][p][p*L]; k_fac_pred then writes
// the finished predictions y_out[r][B][K][p].
static int64_t fac_fwd_ws_floats(const RedcliffDims& d, int B) {
  const int64_t kp = (int64_t)d.K * d.p, nU = rc_nuchunk(d);
  return kp * B * d.h + nU * B * kp + kp * d.p * d.L + kp * d.p + kp * d.h + nU * kp * d.p * d.L;
}

extern "C" size_t redcliff_factor_forward_workspace_floats(const RedcliffDims* d, int32_t B) {
  if (!d || B < 1 || d->K < 1 || d->p < 1 || d->h < 1 || d->L < 1) return 0;
  return (size_t)fac_fwd_ws_floats(*d, B);
}

extern "C" int redcliff_factor_forward(const RedcliffDims* d, int32_t B, const float* Xwin, int64_t x_rstride,
                                       const float* fac, int64_t fac_stride, float* ws, int64_t ws_rstride,
                                       float* y_out, int64_t y_rstride, void* stream) {
  if (!d || !Xwin || !fac || !ws || !y_out || B < 1 || d->R < 1) {
    rc_set_error("factor_forward: bad arguments");
    return REDCLIFF_EINVAL;
  }
  if (d->p > 64 || d->h > 128 || d->L > 64) { rc_set_error("factor_forward: dims outside kernel limits"); return REDCLIFF_ELIMIT; }
  if (d->R > 1 && (ws_rstride < fac_fwd_ws_floats(*d, B) || y_rstride < (int64_t)B * d->K * d->p)) {
    rc_set_error("factor_forward: replica strides smaller than one replica's workspace / predictions");
    return REDCLIFF_EINVAL;
  }
  StepCtx c;
  memset(&c, 0, sizeof(c));
  c.nrep = d->R;
  c.rident = 1;
  c.d = *d;
  c.d.Bmax = B;
  c.d.T = d->L;
  c.B = B;
  c.Bg = B;
  c.Lmax = d->L;
  c.Ls = d->L;
  c.X = Xwin;
  c.xr = x_rstride;
  c.fac = const_cast<float*>(fac);
  c.fs = fac_stride;
  c.ws = ws;
  c.wss = ws_rstride;
  c.fo = rc_fac_off(*d);
  const int64_t kp = (int64_t)d->K * d->p;
  c.wo.a = 0;
  c.wo.y = kp * B * d->h;
  c.wo.G = c.wo.y + (int64_t)rc_nuchunk(*d) * B * kp;
  c.wo.G0 = c.wo.G + kp * d->p * d->L;
  c.wo.w1 = c.wo.G0 + kp * d->p;
  c.wo.gq = c.wo.w1 + kp * d->h;
  rc_ctx_magics(c);
  int rc = rc_launch_fac_fwd(c, (hipStream_t)stream);
  if (rc) return rc;
  const int64_t n = kp * B;
  hipLaunchKernelGGL(k_fac_pred, dim3((unsigned)((n + 255) / 256), d->R), dim3(256), 0, (hipStream_t)stream, ws,
                     ws_rstride, c.wo.y, B, B, (int)kp, rc_nuchunk(*d), y_out, y_rstride);
  return rc_check(hipGetLastError(), "k_fac_pred");
}

// Per-factor predictions of the last RC_STORE_OUTPUTS step (redcliff_train_step) from its workspace
// (R replica slices): y_out[r][b][k][j] for the step's B windows.
extern "C" int redcliff_step_predictions(const RedcliffDims* d, int32_t B, const void* ws, float* y_out,
                                         int64_t y_rstride, void* stream) {
  if (!d || !ws || !y_out || B < 1 || B > d->Bmax || d->R < 1) {
    rc_set_error("step_predictions: bad arguments");
    return REDCLIFF_EINVAL;
  }
  const WsOff o = rc_ws_off(*d);
  const int64_t kp = (int64_t)d->K * d->p, n = kp * B;
  if (d->R > 1 && y_rstride < n) { rc_set_error("step_predictions: y_rstride < B*K*p"); return REDCLIFF_EINVAL; }
  hipLaunchKernelGGL(k_fac_pred, dim3((unsigned)((n + 255) / 256), d->R), dim3(256), 0, (hipStream_t)stream,
                     (const float*)ws, o.total, o.y, B, d->Bmax, (int)kp, rc_nuchunk(*d), y_out, y_rstride);
  return rc_check(hipGetLastError(), "k_fac_pred");
}
