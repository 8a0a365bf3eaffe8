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

namespace {

#define FK_BT 128   // batch rows per forward tile (16 row-groups x 8)
#define FK_QT 32    // contraction tile
#define FB_BT 32    // batch rows per backward tile
#define FB_QT 64    // dW0 columns per backward tile

__device__ inline float xwin(const StepCtx& c, const RcDiv& dL, const float* X, int b, int q) {
  const int L = c.d.L;
  const int ch = dL.div(q), t = q - ch * L;
  return X[((c.row0 + b) * c.d.T + (c.Lmax - L + t)) * c.d.p + ch];
}

// ------------------------------------------------------------------------------------------
// K2a: forward of every (factor, channel) network, FAC_UC hidden units per workgroup.
// grid (K*p*nU, R).  Writes relu activations a[kj][b][u], the partial output
// ypart[uc][b][k][j] = sum_{u in chunk} W1[u] a[b][u] (+ b1 in chunk 0), the chunk's
// squared layer-0 group norms gq[uc][kj][q] and a snapshot of W1 for the backward.
__global__ __launch_bounds__(RC_BLOCK) void k_fac_fwd(StepCtx c) {
  const RedcliffDims& d = c.d;
  const int nU = rc_nuchunk(d);
  const int r = blockIdx.y, kj = blockIdx.x / nU, uc = blockIdx.x - kj * nU;
  const int p = d.p, h = d.h, K = d.K;
  const int k = kj / p, j = kj - k * p;
  const int Q = p * d.L;
  const int u0 = uc * FAC_UC;
  const float* P = c.fac + r * c.fs;
  const float* W0 = P + c.fo.W0 + (int64_t)kj * h * Q;
  const float* b0 = P + c.fo.b0 + (int64_t)kj * h;
  const float* W1 = P + c.fo.W1 + (int64_t)kj * h;
  const float b1 = uc == 0 ? P[c.fo.b1 + kj] : 0.f;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const int tid = threadIdx.x, tb = tid >> 4, tu = tid & 15;
  const int u = u0 + tu;
  const RcDiv dL(d.L);

  __shared__ float Xs[FK_BT * (FK_QT + 1)];
  __shared__ float Ws[FAC_UC * (FK_QT + 1)];

  for (int bc = 0; bc < c.B; bc += FK_BT) {
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int q0 = 0; q0 < Q; q0 += FK_QT) {
      rc_stage<8>(FK_BT * FK_QT, [&](int e) {
        const int bb = e / FK_QT, qq = e - bb * FK_QT;
        const int b = bc + bb, q = q0 + qq;
        return (b < c.B && q < Q) ? xwin(c, dL, X, b, q) : 0.f;
      }, [&](int e, float v) { Xs[(e / FK_QT) * (FK_QT + 1) + e % FK_QT] = v; });
      rc_stage<2>(FAC_UC * FK_QT, [&](int e) {
        const int uu = e / FK_QT, qq = e - uu * FK_QT;
        const int q = q0 + qq;
        return (u0 + uu < h && q < Q) ? W0[(int64_t)(u0 + uu) * Q + q] : 0.f;
      }, [&](int e, float v) { Ws[(e / FK_QT) * (FK_QT + 1) + e % FK_QT] = v; });
      __syncthreads();
      if (bc == 0 && tid < FK_QT && q0 + tid < Q) {
        // squared group norms of the chunk's 16 units (GC, models/cmlp.py:162-166), pre-update
        float sq = 0.f;
        for (int uu = 0; uu < FAC_UC; ++uu) {
          const float w = Ws[uu * (FK_QT + 1) + tid];
          sq += w * w;
        }
        ws[c.wo.gq + ((int64_t)uc * K * p + kj) * Q + q0 + tid] = sq;
      }
#pragma unroll 8
      for (int qq = 0; qq < FK_QT; ++qq) {
        const float wv = Ws[tu * (FK_QT + 1) + qq];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += Xs[(tb + 16 * i) * (FK_QT + 1) + qq] * wv;
      }
      __syncthreads();
    }
    const float bu = u < h ? b0[u] : 0.f, w1 = u < h ? W1[u] : 0.f;
    if (bc == 0 && tb == 0 && u < h) ws[c.wo.w1 + (int64_t)kj * h + u] = w1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int b = bc + tb + 16 * i;
      float ys = 0.f;
      if (u < h) {
        const float a = fmaxf(acc[i] + bu, 0.f);
        if (b < c.B) ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u] = a;
        ys = w1 * a;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) ys += __shfl_xor(ys, o, 64);
      if (tu == 0 && b < c.B) ws[c.wo.y + (((int64_t)uc * d.Bmax + b) * K + k) * p + j] = ys + b1;
    }
  }
}

// ------------------------------------------------------------------------------------------
// K2b: mixing, forecast loss, adjacency L1, backward and Adam.  grid (K*p*nU*nQ, R):
// workgroup (network kj, hidden chunk uc, dW0 column tile qc).  The cheap per-window work
// (x_sim, residual, dL/dy, adjacency-L1 signs) is recomputed by every workgroup of a network;
// its outputs (dL/dw partials, loss values, dL/dA) are written by the (uc, qc) = (0, 0) one.
__global__ __launch_bounds__(RC_BLOCK) void k_fac_bwd(StepCtx c, int nUl, int nQ) {
  // nUl x nQ workgroups per network (1 x 1 when there is no factor update)
  const RedcliffDims& d = c.d;
  const int nU = rc_nuchunk(d);
  const int r = blockIdx.y;
  const int kj = blockIdx.x / (nUl * nQ);
  const int rem0 = blockIdx.x - kj * nUl * nQ;
  const int uc = rem0 / nQ, qc = rem0 - uc * nQ;
  const bool lead = (uc == 0 && qc == 0);
  const int p = d.p, h = d.h, K = d.K, L = d.L;
  const int k = kj / p, j = kj - k * p;
  const int Q = p * L;
  const int u0 = uc * FAC_UC, q0 = qc * FB_QT;
  float* P = c.fac + r * c.fs;
  float* PM = c.facM + r * c.fs;
  float* PV = c.facV + r * c.fs;
  float* GF = c.gF + r * c.fs;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int tid = threadIdx.x;
  const int B = c.B;
  const RcDiv dL(d.L), dK(K);
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const bool fgrad = (c.flags & RC_STEP_B) || (c.flags & RC_STEP_A);
  const bool adj_grad = fgrad && (c.flags & RC_LOSS_ADJ);
  const bool values = c.flags & RC_VALUES;

  extern __shared__ float sm[];
  float* dyl = sm;             // [Bmax]
  float* wk = dyl + d.Bmax;    // [Bmax]  w_bk (post-sigmoid)
  float* Gs = wk + d.Bmax;     // [Q]
  float* dGs = Gs + Q;         // [Q]
  float* Acol = dGs + Q;       // [p]
  float* lwt = Acol + p;       // [L]
  float* red = lwt + L;        // [16]
  float* dAp = red + 16;       // [p*Ls]
  float* ybuf = dAp + p * c.Ls;  // [Bmax][K]
  float* tiles = ybuf + d.Bmax * d.K;

  // ---- part 1: mixture x_sim = sum_k w_k y_k, forecast residual, dL/dy and dL/dw (forecast)
  const float gscale = (c.flags & RC_LOSS_FORECAST) ? hy.c_forecast * (2.f / (float)c.Bg) : 0.f;
  // ybuf[b][k'] = sum over hidden chunks of the per-factor predictions (fixed order)
  rc_stage<2>(B * K, [&](int e) {
    const int b = dK.div(e), kk = e - b * K;
    const float* yp = ws + c.wo.y + ((int64_t)b * K + kk) * p + j;
    const int64_t qs = (int64_t)d.Bmax * K * p;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = q < nU ? yp[q * qs] : 0.f;
    float yv = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < nU) yv += v[q];
    return yv;
  }, [&](int e, float v) { ybuf[e] = v; });
  __syncthreads();
  float fsum = 0.f;
  for (int b = tid; b < B; b += RC_BLOCK) {
    const float* wr = ws + c.wo.w + (int64_t)b * K;
    const float xt = (c.flags & (RC_LOSS_FORECAST | RC_VALUES)) ? X[((c.row0 + b) * d.T + c.Lmax) * p + j] : 0.f;
    float xs = 0.f;
    for (int kk = 0; kk < K; ++kk) {
      const float yv = ybuf[b * K + kk];
      const float we = sig ? rc_sigmoid(ecc * wr[kk]) : wr[kk];
      xs = (kk == 0) ? we * yv : xs + we * yv;
    }
    const float yk = ybuf[b * K + k];
    // the target X[:, Lmax] exists only when a loss is requested (forward() passes X[:, :Lmax])
    const float res = (c.flags & (RC_LOSS_FORECAST | RC_VALUES)) ? xs - xt : 0.f;
    const float wb = sig ? rc_sigmoid(ecc * wr[k]) : wr[k];
    const float g = gscale * res;
    wk[b] = wb;
    dyl[b] = g * wb;
    if (lead && fgrad) ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k] = g * yk;
    if (lead && k == 0) {
      fsum += res * res;
      ws[c.wo.xsim + (int64_t)b * p + j] = xs;
    }
  }
  if (values && lead && k == 0) {
    const float t = rc_block_sum(fsum, red);
    if (tid == 0) ws[c.wo.lossp + j] = t;
  }

  // ---- group norms G[kj][c][t] = sqrt(sum over hidden chunks), G0[kj][c] (cmlp.py:147-167)
  const bool adj_on = adj_grad || (values && lead);
  const int Ls = c.Ls;
  if (adj_on || lead) {
    for (int e = tid; e < Q; e += RC_BLOCK) {
      float sq = 0.f;
      for (int q = 0; q < nU; ++q) sq += ws[c.wo.gq + ((int64_t)q * K * p + kj) * Q + e];
      dGs[e] = sq;
      const float g = sqrtf(sq);
      Gs[e] = g;
      if (lead) ws[c.wo.G + (int64_t)kj * Q + e] = g;
    }
    __syncthreads();
    if (lead)
      for (int cc = tid; cc < p; cc += RC_BLOCK) {
        float sq = 0.f;
        for (int t = 0; t < L; ++t) sq += dGs[cc * L + t];
        ws[c.wo.G0 + (int64_t)kj * p + cc] = sqrtf(sq);
      }
    __syncthreads();
  }
  // ---- part 2: adjacency L1 of the conditional GC estimate  w_bk G_k[j][c][t] + A[c][j]
  if (adj_on) {
    for (int e = tid; e < Q; e += RC_BLOCK) dGs[e] = 0.f;
    for (int cc = tid; cc < p; cc += RC_BLOCK) Acol[cc] = E[c.eo.A + cc * p + j];
    for (int i = tid; i < Ls; i += RC_BLOCK) lwt[i] = logf((float)(i + 2));
    __syncthreads();
    if (lead) {
      float vsum = 0.f;
      for (int b = tid; b < B; b += RC_BLOCK) {
        const float wb = wk[b];
        float t = 0.f, v = 0.f;
        for (int cc = 0; cc < p; ++cc)
          for (int i = 0; i < Ls; ++i) {
            const float g = Gs[cc * L + (L - Ls + i)];
            const float val = wb * g + Acol[cc];
            t += lwt[i] * rc_sign(val) * g;
            v += lwt[i] * fabsf(val);
          }
        if (adj_grad) ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k] += hy.c_adj * t;
        vsum += v;
      }
      if (values) {
        const float t = rc_block_sum(vsum, red);
        if (tid == 0) ws[c.wo.lossp + p + kj] = hy.c_adj * t;
      }
    }
    if (adj_grad) {
      for (int e = tid; e < p * Ls; e += RC_BLOCK) {
        const int cc = e / Ls, i = e - cc * Ls;
        const int q = cc * L + (L - Ls + i);
        const float g = Gs[q];
        float sw = 0.f, s1 = 0.f;
        for (int b = 0; b < B; ++b) {
          const float sg = rc_sign(wk[b] * g + Acol[cc]);
          sw += sg * wk[b];
          s1 += sg;
        }
        dGs[q] = hy.c_adj * lwt[i] * sw;
        dAp[e] = hy.c_adj * lwt[i] * s1;
      }
      __syncthreads();
      if (lead && (c.flags & RC_STEP_A)) {
        for (int cc = tid; cc < p; cc += RC_BLOCK) {
          float s = 0.f;
          for (int i = 0; i < Ls; ++i) s += dAp[cc * Ls + i];
          ws[c.wo.dAadj + ((int64_t)k * p + cc) * p + j] = s;  // d/dA[c][j]
        }
      }
    }
  }
  if (!(c.flags & RC_STEP_B)) return;
  __syncthreads();

  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  const float* aw = ws + c.wo.a + (int64_t)kj * d.Bmax * h;
  const float* W1 = ws + c.wo.w1 + (int64_t)kj * h;  // pre-update snapshot written by K2a
  // ---- part 3a (column tile 0): output-layer / bias gradients of the chunk's hidden units
  if (qc == 0) {
    const int uu = tid & 15, part = tid >> 4;  // 16 slices of the batch per hidden unit
    const int u = u0 + uu;
    float dW1u = 0.f, db0u = 0.f;
    if (u < h) {
      const float w1 = W1[u];
      for (int b = part; b < B; b += 16) {
        const float av = aw[(int64_t)b * h + u];
        dW1u += dyl[b] * av;
        db0u += av > 0.f ? dyl[b] * w1 : 0.f;
      }
    }
    float* rA = tiles;              // [16][16]
    float* rB = tiles + 256;
    rA[tid] = dW1u;
    rB[tid] = db0u;
    float db1 = 0.f;
    if (uc == 0)
      for (int b = tid; b < B; b += RC_BLOCK) db1 += dyl[b];
    db1 = rc_block_sum(db1, red);
    if (tid < 16 && u0 + tid < h) {
      float g1 = 0.f, g0 = 0.f;
      for (int s = 0; s < 16; ++s) {
        g1 += rA[s * 16 + tid];
        g0 += rB[s * 16 + tid];
      }
      const int64_t ib = c.fo.b0 + (int64_t)kj * h + u0 + tid;
      const int64_t iw = c.fo.W1 + (int64_t)kj * h + u0 + tid;
      rc_update(c, P, PM, PV, GF, ib, g0, as);
      rc_update(c, P, PM, PV, GF, iw, g1, as);
    }
    if (uc == 0 && tid == 0) rc_update(c, P, PM, PV, GF, c.fo.b1 + kj, db1, as);
    __syncthreads();
  }

  // ---- part 3b: dW0 tile = dz^T Xw (+ adjacency-L1 term through the group norms) and Adam
  float* W0 = P + c.fo.W0 + (int64_t)kj * h * Q;
  float* M0 = PM + c.fo.W0 + (int64_t)kj * h * Q;
  float* V0 = PV + c.fo.W0 + (int64_t)kj * h * Q;
  float* G0w = GF + c.fo.W0 + (int64_t)kj * h * Q;
  float* dZs = tiles + 512;                  // [FB_BT][FAC_UC+1]
  float* Xs = dZs + FB_BT * (FAC_UC + 1);    // [FB_BT][FB_QT+1]
  float* w1s = Xs + FB_BT * (FB_QT + 1);     // [FAC_UC]
  if (tid < FAC_UC) w1s[tid] = (u0 + tid < h) ? W1[u0 + tid] : 0.f;
  const int tq = tid & 15, tu = tid >> 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int bb0 = 0; bb0 < B; bb0 += FB_BT) {
    __syncthreads();
    rc_stage<2>(FB_BT * FAC_UC, [&](int e) {
      const int bb = e / FAC_UC, uu = e - bb * FAC_UC;
      const int b = bb0 + bb, u = u0 + uu;
      return (b < B && u < h) ? aw[(int64_t)b * h + u] : 0.f;
    }, [&](int e, float av) {
      const int bb = e / FAC_UC, uu = e - bb * FAC_UC;
      dZs[bb * (FAC_UC + 1) + uu] = av > 0.f ? dyl[bb0 + bb] * w1s[uu] : 0.f;
    });
    rc_stage<8>(FB_BT * FB_QT, [&](int e) {
      const int bb = e / FB_QT, qq = e - bb * FB_QT;
      const int b = bb0 + bb, q = q0 + qq;
      return (b < B && q < Q) ? xwin(c, dL, X, b, q) : 0.f;
    }, [&](int e, float v) { Xs[(e / FB_QT) * (FB_QT + 1) + e % FB_QT] = v; });
    __syncthreads();
#pragma unroll 8
    for (int bb = 0; bb < FB_BT; ++bb) {
      const float zv = dZs[bb * (FAC_UC + 1) + tu];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[jj] += zv * Xs[bb * (FB_QT + 1) + tq + 16 * jj];
    }
  }
  {
    const int u = u0 + tu;
    if (u < h) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int q = q0 + tq + 16 * jj;
        if (q >= Q) continue;
        const int64_t idx = (int64_t)u * Q + q;
        float g = acc[jj];
        if (adj_grad && Gs[q] > 0.f) g += dGs[q] * (W0[idx] / Gs[q]);
        rc_update(c, W0, M0, V0, G0w, idx, g, as);
      }
    }
  }
}

int fac_bwd_lds_floats(const RedcliffDims& d, int Ls) {
  const int Q = d.p * d.L;
  return 2 * d.Bmax + 2 * Q + d.p + d.L + 16 + d.p * Ls + d.Bmax * d.K + 512 + FB_BT * (FAC_UC + 1) + FB_BT * (FB_QT + 1) + FAC_UC;
}

}  // namespace

int rc_launch_fac_fwd(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  if (d.h > 128 || d.p * d.L > 4096) { rc_set_error("factor forward: h <= 128 and p*L <= 4096 required"); return REDCLIFF_ELIMIT; }
  hipLaunchKernelGGL(k_fac_fwd, dim3(d.K * d.p * rc_nuchunk(d), d.R), dim3(RC_BLOCK), 0, s, c);
  return rc_check(hipGetLastError(), "k_fac_fwd");
}

int rc_launch_fac_bwd(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int Q = d.p * d.L;
  const int nQ = (c.flags & RC_STEP_B) ? (Q + FB_QT - 1) / FB_QT : 1;
  const size_t lds = sizeof(float) * (size_t)fac_bwd_lds_floats(d, c.Ls);
  if (lds > RC_LDS_LIMIT_FLOATS * sizeof(float)) { rc_set_error("factor backward: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  // without a factor update only the lead workgroup of each network has work
  const int nUl = (c.flags & RC_STEP_B) ? rc_nuchunk(d) : 1;
  hipLaunchKernelGGL(k_fac_bwd, dim3(d.K * d.p * nUl * nQ, d.R), dim3(RC_BLOCK), lds, s, c, nUl, nQ);
  return rc_check(hipGetLastError(), "k_fac_bwd");
}

// Stand-alone forward of K cMLPs on B windows Xwin[B][L][p] (cMLP.forward, models/cmlp.py:90-101,
// and the per-factor predictions of REDCLIFF forward).  Per replica the workspace holds
// a[K][p][B][h] | y[nU][B][K][p] (partials over hidden chunks) | G[K][p][p][L] | G0[K][p][p] | w1[K][p][h]
// | gq[nU][K][p][p*L].  G / G0 are left unset (use redcliff_gc_norms).
extern "C" int redcliff_factor_forward(const RedcliffDims* d, int32_t B, const float* Xwin, int64_t x_rstride,
                                       const float* fac, int64_t fac_stride, float* ws, int64_t ws_rstride,
                                       void* stream) {
  if (!d || !Xwin || !fac || !ws || B < 1) { rc_set_error("factor_forward: bad arguments"); return REDCLIFF_EINVAL; }
  if (d->p > 64 || d->h > 128 || d->L > 64) { rc_set_error("factor_forward: dims outside kernel limits"); return REDCLIFF_ELIMIT; }
  StepCtx c;
  memset(&c, 0, sizeof(c));
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
  return rc_launch_fac_fwd(c, (hipStream_t)stream);
}
