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

__device__ inline float xwin(const StepCtx& c, const float* X, int b, int q) {
  const int L = c.d.L;
  const int t = q % L, ch = q / L;
  return X[((c.row0 + b) * c.d.T + (c.Lmax - L + t)) * c.d.p + ch];
}

// ------------------------------------------------------------------------------------------
// K2a: forward of every (factor, channel) network.  grid (K*p, R).
template <int TN>
__global__ __launch_bounds__(RC_BLOCK) void k_fac_fwd(StepCtx c) {
  const RedcliffDims& d = c.d;
  const int r = blockIdx.y, kj = blockIdx.x;
  const int p = d.p, h = d.h, K = d.K;
  const int k = kj / p, j = kj - k * p;
  const int Q = p * d.L;
  const int HP = 16 * TN;
  const float* P = c.fac + r * c.fs;
  const float* W0 = P + c.fo.W0 + (int64_t)kj * h * Q;
  const float* b0 = P + c.fo.b0 + (int64_t)kj * h;
  const float* W1 = P + c.fo.W1 + (int64_t)kj * h;
  const float b1 = P[c.fo.b1 + kj];
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const int tid = threadIdx.x, tb = tid >> 4, tu = tid & 15;

  __shared__ float Xs[FK_BT * (FK_QT + 1)];
  __shared__ float Ws[16 * TN * (FK_QT + 1)];

  for (int bc = 0; bc < c.B; bc += FK_BT) {
    float acc[8][TN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) acc[i][jj] = 0.f;
    for (int q0 = 0; q0 < Q; q0 += FK_QT) {
      for (int e = tid; e < FK_BT * FK_QT; e += RC_BLOCK) {
        const int bb = e / FK_QT, qq = e - bb * FK_QT;
        const int b = bc + bb, q = q0 + qq;
        Xs[bb * (FK_QT + 1) + qq] = (b < c.B && q < Q) ? xwin(c, X, b, q) : 0.f;
      }
      for (int e = tid; e < HP * FK_QT; e += RC_BLOCK) {
        const int u = e / FK_QT, qq = e - u * FK_QT;
        const int q = q0 + qq;
        Ws[u * (FK_QT + 1) + qq] = (u < h && q < Q) ? W0[(int64_t)u * Q + q] : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int qq = 0; qq < FK_QT; ++qq) {
        float xv[8], wv[TN];
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = Xs[(tb + 16 * i) * (FK_QT + 1) + qq];
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) wv[jj] = Ws[(tu + 16 * jj) * (FK_QT + 1) + qq];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int jj = 0; jj < TN; ++jj) acc[i][jj] += xv[i] * wv[jj];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int b = bc + tb + 16 * i;
      float ys = 0.f;
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int u = tu + 16 * jj;
        if (u < h) {
          const float a = fmaxf(acc[i][jj] + b0[u], 0.f);
          if (b < c.B) ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u] = a;
          ys += W1[u] * a;
        }
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) ys += __shfl_xor(ys, o, 64);
      if (tu == 0 && b < c.B) ws[c.wo.y + ((int64_t)b * K + k) * p + j] = ys + b1;
    }
  }
  // group norms of this network's layer-0 weights (GC, models/cmlp.py:162-166)
  for (int e = tid; e < Q; e += RC_BLOCK) {
    float s = 0.f;
    for (int u = 0; u < h; ++u) {
      const float w = W0[(int64_t)u * Q + e];
      s += w * w;
    }
    ws[c.wo.G + (int64_t)kj * Q + e] = sqrtf(s);
  }
  for (int cc = tid; cc < p; cc += RC_BLOCK) {
    float s = 0.f;
    for (int u = 0; u < h; ++u)
      for (int t = 0; t < d.L; ++t) {
        const float w = W0[(int64_t)u * Q + cc * d.L + t];
        s += w * w;
      }
    ws[c.wo.G0 + (int64_t)kj * p + cc] = sqrtf(s);
  }
}

// ------------------------------------------------------------------------------------------
// K2b: mixing, forecast loss, adjacency L1, backward and Adam of every network.
// grid (K*p, R).
template <int TN>
__global__ __launch_bounds__(RC_BLOCK) void k_fac_bwd(StepCtx c) {
  const RedcliffDims& d = c.d;
  const int r = blockIdx.y, kj = blockIdx.x;
  const int p = d.p, h = d.h, K = d.K, L = d.L;
  const int k = kj / p, j = kj - k * p;
  const int Q = p * L;
  const int HP = 16 * TN;
  float* P = c.fac + r * c.fs;
  float* PM = c.facM + r * c.fs;
  float* PV = c.facV + r * c.fs;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int tid = threadIdx.x;
  const int B = c.B;
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
  float* tiles = dAp + p * c.Ls;

  // ---- part 1: mixture x_sim = sum_k w_k y_k, forecast residual, dL/dy and dL/dw (forecast)
  const float gscale = (c.flags & RC_LOSS_FORECAST) ? hy.c_forecast * (2.f / (float)B) : 0.f;
  float fsum = 0.f;
  for (int b = tid; b < B; b += RC_BLOCK) {
    const float* wr = ws + c.wo.w + (int64_t)b * K;
    const float* yr = ws + c.wo.y + (int64_t)b * K * p;
    float xs = 0.f;
    for (int kk = 0; kk < K; ++kk) {
      const float we = sig ? rc_sigmoid(ecc * wr[kk]) : wr[kk];
      xs = (kk == 0) ? we * yr[kk * p + j] : xs + we * yr[kk * p + j];
    }
    // the target X[:, Lmax] exists only when a loss is requested (forward() passes X[:, :Lmax])
    const float res = (c.flags & (RC_LOSS_FORECAST | RC_VALUES)) ? xs - X[((c.row0 + b) * d.T + c.Lmax) * p + j] : 0.f;
    const float wb = sig ? rc_sigmoid(ecc * wr[k]) : wr[k];
    const float g = gscale * res;
    wk[b] = wb;
    dyl[b] = g * wb;
    if (fgrad) ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k] = g * yr[k * p + j];
    if (k == 0) {
      fsum += res * res;
      ws[c.wo.xsim + (int64_t)b * p + j] = xs;
    }
  }
  if (values && k == 0) {
    const float t = rc_block_sum(fsum, red);
    if (tid == 0) ws[c.wo.lossp + j] = t;
  }

  // ---- part 2: adjacency L1 of the conditional GC estimate  w_bk G_k[j][c][t] + A[c][j]
  const bool adj_on = adj_grad || values;
  const int Ls = c.Ls;
  if (adj_on) {
    for (int e = tid; e < Q; e += RC_BLOCK) {
      Gs[e] = ws[c.wo.G + (int64_t)kj * Q + e];
      dGs[e] = 0.f;
    }
    for (int cc = tid; cc < p; cc += RC_BLOCK) Acol[cc] = E[c.eo.A + cc * p + j];
    for (int i = tid; i < Ls; i += RC_BLOCK) lwt[i] = logf((float)(i + 2));
    __syncthreads();
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
      if (c.flags & RC_STEP_A) {
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

  // ---- part 3a: output layer and ReLU backward (dz overwrites the stored activations)
  float* aw = ws + c.wo.a + (int64_t)kj * d.Bmax * h;
  float* W1 = P + c.fo.W1 + (int64_t)kj * h;
  float dW1u = 0.f, db0u = 0.f;
  if (tid < h) {
    const float w1 = W1[tid];
    for (int b = 0; b < B; ++b) {
      const float av = aw[(int64_t)b * h + tid];
      dW1u += dyl[b] * av;
      const float dz = av > 0.f ? dyl[b] * w1 : 0.f;
      db0u += dz;
      aw[(int64_t)b * h + tid] = dz;
    }
  }
  float db1 = 0.f;
  for (int b = tid; b < B; b += RC_BLOCK) db1 += dyl[b];
  db1 = rc_block_sum(db1, red);  // includes a __syncthreads: dz visible to the workgroup

  // ---- part 3b: dW0 = dz^T Xw (+ adjacency-L1 term through the group norms) and Adam
  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  float* W0 = P + c.fo.W0 + (int64_t)kj * h * Q;
  float* M0 = PM + c.fo.W0 + (int64_t)kj * h * Q;
  float* V0 = PV + c.fo.W0 + (int64_t)kj * h * Q;
  float* dZs = tiles;                         // [FB_BT][HP+1]
  float* Xs = dZs + FB_BT * (HP + 1);         // [FB_BT][FB_QT+1]
  const int tq = tid & 15, tu = tid >> 4;
  for (int q0 = 0; q0 < Q; q0 += FB_QT) {
    float acc[TN][4];
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = 0.f;
    for (int bb0 = 0; bb0 < B; bb0 += FB_BT) {
      for (int e = tid; e < FB_BT * HP; e += RC_BLOCK) {
        const int bb = e / HP, u = e - bb * HP;
        const int b = bb0 + bb;
        dZs[bb * (HP + 1) + u] = (b < B && u < h) ? aw[(int64_t)b * h + u] : 0.f;
      }
      for (int e = tid; e < FB_BT * FB_QT; e += RC_BLOCK) {
        const int bb = e / FB_QT, qq = e - bb * FB_QT;
        const int b = bb0 + bb, q = q0 + qq;
        Xs[bb * (FB_QT + 1) + qq] = (b < B && q < Q) ? xwin(c, X, b, q) : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int bb = 0; bb < FB_BT; ++bb) {
        float zv[TN], xv[4];
#pragma unroll
        for (int i = 0; i < TN; ++i) zv[i] = dZs[bb * (HP + 1) + tu + 16 * i];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) xv[jj] = Xs[bb * (FB_QT + 1) + tq + 16 * jj];
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[i][jj] += zv[i] * xv[jj];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int u = tu + 16 * i;
      if (u >= h) continue;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int q = q0 + tq + 16 * jj;
        if (q >= Q) continue;
        const int64_t idx = (int64_t)u * Q + q;
        float pw = W0[idx];
        float g = acc[i][jj];
        if (adj_grad && Gs[q] > 0.f) g += dGs[q] * (pw / Gs[q]);
        float mm = M0[idx], vv = V0[idx];
        rc_adam(pw, mm, vv, g, as);
        W0[idx] = pw; M0[idx] = mm; V0[idx] = vv;
      }
    }
  }
  // ---- part 3c: biases and the output layer
  if (tid < h) {
    const int64_t ib = c.fo.b0 + (int64_t)kj * h + tid;
    rc_adam(P[ib], PM[ib], PV[ib], db0u, as);
    const int64_t iw = c.fo.W1 + (int64_t)kj * h + tid;
    rc_adam(P[iw], PM[iw], PV[iw], dW1u, as);
  }
  if (tid == 0) {
    const int64_t i1 = c.fo.b1 + kj;
    rc_adam(P[i1], PM[i1], PV[i1], db1, as);
  }
}

template <int TN>
int launch_fwd_t(const StepCtx& c, hipStream_t s) {
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fac_fwd<TN>), dim3(c.d.K * c.d.p, c.d.R), dim3(RC_BLOCK), 0, s, c);
  return rc_check(hipGetLastError(), "k_fac_fwd");
}

template <int TN>
int launch_bwd_t(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int Q = d.p * d.L;
  const size_t lds = sizeof(float) * (2 * (size_t)d.Bmax + 2 * Q + d.p + d.L + 16 + (size_t)d.p * c.Ls +
                                      FB_BT * (16 * TN + 1) + FB_BT * (FB_QT + 1));
  if (lds > RC_LDS_LIMIT_FLOATS * sizeof(float)) { rc_set_error("factor backward: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fac_bwd<TN>), dim3(d.K * d.p, d.R), dim3(RC_BLOCK), lds, s, c);
  return rc_check(hipGetLastError(), "k_fac_bwd");
}

}  // namespace

int rc_launch_fac_fwd(const StepCtx& c, hipStream_t s) {
  const int h = c.d.h;
  if (h <= 16) return launch_fwd_t<1>(c, s);
  if (h <= 32) return launch_fwd_t<2>(c, s);
  if (h <= 64) return launch_fwd_t<4>(c, s);
  if (h <= 128) return launch_fwd_t<8>(c, s);
  rc_set_error("factor hidden width %d > 128", h);
  return REDCLIFF_ELIMIT;
}

int rc_launch_fac_bwd(const StepCtx& c, hipStream_t s) {
  const int h = c.d.h;
  if (h <= 16) return launch_bwd_t<1>(c, s);
  if (h <= 32) return launch_bwd_t<2>(c, s);
  if (h <= 64) return launch_bwd_t<4>(c, s);
  if (h <= 128) return launch_bwd_t<8>(c, s);
  rc_set_error("factor hidden width %d > 128", h);
  return REDCLIFF_ELIMIT;
}

// Stand-alone forward of K cMLPs on B windows Xwin[B][L][p] (cMLP.forward, models/cmlp.py:90-101,
// and the per-factor predictions of REDCLIFF forward).  Per replica the workspace holds
// a[K][p][B][h] | y[B][K][p] | G[K][p][p][L] | G0[K][p][p].
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
  c.wo.G = c.wo.y + (int64_t)B * kp;
  c.wo.G0 = c.wo.G + kp * d->p * d->L;
  return rc_launch_fac_fwd(c, (hipStream_t)stream);
}
