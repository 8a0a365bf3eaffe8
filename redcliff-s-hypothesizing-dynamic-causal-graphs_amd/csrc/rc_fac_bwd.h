// rc_fac_bwd.h -- the vector-path factor backward workgroup (mixing, forecast loss, adjacency
// L1, backward and Adam of one network x hidden chunk x dW0 column tile), shared by the
// stand-alone launch k_fac_bwd (rc_factor.hip) and the merged backward launch k_bwd_merged
// (rc_embed.hip).  Included inside an anonymous namespace by both translation units.
//
// Reference: models/cmlp.py:12-35, :147-167; models/redcliff_s_cmlp_withStateSmoothing.py:
// 326-385 (x_sim = sum_k w_k * pred_k), :629 (forecast MSE), :696-715 (lag-weighted adjacency
// L1 of the conditional GC estimate w_bk * G_k[..., -min(L,F):] + A^T).
#pragma once
#include "rc_common.h"

namespace {

#define FB_BT 128   // windows per backward tile (the whole batch at B <= 128)
#define FB_QT 64    // dW0 columns per backward tile
#ifndef RC_FB_MFMA
#define RC_FB_MFMA 1  // activation recompute and dW0 tile on v_mfma_f32_16x16x4_f32 (same chains)
#endif

template <class Div>
__device__ inline float xwin(const StepCtx& c, const Div& dL, const float* X, int b, int q) {
  const int L = c.d.L;
  const int ch = dL.div(q), t = q - ch * L;
  return X[((c.row0 + b) * c.d.T + (c.Lmax - L + t)) * c.d.p + ch];
}

// ------------------------------------------------------------------------------------------
// K2b: mixing, forecast loss, adjacency L1, backward and Adam.  grid (K*p*nU*nQ, R):
// workgroup (network kj, hidden chunk uc, dW0 column tile qc).  The cheap per-window work
// (x_sim, residual, dL/dy, adjacency-L1 signs) is recomputed by every workgroup of a network;
// its outputs (dL/dw partials, loss values, dL/dA) are written by the (uc, qc) = (0, 0) one.
// Latency structure: every global operand of the workgroup -- predictions, embedder outputs,
// target, group-norm partials, A column, the chunk's activations, the window tile and the
// Adam state of the parameters it updates -- is requested in ONE staging pass at the start;
// the rest is LDS / register work and one store pass.
__host__ __device__ inline int fb_tsz(const RedcliffDims& d) {
  const int a = d.Bmax > RC_BLOCK ? d.Bmax : RC_BLOCK, b = d.p * d.L;
  return a > b ? a : b;
}

__device__ inline void rc_adam_pre(const StepCtx& c, float* P, float* M, float* V, float* G, int64_t idx, float g,
                                   const RcAdamScalars& s, float pp, float mm, float vv) {
  if (c.flags & RC_GRAD_ONLY) {
    G[idx] = g;
    return;
  }
  rc_adam(pp, mm, vv, g, s);
  P[idx] = pp; M[idx] = mm; V[idx] = vv;
}

// One workgroup (network kj, hidden chunk uc, dW0 column tile qc) of replica r.  publish != nullptr
// (the merged backward launch, k_bwd_merged): the lead workgroup of each network signals, after
// its dL/dw partials, group norms and dL/dA records are in memory, by an agent-scope release and
// an increment of *publish (the embedder-backward workgroups of the same launch wait for all K*p).
// role (split-lead step, rc_capi.hip): RC_FB_ALL = records and update; RC_FB_RECORDS = the lead's
// records only (one workgroup per network, returns before the update); RC_FB_UPDATE = the update
// only (no workgroup writes the records).  The arithmetic of every part is the same in each role.
__device__ __forceinline__ void fac_bwd_wg(const StepCtx& c, int nUl, int nQ, int kj, int uc, int qc, int r, float* sm,
                           unsigned* publish, int role = RC_FB_ALL) {
  const RedcliffDims& d = c.d;
  const int nU = rc_nuchunk(d);
  const bool lead = (uc == 0 && qc == 0) && role != RC_FB_UPDATE;
  const bool sc1 = publish != nullptr;  // payload read inside this launch: write-through stores
  (void)nUl;
  (void)nQ;
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
  const RcDiv32 dL(d.L, c.mg[RC_MG_L]), dB(B, c.mg[RC_MG_B]);
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const bool fgrad = (c.flags & RC_STEP_B) || (c.flags & RC_STEP_A);
  const bool adj_grad = fgrad && (c.flags & RC_LOSS_ADJ);
  const bool values = c.flags & RC_VALUES;
  const bool stepB = c.flags & RC_STEP_B;
  const bool tgt = c.flags & (RC_LOSS_FORECAST | RC_VALUES);
  const int Ls = c.Ls;
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_BWD, 0);

  float* ybuf = sm;                        // [Bmax][K]  per-factor predictions
  float* wrl = ybuf + d.Bmax * K;          // [Bmax][K]  raw embedder outputs
  float* xt = wrl + d.Bmax * K;            // [Bmax]     forecast target X[:, Lmax, j]
  float* dyl = xt + d.Bmax;                // [Bmax]     dL/dy_bk
  float* wk = dyl + d.Bmax;                // [Bmax]     w_bk (post-sigmoid)
  float* sqs = wk + d.Bmax;                // [Q]        squared group norms
  float* Gs = sqs + Q;                     // [Q]
  float* dGs = Gs + Q;                     // [Q]
  float* Acol = dGs + Q;                   // [p]
  float* lwt = Acol + p;                   // [L]
  float* red = lwt + L;                    // [16]
  float* rA = red + 16;                    // [2*RC_BLOCK] reduction partials
  float* rB = rA + RC_BLOCK;
  float* tpart = rB + RC_BLOCK;            // [fb_tsz]  lead's window partials, then dL/dA items
  float* awl = tpart + fb_tsz(d);          // [FB_BT][17] chunk activations / dZ
  float* Xs = awl + FB_BT * (FAC_UC + 1);  // [FB_BT][FB_QT+1] window tile
  float* w1s = Xs + FB_BT * (FB_QT + 1);   // [FAC_UC] W1 snapshot of the chunk
  float* Wc = w1s + FAC_UC;                // [FAC_UC][FB_QT+1] the chunk's W0 rows (recompute)
  float* bc0 = Wc + FAC_UC * (FB_QT + 1);  // [FAC_UC]          and its b0
  // p*L <= FB_QT: the hidden activations are recomputed here from the window tile and the
  // chunk's (pre-update) W0 rows -- the forward's exact fmaf chain, so the same bits -- instead of
  // being written by the forward and read back (2 MB each way per D4IC step)
  const bool recompute = rc_fac_recompute(d);

  // ---- staging: one pass for everything the workgroup reads, except for the lead workgroup of
  // a merged launch, which stages only what its published records need (predictions, embedder
  // outputs, targets, group-norm partials, A column), publishes, and then stages the operands of
  // its own dW0 / Adam work (the embedder workgroups of the launch wait for the K*p leads)
  // the dW0 tile elements of this thread: (unit u0 + tu + ..., column q0 + tq + ...); with the
  // matrix-core products (RC_FB_MFMA) a lane holds the 16x16x4 result layout: units
  // u0 + 4 (lane >> 4) + jj, column q0 + 16 wave + (lane & 15)
  const int fl15 = tid & 15, flg = (tid >> 4) & 3, fwv = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto tile_u = [&](int jj) { return RC_FB_MFMA ? 4 * flg + jj : (tid >> 4); };
  auto tile_q = [&](int jj) { return RC_FB_MFMA ? 16 * fwv + fl15 : (tid & 15) + 16 * jj; };
  const int tq = tid & 15, tu = tid >> 4;
  const int64_t kjW0 = c.fo.W0 + (int64_t)kj * h * Q;
  float pw[4] = {0.f, 0.f, 0.f, 0.f}, pm[4] = {0.f, 0.f, 0.f, 0.f}, pv[4] = {0.f, 0.f, 0.f, 0.f};
  float sb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s1[3] = {0.f, 0.f, 0.f};
  const bool gonly = c.flags & RC_GRAD_ONLY;
  const bool split = lead && publish != nullptr;
  auto adam_loads = [&]() {
    if (stepB && !gonly) {  // Adam state of the parameters this thread updates
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int u = u0 + tile_u(jj), q = q0 + tile_q(jj);
        if (u < h && q < Q) {
          const int64_t idx = kjW0 + (int64_t)u * Q + q;
          pw[jj] = P[idx]; pm[jj] = PM[idx]; pv[jj] = PV[idx];
        }
      }
      if (qc == 0 && tid < FAC_UC && u0 + tid < h) {
        const int64_t ib = c.fo.b0 + (int64_t)kj * h + u0 + tid, iw = c.fo.W1 + (int64_t)kj * h + u0 + tid;
        sb[0] = P[ib]; sb[1] = PM[ib]; sb[2] = PV[ib];
        sb[3] = P[iw]; sb[4] = PM[iw]; sb[5] = PV[iw];
      }
      if (qc == 0 && uc == 0 && tid == 0) {
        const int64_t i1 = c.fo.b1 + kj;
        s1[0] = P[i1]; s1[1] = PM[i1]; s1[2] = PV[i1];
      }
    }
  };
  if (!split && role != RC_FB_RECORDS) adam_loads();
  const float* aw = ws + c.wo.a + (int64_t)kj * d.Bmax * h;
  const float* W1snap = ws + c.wo.w1 + (int64_t)kj * h;  // pre-update snapshot written by the forward
  const int64_t ys_ = (int64_t)d.Bmax * K * p;
  const int nb0 = min(B, FB_BT);
  // the dW0 / Adam operands (late: staged after the lead's publish)
  auto stage_update = [&](bool on) {
    rc_stage_all(
        rc_seg<1>(on && stepB ? FAC_UC : 0, [&](int e) { return u0 + e < h ? W1snap[u0 + e] : 0.f; },
                  [&](int e, float v) { w1s[e] = v; }),
        rc_seg<8>(on && stepB && !recompute ? nb0 * FAC_UC : 0, [&](int e) {
          const int bb = e >> 4, uu = e & 15;
          return u0 + uu < h ? aw[(int64_t)bb * h + u0 + uu] : 0.f;
        }, [&](int e, float v) { awl[(e >> 4) * (FAC_UC + 1) + (e & 15)] = v; }),
        rc_seg<4>(on && stepB && recompute ? FAC_UC * Q : 0, [&](int e) {
          const int uu = e / Q, q = e - uu * Q;
          return u0 + uu < h ? P[kjW0 + (int64_t)(u0 + uu) * Q + q] : 0.f;
        }, [&](int e, float v) { Wc[(e / Q) * (FB_QT + 1) + e % Q] = v; }),
        rc_seg<1>(on && stepB && recompute ? FAC_UC : 0, [&](int e) {
          return u0 + e < h ? P[c.fo.b0 + (int64_t)kj * h + u0 + e] : 0.f;
        }, [&](int e, float v) { bc0[e] = v; }),
        rc_seg<32>(on && stepB ? nb0 * FB_QT : 0, [&](int e) {
          const int bb = e >> 6, qq = e & 63;
          return q0 + qq < Q ? xwin(c, dL, X, bb, q0 + qq) : 0.f;
        }, [&](int e, float v) { Xs[(e >> 6) * (FB_QT + 1) + (e & 63)] = v; }));
  };
  if (!split && role != RC_FB_RECORDS) stage_update(true);
  // The two partial sums come last and load every slot unconditionally (slots >= nU read slot 0
  // and are not added): a guarded load is a branch, and a sum between branches waits for its
  // loads before the next element's are issued -- one memory round per element otherwise.
  rc_stage_all(
      rc_seg<8>(B * K, [&](int e) { return ws[c.wo.w + e]; }, [&](int e, float v) { wrl[e] = v; }),
      rc_seg<1>(tgt ? B : 0, [&](int b) { return X[((c.row0 + b) * d.T + c.Lmax) * p + j]; },
                [&](int b, float v) { xt[b] = v; }),
      rc_seg<1>(p, [&](int cc) { return E[c.eo.A + cc * p + j]; }, [&](int cc, float v) { Acol[cc] = v; }),
      rc_seg<8>(B * K, [&](int e) {  // sum of the nU hidden-chunk partials (fixed order); e = kk * B + b
        const int kk = dB.div(e), b = e - kk * B;
        const float* yp = ws + c.wo.y + rc_y_idx(d, 0, kk * p + j, b);
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = yp[(q < nU ? q : 0) * ys_];
        float yv = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) yv += q < nU ? v[q] : 0.f;
        return yv;
      }, [&](int e, float v) {
        const int kk = dB.div(e);
        ybuf[(e - kk * B) * K + kk] = v;
      }),
      rc_seg<1>(Q, [&](int e) {  // the nU (<= 8) partials loaded together, summed in slot order
        const float* gp = ws + c.wo.gq + (int64_t)kj * Q + e;
        const int64_t gs_ = (int64_t)K * p * Q;
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = gp[(q < nU ? q : 0) * gs_];
        float sq = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) sq += q < nU ? v[q] : 0.f;
        return sq;
      }, [&](int e, float v) { sqs[e] = v; }));
  for (int i = tid; i < Ls; i += RC_BLOCK) lwt[i] = logf((float)(i + 2));
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 16);

  // ---- part 1: mixture x_sim = sum_k w_k y_k, forecast residual, dL/dy and dL/dw (forecast)
  const float gscale = (c.flags & RC_LOSS_FORECAST) ? hy.c_forecast * (2.f / (float)c.Bg) : 0.f;
  float fsum = 0.f;
  for (int b = tid; b < B; b += RC_BLOCK) {
    const float* wr = wrl + b * K;
    float xs = 0.f;
    for (int kk = 0; kk < K; ++kk) {
      const float we = sig ? rc_sigmoid(ecc * wr[kk]) : wr[kk];
      xs = (kk == 0) ? we * ybuf[b * K + kk] : xs + we * ybuf[b * K + kk];
    }
    const float res = tgt ? xs - xt[b] : 0.f;
    const float wb = sig ? rc_sigmoid(ecc * wr[k]) : wr[k];
    const float g = gscale * res;
    wk[b] = wb;
    dyl[b] = g * wb;
    if (lead && fgrad && !adj_grad) rc_store_payload(ws + c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k, g * ybuf[b * K + k], sc1);
    if (lead && adj_grad) tpart[b] = g * ybuf[b * K + k];  // forecast part, adjacency part added below
    if (lead && k == 0) {
      fsum += res * res;
      ws[c.wo.xsim + (int64_t)b * p + j] = xs;
    }
  }
  // ---- group norms G[kj][c][t] (cmlp.py:147-167)
  for (int e = tid; e < Q; e += RC_BLOCK) {
    const float g = sqrtf(sqs[e]);
    Gs[e] = g;
    dGs[e] = 0.f;
    if (lead) ws[c.wo.G + (int64_t)kj * Q + e] = g;
  }
  if (values && lead && k == 0) {
    const float t = rc_block_sum(fsum, red);
    if (tid == 0) ws[c.wo.lossp + j] = t;
  }
  __syncthreads();
  if (lead)
    for (int cc = tid; cc < p; cc += RC_BLOCK) {
      float sq = 0.f;
      for (int t = 0; t < L; ++t) sq += sqs[cc * L + t];
      ws[c.wo.G0 + (int64_t)kj * p + cc] = sqrtf(sq);
    }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 17);

  // ---- part 2: adjacency L1 of the conditional GC estimate  w_bk G_k[j][c][t] + A[c][j]
  if (lead && (adj_grad || values)) {
    // (window, channel slice) items: nsl slices of the p channels per window
    const int nsl = B >= RC_BLOCK ? 1 : RC_BLOCK / B;
    const int b = tid % B, sl = tid / B;
    float t = 0.f, v = 0.f;
    if (tid < nsl * B) {
      const float wb = wk[b];
      for (int cc = sl; cc < p; cc += nsl)
#pragma unroll 4
        for (int i = 0; i < Ls; ++i) {
          const float g = Gs[cc * L + (L - Ls + i)];
          const float val = wb * g + Acol[cc];
          t += lwt[i] * rc_sign(val) * g;
          if (values) v += lwt[i] * fabsf(val);
        }
    }
    for (int bb = tid + RC_BLOCK; bb < B; bb += RC_BLOCK) {  // B > 256: remaining windows, whole rows
      const float wb = wk[bb];
      float tb = 0.f;
      for (int cc = 0; cc < p; ++cc)
        for (int i = 0; i < Ls; ++i) {
          const float g = Gs[cc * L + (L - Ls + i)];
          const float val = wb * g + Acol[cc];
          tb += lwt[i] * rc_sign(val) * g;
          if (values) v += lwt[i] * fabsf(val);
        }
      if (adj_grad) rc_store_payload(ws + c.wo.dwp + ((int64_t)j * d.Bmax + bb) * K + k, tpart[bb] + hy.c_adj * tb, sc1);
    }
    rA[tid] = t;
    __syncthreads();
    if (adj_grad && tid < B && tid < RC_BLOCK) {
      float s = 0.f;
      for (int q = 0; q < nsl; ++q) s += rA[q * B + tid];
      rc_store_payload(ws + c.wo.dwp + ((int64_t)j * d.Bmax + tid) * K + k, tpart[tid] + hy.c_adj * s, sc1);
    }
    if (values) {
      const float tv = rc_block_sum(v, red);
      if (tid == 0) ws[c.wo.lossp + p + kj] = hy.c_adj * tv;
    }
  }
  if (adj_grad) {
    // dL/dG[q] (q in the lag slice) and dL/dA[c][j]: items (q, window slice)
    const int ni = p * Ls;
    const int nsl = ni >= RC_BLOCK ? 1 : RC_BLOCK / ni;
    const bool needA = lead && (c.flags & RC_STEP_A);
    __syncthreads();
    for (int it = tid; it < ni * nsl; it += RC_BLOCK) {
      const int e = it % ni, sl = it / ni;
      const int cc = e / Ls, i = e - cc * Ls;
      const float g = Gs[cc * L + (L - Ls + i)];
      float sw = 0.f, s1v = 0.f;
#pragma unroll 8
      for (int b = sl; b < B; b += nsl) {  // (unrolled: the LDS reads of 8 windows in flight, same order)
        const float sg = rc_sign(wk[b] * g + Acol[cc]);
        sw += sg * wk[b];
        s1v += sg;
      }
      if (nsl == 1) {
        dGs[cc * L + (L - Ls + i)] = hy.c_adj * lwt[i] * sw;
        tpart[e] = hy.c_adj * lwt[i] * s1v;  // reused: the lead's window partials are consumed
      } else {
        rA[it] = sw;
        rB[it] = s1v;
      }
    }
    __syncthreads();
    if (nsl > 1)
      for (int e = tid; e < ni; e += RC_BLOCK) {
        float sw = 0.f, s1v = 0.f;
        for (int q = 0; q < nsl; ++q) {
          sw += rA[q * ni + e];
          s1v += rB[q * ni + e];
        }
        const int cc = e / Ls, i = e - cc * Ls;
        dGs[cc * L + (L - Ls + i)] = hy.c_adj * lwt[i] * sw;
        tpart[e] = hy.c_adj * lwt[i] * s1v;
      }
    __syncthreads();
    if (needA)
      for (int cc = tid; cc < p; cc += RC_BLOCK) {
        float s = 0.f;
        for (int i = 0; i < Ls; ++i) s += tpart[cc * Ls + i];
        rc_store_payload(ws + c.wo.dAadj + ((int64_t)k * p + cc) * p + j, s, sc1);  // d/dA[c][j]
      }
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 18);
  if (publish && lead) {
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_WAIT, 1);  // trace builds: the lead's publish time (end slot)
    rc_publish(publish);
  }
  if (!stepB || role == RC_FB_RECORDS) return;
  if (split) {  // the lead's own update operands, after its records are out
    adam_loads();
    stage_update(true);
  }
  __syncthreads();

  // trace builds: the update part's phases are recorded by the (network 0, chunk 1) workgroup
  const int tbx = (kj == 0 && uc == 1 && qc == 0 && role == RC_FB_ALL) ? 0 : 1;
  (void)tbx;
  RC_PHASE(c.ws, c.wo.total, tbx, 19);
  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  // ---- part 3: over window tiles of FB_BT (one tile when B <= 128; the first is already staged)
  const int uu = tid & 15, part = tid >> 4;  // 3a: 16 slices of the batch per hidden unit
  float dW1u = 0.f, db0u = 0.f, db1 = 0.f;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  auto recompute_a_mfma = [&](int nb) {
    // a[b][u] = relu(sum_q Xw[b][q] W0[u][q] + b0[u]) as 16x16x4 tiles (rows b, columns u), a
    // k-ascending fmaf chain per output from 0: the forward's chain, so the same bits; the
    // columns q >= Q of the last k step are zeros (exact no-ops).  Wave w: window tiles w, w + 4.
    for (int bt = fwv; bt < (nb + 15) / 16; bt += 4) {
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const float* xr = Xs + (16 * bt + fl15) * (FB_QT + 1);
      const float* wr = Wc + fl15 * (FB_QT + 1);
      for (int k0 = 0; k0 < Q; k0 += 4) {
        const int k = k0 + flg;
        const float av = k < Q ? xr[k] : 0.f, bv = k < Q ? wr[k] : 0.f;
        z = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, z, 0, 0, 0);
      }
      const bool uin = u0 + fl15 < h;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int b = 16 * bt + 4 * flg + reg;
        if (b < nb) awl[b * (FAC_UC + 1) + fl15] = uin ? fmaxf(z[reg] + bc0[fl15], 0.f) : 0.f;
      }
    }
    __syncthreads();
  };
  auto recompute_a = [&](int nb) {  // a = relu(Xw W0^T + b0), rc_forward.hip's chain (q ascending)
    // thread: windows {bp, bp + 64} x units 4*uq .. 4*uq+3 (FB_BT = 128 = 2 x 64, FAC_UC = 16 = 4 x 4):
    // 6 LDS reads per 8 fmaf; every output keeps its own chain z = fmaf(x_q, w_q, z), q ascending
    const int bp = tid >> 2, u4 = (tid & 3) * 4;
    const float* x0 = Xs + bp * (FB_QT + 1);
    const float* x1 = Xs + (bp + 64) * (FB_QT + 1);
    const float* wr = Wc + u4 * (FB_QT + 1);
    float z0[4] = {0.f, 0.f, 0.f, 0.f}, z1[4] = {0.f, 0.f, 0.f, 0.f};
    if (bp < nb) {
      for (int q = 0; q < Q; ++q) {
        const float a0 = x0[q], a1 = x1[q];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float w = wr[i * (FB_QT + 1) + q];
          z0[i] = fmaf(a0, w, z0[i]);
          z1[i] = fmaf(a1, w, z1[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool uin = u0 + u4 + i < h;
        awl[bp * (FAC_UC + 1) + u4 + i] = uin ? fmaxf(z0[i] + bc0[u4 + i], 0.f) : 0.f;
        if (bp + 64 < nb) awl[(bp + 64) * (FAC_UC + 1) + u4 + i] = uin ? fmaxf(z1[i] + bc0[u4 + i], 0.f) : 0.f;
      }
    }
    __syncthreads();
  };
  for (int bt = 0; bt < B; bt += FB_BT) {
    const int nb = min(FB_BT, B - bt);
    if (bt > 0) {
      __syncthreads();
      rc_stage_all(
          rc_seg<8>(recompute ? 0 : nb * FAC_UC, [&](int e) {
            const int bb = e >> 4, u = e & 15;
            return u0 + u < h ? aw[(int64_t)(bt + bb) * h + u0 + u] : 0.f;
          }, [&](int e, float v) { awl[(e >> 4) * (FAC_UC + 1) + (e & 15)] = v; }),
          rc_seg<32>(nb * FB_QT, [&](int e) {
            const int bb = e >> 6, qq = e & 63;
            return q0 + qq < Q ? xwin(c, dL, X, bt + bb, q0 + qq) : 0.f;
          }, [&](int e, float v) { Xs[(e >> 6) * (FB_QT + 1) + (e & 63)] = v; }));
      __syncthreads();
    }
    if (recompute) {
      if (RC_FB_MFMA)
        recompute_a_mfma(nb);
      else
        recompute_a(nb);
    }
    RC_PHASE(c.ws, c.wo.total, tbx, 20);
    // 3a (column tile 0): output-layer / bias gradients of the chunk's hidden units
    if (qc == 0) {
      const float w1 = w1s[uu];
      for (int bb = part; bb < nb; bb += 16) {
        const float av = awl[bb * (FAC_UC + 1) + uu];
        dW1u += dyl[bt + bb] * av;
        db0u += av > 0.f ? dyl[bt + bb] * w1 : 0.f;
      }
      if (uc == 0)
        for (int bb = tid; bb < nb; bb += RC_BLOCK) db1 += dyl[bt + bb];
    }
    __syncthreads();
    // dZ = [a > 0] dL/dy W1 in place of the activations
    for (int e = tid; e < nb * FAC_UC; e += RC_BLOCK) {
      const int bb = e >> 4, u = e & 15;
      const float av = awl[bb * (FAC_UC + 1) + u];
      awl[bb * (FAC_UC + 1) + u] = av > 0.f ? dyl[bt + bb] * w1s[u] : 0.f;
    }
    __syncthreads();
    // 3b: dW0 tile partial = dZ^T Xw, per element an fmaf chain over the windows in order
    if (RC_FB_MFMA) {
      // 16x16x4 tiles: rows u (A[u][b] = dZ[b][u]), columns q = 16 wave + l15, k = the windows
      // (rows >= nb of the last k step are zeros: exact no-ops); the result layout is tile_u /
      // tile_q's
      f32x4 a4 = {acc[0], acc[1], acc[2], acc[3]};
      const float* xc = Xs + 16 * fwv + fl15;
      for (int k0 = 0; k0 < nb; k0 += 4) {
        const int b = k0 + flg;
        const float av = b < nb ? awl[b * (FAC_UC + 1) + fl15] : 0.f;
        const float bv = b < nb ? xc[b * (FB_QT + 1)] : 0.f;
        a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, a4, 0, 0, 0);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[jj] = a4[jj];
    } else {
#pragma unroll 8
      for (int bb = 0; bb < nb; ++bb) {
        const float zv = awl[bb * (FAC_UC + 1) + tu];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[jj] += zv * Xs[bb * (FB_QT + 1) + tq + 16 * jj];
      }
    }
  }
  RC_PHASE(c.ws, c.wo.total, tbx, 21);
  if (qc == 0) {
    rA[tid] = dW1u;
    rB[tid] = db0u;
    if (uc == 0) db1 = rc_block_sum(db1, red);
    __syncthreads();
    if (tid < 16 && u0 + tid < h) {
      float g1 = 0.f, g0 = 0.f;
      for (int s2 = 0; s2 < 16; ++s2) {
        g1 += rA[s2 * 16 + tid];
        g0 += rB[s2 * 16 + tid];
      }
      rc_adam_pre(c, P, PM, PV, GF, c.fo.b0 + (int64_t)kj * h + u0 + tid, g0, as, sb[0], sb[1], sb[2]);
      rc_adam_pre(c, P, PM, PV, GF, c.fo.W1 + (int64_t)kj * h + u0 + tid, g1, as, sb[3], sb[4], sb[5]);
    }
    if (uc == 0 && tid == 0) rc_adam_pre(c, P, PM, PV, GF, c.fo.b1 + kj, db1, as, s1[0], s1[1], s1[2]);
  }
  RC_PHASE(c.ws, c.wo.total, tbx, 22);
  // dW0 tile: + adjacency-L1 term through the group norms, then Adam
  {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int u = u0 + tile_u(jj), q = q0 + tile_q(jj);
      if (u >= h || q >= Q) continue;
      const int64_t idx = kjW0 + (int64_t)u * Q + q;
      float g = acc[jj];
      if (adj_grad && Gs[q] > 0.f) g += dGs[q] * ((gonly ? P[idx] : pw[jj]) / Gs[q]);
      rc_adam_pre(c, P, PM, PV, GF, idx, g, as, pw[jj], pm[jj], pv[jj]);
    }
  }
  RC_PHASE(c.ws, c.wo.total, tbx, 23);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_BWD, 1);
}

inline int fac_bwd_lds_floats(const RedcliffDims& d) {
  const int Q = d.p * d.L;
  return 2 * d.Bmax * d.K + 3 * d.Bmax + 3 * Q + d.p + d.L + 16 + 2 * RC_BLOCK + fb_tsz(d) +
         FB_BT * (FAC_UC + 1) + FB_BT * (FB_QT + 1) + FAC_UC + FAC_UC * (FB_QT + 1) + FAC_UC;
}


}  // namespace
