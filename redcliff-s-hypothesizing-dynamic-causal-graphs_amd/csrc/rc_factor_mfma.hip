// rc_factor_mfma.hip -- the K x p factor networks as grouped GEMMs on the gfx950 matrix
// cores, for layer-0 contractions long enough to pay off (the stress config p=64, L=20:
// p*L = 1280, K*p*h = 12,800 hidden units; BASELINE configs[4]).
//
// Reference: models/cmlp.py:12-35 (MLP: Conv1d(p, h, L) -> ReLU -> Conv1d(h, 1, 1)),
// models/cmlp.py:147-167 (group norms), ...withStateSmoothing.py:326-385 (x_sim mixing),
// :629 (forecast MSE), :696-715 (lag-weighted adjacency L1 of w_bk G_k + A^T).
//
// With num_sims == 1 the factor forward is one GEMM  Z[b][(kj,u)] = sum_q Xw[b][q] W0[kj][u][q]
// (B x p*L x K*p*h) and the layer-0 weight gradient another, dW0[kj][u][q] = sum_b dZ[b][(kj,u)]
// Xw[b][q].  Both run on v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate: every product rounded
// once, exactly an fmaf chain -- cdna_hip_programming.md §3): one 32-column block = one network
// (hidden units padded to 32), so the bias / ReLU / output-layer epilogue and the Adam update
// stay per network.  The small per-network work between the GEMMs (mixing, residual, penalty
// gradients, output-layer updates) runs once per network in k_fac_mix instead of once per tile.
//
// Kernel chain: k_xwin (windows -> Xw[b][q], q = c*L + t) -> k_fac_fwd_mfma -> k_fac_mix ->
// k_fac_bwd_mfma (dW0 GEMM + adjacency-L1 term + Adam epilogue).
#include <cstdlib>
#include <cstring>

#include "rc_common.h"
// k_fac_bwd_mfma occupancy (measured on the R = 32 D4IC grid and C5): without the epilogue-operand
// prefetch the kernel fits 3 waves per SIMD without spills, which hides more latency than the
// prefetch did at 2 waves (grid step 0.54 -> 0.51 ms, fac_bwd 140 -> 114 us; C5 0.52 -> 0.50 ms);
// 4 waves spill.  Same arithmetic either way.
#ifndef RC_FB_WAVES
#define RC_FB_WAVES 3
#endif
#ifndef RC_FB_PREFETCH
#define RC_FB_PREFETCH 0
#endif
#ifndef RC_FB_WAVES4  // the short-contraction variant also holds the recompute operands
#define RC_FB_WAVES4 2
#endif

namespace {

#define MF_BT 64   // windows per forward tile (2 row blocks of 32)
#define MF_QC 32   // contraction chunk per staging step (16 MFMA k-steps)
#define MB_BC 32   // windows per backward staging step

__device__ inline float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------------------------------
// Window transpose: Xw[b][c*L + t] = X[row0 + b][Lmax - L + t][c], zero-padded to Qp columns.
// grid (ceil(B * Qp / (4 * 256)), R): 4 elements (window b, source offset e = t*p + c of its
// contiguous L*p slice) per thread, every load issued before the stores.
#define XW_PER 4
__global__ __launch_bounds__(RC_BLOCK) void k_xwin(StepCtx c) {
  const int r = rc_rep(c, blockIdx.y);
  const RedcliffDims& d = c.d;
  const int L = d.L, p = d.p, Q = p * L, Qp = rc_qpad(d), n = c.B * Qp;
  const float* src = c.X + r * c.xr + (c.row0 * d.T + (c.Lmax - L)) * p;
  float* dst = c.ws + r * c.wss + c.wo.xw;
  const RcDiv dq(Qp), dp(p);
  const int e0 = blockIdx.x * XW_PER * RC_BLOCK + threadIdx.x;
  float v[XW_PER];
#pragma unroll
  for (int u = 0; u < XW_PER; ++u) {
    const int e = e0 + u * RC_BLOCK, b = dq.div(e), k = e - b * Qp;
    v[u] = (e < n && k < Q) ? src[(int64_t)b * d.T * p + k] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < XW_PER; ++u) {
    const int e = e0 + u * RC_BLOCK, b = dq.div(e), k = e - b * Qp;
    if (e >= n) continue;
    if (k < Q) {
      const int t = dp.div(k), ch = k - t * p;
      dst[(int64_t)b * Qp + ch * L + t] = v[u];
    } else {
      dst[e] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Forward GEMM.  Column blocks cb = (network kj, 32-unit hidden block ub), nUB = ceil(h/32) per
// network; grid (ceil(K*p*nUB/2), ceil(B/64), R); 4 waves: wave w owns rows 32*(w&1) of the
// 64-row tile and column block 2*blockIdx.x + (w>>1), one 32x32 accumulator.  The next chunk's
// operands are loaded into registers while the current chunk's 16 MFMA k-steps run from LDS.
// Epilogue: a = relu(z + b0) -> ws.a (backward), partial y_ub = sum_{u in ub} W1[u] a[u]
// (+ b1 in block 0) -> ws.y slot ub, squared group norms gq[ub][kj][q] = sum_{u in ub} W0[u][q]^2
// (first row block), W1 snapshot.
__host__ __device__ inline int mf_nub(const RedcliffDims& d) { return (d.h + 31) / 32; }
// Short contractions (p*L <= 64, the k_fac_bwd_mfma<4> launch): the backward recomputes the
// hidden activations and forms the output-layer gradients, so neither the forward's activation
// store nor the mixing kernel's activation reads happen.
__host__ __device__ inline bool mf_recompute(const RedcliffDims& d) { return d.p * d.L <= 64; }

__global__ __launch_bounds__(RC_BLOCK) void k_fac_fwd_mfma(StepCtx c) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.z);
  const int cb0 = blockIdx.x * 2, b0 = blockIdx.y * MF_BT;
  const int p = d.p, h = d.h, K = d.K, Q = p * d.L, Qp = rc_qpad(d), KP = K * p, nUB = mf_nub(d);
  const int NB = KP * nUB;
  const float* P = c.fac + r * c.fs;
  float* ws = c.ws + r * c.wss;
  const float* Xw = ws + c.wo.xw;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nb = min(MF_BT, c.B - b0);

  __shared__ float Xs[MF_BT][MF_QC + 1];
  __shared__ float Ws[64][MF_QC + 1];  // [blk*32 + u][q]

  // staging maps: X 64x32 = 512 float4 (2 per thread); W 64x32 = 2048 floats (8 per thread)
  float4 xr[2];
  float wr[8];
  auto load = [&](int q0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * RC_BLOCK, row = e >> 3, c4 = (e & 7) * 4;
      xr[i] = row < nb ? ld4(Xw + (int64_t)(b0 + row) * Qp + q0 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + i * RC_BLOCK, uu = e >> 5, qq = e & 31;
      const int cb = cb0 + (uu >> 5), kj = cb / nUB, u = (cb - kj * nUB) * 32 + (uu & 31), q = q0 + qq;
      wr[i] = (cb < NB && u < h && q < Q) ? P[c.fo.W0 + ((int64_t)kj * h + u) * Q + q] : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * RC_BLOCK, row = e >> 3, c4 = (e & 7) * 4;
      Xs[row][c4] = xr[i].x;
      Xs[row][c4 + 1] = xr[i].y;
      Xs[row][c4 + 2] = xr[i].z;
      Xs[row][c4 + 3] = xr[i].w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + i * RC_BLOCK;
      Ws[e >> 5][e & 31] = wr[i];
    }
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const int arow = 32 * (wv & 1) + (lane & 31), bcol = 32 * (wv >> 1) + (lane & 31), kh = lane >> 5;
  load(0);
  for (int q0 = 0; q0 < Qp; q0 += MF_QC) {
    __syncthreads();
    store();
    __syncthreads();
    if (q0 + MF_QC < Qp) load(q0 + MF_QC);
    if (blockIdx.y == 0 && tid < 64) {  // GC group norms of this chunk (pre-update weights), per block
      const int cb = cb0 + (tid >> 5), q = q0 + (tid & 31);
      if (cb < NB && q < Q) {
        const int kj = cb / nUB, ub = cb - kj * nUB;
        float sq = 0.f;
        for (int u = 0; u < 32; ++u) {
          const float w = Ws[(tid >> 5) * 32 + u][tid & 31];
          sq += w * w;
        }
        ws[c.wo.gq + ((int64_t)ub * KP + kj) * Q + q] = sq;
      }
    }
    // k-steps only up to Q (rounded to the step of 2): the zero padding to Qp adds exact zeros
    // (k_fac_bwd_mfma's recompute runs the same (Q + 1) / 2 steps, so both give the same bits)
    const int kmax = Q - q0;
#pragma unroll
    for (int k0 = 0; k0 < MF_QC; k0 += 2) {
      if (k0 < kmax) {
        const float a = Xs[arow][k0 + kh];
        const float bv = Ws[bcol][k0 + kh];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc, 0, 0, 0);
      }
    }
  }
  // ---- epilogue
  const int cb = cb0 + (wv >> 1);
  if (cb >= NB) return;
  const int kj = cb / nUB, ub = cb - kj * nUB, u = ub * 32 + (lane & 31);
  const int k = kj / p, j = kj - k * p;
  const bool uv = u < h;
  const float bu = uv ? P[c.fo.b0 + (int64_t)kj * h + u] : 0.f;
  const float w1 = uv ? P[c.fo.W1 + (int64_t)kj * h + u] : 0.f;
  const float b1 = ub == 0 ? P[c.fo.b1 + kj] : 0.f;
  if (blockIdx.y == 0 && (wv & 1) == 0 && lane < 32 && uv) ws[c.wo.w1 + (int64_t)kj * h + u] = w1;
  const int nU = rc_nuchunk(d);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int b = b0 + 32 * (wv & 1) + mf_row(reg, lane);
    const float a = uv ? fmaxf(acc[reg] + bu, 0.f) : 0.f;
#ifdef RC_RECOMP_DEBUG
    if (uv && b < c.B) ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u] = a;
#else
    if (uv && b < c.B && !mf_recompute(d)) ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u] = a;
#endif
    float ys = w1 * a;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ys += __shfl_xor(ys, o, 64);  // within the 32-lane half
    if (b < c.B) {
      const int l = lane & 31;
      // slot ub holds this block's partial; block 0 also clears the slots past nUB
      if (l == 0) ws[c.wo.y + rc_y_idx(d, ub, kj, b)] = ys + b1;
      else if (ub == 0 && l >= nUB && l < nU) ws[c.wo.y + rc_y_idx(d, l, kj, b)] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Per-network work between the GEMMs.  grid (K*p, R), one workgroup per network kj:
//   x_sim = sum_k w_k y_k, forecast residual, dL/dy (-> ws.dyl), dL/dw (forecast + adjacency
//   terms, -> ws.dwp), group norms G / G0, adjacency-L1 value and its gradients wrt the
//   lagged group norms (-> ws.dgs, used by the dW0 epilogue) and A (-> ws.dAadj), and the
//   output-layer / hidden-bias gradients + Adam (b0, W1, b1).
// k_fac_mix: predictions staged per thread per round of loads (each with its nUB slot partials)
#ifndef RC_MIX_STAGE_U
#define RC_MIX_STAGE_U 2
#endif
template <int NT>
__global__ __launch_bounds__(NT) void k_fac_mix(StepCtx c, int xcd) {
  const RedcliffDims& d = c.d;
  // xcd: every network of one replica on one XCD (rc_xcd_order): the K networks of a channel
  // read the same y rows, and the replica's w and window targets are shared by all of them
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) rc_xcd_order(gridDim.x, gridDim.y, bx, by);
  const int r = rc_rep(c, by), kj = bx;
  const int p = d.p, h = d.h, K = d.K, L = d.L, Q = p * L, B = c.B;
  const int k = kj / p, j = kj - k * p;
  float* P = c.fac + r * c.fs;
  float* PM = c.facM + r * c.fs;
  float* PV = c.facV + r * c.fs;
  float* GF = c.gF + r * c.fs;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int tid = threadIdx.x;
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const bool fgrad = (c.flags & RC_STEP_B) || (c.flags & RC_STEP_A);
  const bool adj_grad = fgrad && (c.flags & RC_LOSS_ADJ);
  const bool values = c.flags & RC_VALUES;
  const int Ls = c.Ls;

  extern __shared__ float sm[];
  float* dyl = sm;             // [Bmax]
  float* wk = dyl + d.Bmax;    // [Bmax]  w_bk (post-sigmoid)
  float* Gs = wk + d.Bmax;     // [Q]
  float* sqs = Gs + Q;         // [Q]
  float* Acol = sqs + Q;       // [p]
  float* lwt = Acol + p;       // [L]
  float* red = lwt + L;        // [16]
  float* dAp = red + 16;       // [p*Ls]
  float* ybuf = dAp + p * Ls;  // [Bmax][K]
  float* rA = ybuf + d.Bmax * K;  // [256]
  float* rB = rA + RC_BLOCK;      // [256]
  float* dwf = rB + RC_BLOCK;     // [Bmax]  forecast part of dL/dw_bk

  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_MIX, 0);
  // NT < 256 (B <= 128, fac_mix_nt): the block sums run over the windows in the layout of a
  // 256-thread workgroup, window b = virtual thread vv * NT + tid, so every sum keeps its order
  constexpr int NV = RC_BLOCK / NT;
  auto vsum256 = [&](const float (&v)[NV]) {  // rc_block_sum over the virtual layout, every thread gets it
    __syncthreads();
#pragma unroll
    for (int vv = 0; vv < NV; ++vv) {
      const float w = rc_wave_sum(v[vv]);
      if ((tid & 63) == 0) red[vv * (NT / 64) + (tid >> 6)] = w;
    }
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < RC_BLOCK / 64; ++i) t += red[i];
    __syncthreads();
    return t;
  };
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 16);
  // ---- mixture, forecast residual, dL/dy, forecast part of dL/dw
  const float gscale = (c.flags & RC_LOSS_FORECAST) ? hy.c_forecast * (2.f / (float)c.Bg) : 0.f;
  const int nUB = c.fslots;  // y / group-norm slots of the forward (16- or 32-unit blocks)
  // the nUB (<= 8) slot partials of every prediction requested together, summed in slot order;
  // element e = kk * B + b (consecutive windows of one network: contiguous in y) -> ybuf[b][kk]
  const RcDiv dB(B);
  rc_stage<RC_MIX_STAGE_U, NT>(B * K, [&](int e) {
    const int kk = dB.div(e), b = e - kk * B;
    const float* yp = ws + c.wo.y + rc_y_idx(d, 0, kk * p + j, b);
    const int64_t ys_ = (int64_t)d.Bmax * K * p;
    float v[8];
#pragma unroll
    for (int ub = 0; ub < 8; ++ub) v[ub] = ub < nUB ? yp[ub * ys_] : 0.f;
    float yv = v[0];
#pragma unroll
    for (int ub = 1; ub < 8; ++ub)
      if (ub < nUB) yv += v[ub];
    return yv;
  }, [&](int e, float v) {
    const int kk = dB.div(e);
    ybuf[(e - kk * B) * K + kk] = v;
  });
  __syncthreads();
  float fsum[NV];
#pragma unroll
  for (int vv = 0; vv < NV; ++vv) fsum[vv] = 0.f;
  for (int b = tid, it = 0; b < B; b += NT, ++it) {
    const float* wr = ws + c.wo.w + (int64_t)b * K;
    const bool tgt = c.flags & (RC_LOSS_FORECAST | RC_VALUES);
    const float xt = tgt ? X[((c.row0 + b) * d.T + c.Lmax) * p + j] : 0.f;
    float xs = 0.f;
    for (int kk = 0; kk < K; ++kk) {
      const float we = sig ? rc_sigmoid(ecc * wr[kk]) : wr[kk];
      xs = (kk == 0) ? we * ybuf[b * K + kk] : xs + we * ybuf[b * K + kk];
    }
    const float res = tgt ? xs - xt : 0.f;
    const float wb = sig ? rc_sigmoid(ecc * wr[k]) : wr[k];
    const float g = gscale * res;
    wk[b] = wb;
    dyl[b] = g * wb;
    ws[c.wo.dyl + (int64_t)kj * d.Bmax + b] = g * wb;
    dwf[b] = g * ybuf[b * K + k];
    if (fgrad && !adj_grad) ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k] = dwf[b];
    if (k == 0) {
      fsum[min(it, NV - 1)] += res * res;  // (NT < 256: one window per virtual slot)
      ws[c.wo.xsim + (int64_t)b * p + j] = xs;
    }
  }
  if (values && k == 0) {
    const float t = vsum256(fsum);
    if (tid == 0) ws[c.wo.lossp + j] = t;
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 17);
  // ---- group norms G[kj][c][t], G0[kj][c] (cmlp.py:147-167) from the forward's squared norms
  for (int e = tid; e < Q; e += NT) {
    const float* gp = ws + c.wo.gq + (int64_t)kj * Q + e;
    const int64_t gs_ = (int64_t)K * p * Q;
    float v[8];
#pragma unroll
    for (int ub = 0; ub < 8; ++ub) v[ub] = ub < nUB ? gp[ub * gs_] : 0.f;
    float sq = v[0];
#pragma unroll
    for (int ub = 1; ub < 8; ++ub)
      if (ub < nUB) sq += v[ub];
    sqs[e] = sq;
    Gs[e] = sqrtf(sq);
    ws[c.wo.G + (int64_t)kj * Q + e] = Gs[e];
  }
  __syncthreads();
  for (int cc = tid; cc < p; cc += NT) {
    float sq = 0.f;
    for (int t = 0; t < L; ++t) sq += sqs[cc * L + t];
    ws[c.wo.G0 + (int64_t)kj * p + cc] = sqrtf(sq);
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 18);
  // ---- adjacency L1 of the conditional GC estimate  w_bk G_k[j][c][t] + A[c][j] over the
  // lag slice: pass 1 (thread = window b, half of the channels) gives the value and
  // dL/dw_bk; pass 2 (thread = (c, lag) entry, loop over windows) gives dL/dG (-> ws.dgs) and
  // dL/dA[c][j] (-> ws.dAadj) from one sign evaluation
  const bool adj_on = adj_grad || values;
  if (adj_on) {
    for (int cc = tid; cc < p; cc += NT) Acol[cc] = E[c.eo.A + cc * p + j];
    for (int i = tid; i < Ls; i += NT) lwt[i] = logf((float)(i + 2));
    __syncthreads();
    const int half = tid & 1, hp = (p + 1) / 2, c0 = half * hp, c1 = min(p, c0 + hp);
    // windows in the layout of a 256-thread workgroup (thread vt = vv * NT + tid: window
    // b0 + vt / 2), so the loss value's block sum below keeps one summation order for every NT
    float vsum[NV];
#pragma unroll
    for (int vv = 0; vv < NV; ++vv) vsum[vv] = 0.f;
    for (int b0 = 0; b0 < B; b0 += RC_BLOCK / 2) {
#pragma unroll
      for (int vv = 0; vv < NV; ++vv) {
        const int b = b0 + ((vv * NT + tid) >> 1);
        float t = 0.f, v = 0.f;
        if (b < B) {
          const float wb = wk[b];
          for (int cc = c0; cc < c1; ++cc) {  // this lane's half of the channels
            const float ac = Acol[cc];
            const float* gr = Gs + cc * L + (L - Ls);
#pragma unroll 4
            for (int i = 0; i < Ls; ++i) {
              const float g = gr[i];
              const float val = wb * g + ac;
              t += lwt[i] * rc_sign(val) * g;
              v += lwt[i] * fabsf(val);
            }
          }
        }
        // the two halves of window b are adjacent lanes: combined in fixed order (first + second)
        const float t_hi = __shfl_xor(t, 1), v_hi = __shfl_xor(v, 1);
        if (half == 0 && b < B) {
          if (adj_grad) ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k] = dwf[b] + hy.c_adj * (t + t_hi);
          vsum[vv] += v + v_hi;
        }
      }
    }
    if (values) {  // rc_block_sum's order over the 256-thread layout: wave sums, then the waves in order
      __syncthreads();
#pragma unroll
      for (int vv = 0; vv < NV; ++vv) {
        const float w = rc_wave_sum(vsum[vv]);
        if ((tid & 63) == 0) red[vv * (NT / 64) + (tid >> 6)] = w;
      }
      __syncthreads();
      if (tid == 0) {
        float vs = 0.f;
        for (int i = 0; i < RC_BLOCK / 64; ++i) vs += red[i];
        ws[c.wo.lossp + p + kj] = hy.c_adj * vs;
      }
      __syncthreads();
    }
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 19);
  if (adj_grad) {
    const bool wg = c.flags & RC_STEP_B, ag = c.flags & RC_STEP_A;
    for (int e = tid; e < p * Ls; e += NT) {
      const int cc = e / Ls, i = e - cc * Ls;
      const float g = Gs[cc * L + (L - Ls + i)], ac = Acol[cc];
      float sw = 0.f, s1 = 0.f;
#pragma unroll 8
      for (int b = 0; b < B; ++b) {
        const float sg = rc_sign(wk[b] * g + ac);
        sw += sg * wk[b];
        s1 += sg;
      }
      if (wg) ws[c.wo.dgs + (int64_t)kj * Q + cc * L + (L - Ls + i)] = hy.c_adj * lwt[i] * sw;
      if (ag) dAp[e] = hy.c_adj * lwt[i] * s1;
    }
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 20);
  if (c.flags & RC_STEP_B) {  // dL/dG is zero outside the lag slice (and everywhere without the adj-L1 term)
    for (int q = tid; q < Q; q += NT) {
      const int cc = q / L, tt = q - cc * L;
      if (!adj_grad || tt < L - Ls) ws[c.wo.dgs + (int64_t)kj * Q + q] = 0.f;
    }
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 21);
  if (adj_grad && (c.flags & RC_STEP_A)) {
    __syncthreads();
    for (int cc = tid; cc < p; cc += NT) {
      float s = 0.f;
      for (int i = 0; i < Ls; ++i) s += dAp[cc * Ls + i];
      ws[c.wo.dAadj + ((int64_t)k * p + cc) * p + j] = s;  // d/dA[c][j]
    }
  }
  if (!(c.flags & RC_STEP_B)) {
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_MIX, 1);
    return;
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 22);
  // ---- output layer / hidden bias gradients + Adam: 32 units x 8 batch slices per pass
  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  const float* aw = ws + c.wo.a + (int64_t)kj * d.Bmax * h;
  const float* W1 = ws + c.wo.w1 + (int64_t)kj * h;  // pre-update snapshot written by the forward
  float db1v[NV];
#pragma unroll
  for (int vv = 0; vv < NV; ++vv) db1v[vv] = 0.f;
  for (int b = tid, it = 0; b < B; b += NT, ++it) db1v[min(it, NV - 1)] += dyl[b];
  const float db1 = vsum256(db1v);
  for (int u0 = 0; u0 < ((mf_recompute(d) || NT != RC_BLOCK) ? 0 : h); u0 += 32) {  // else: in k_fac_bwd_mfma<4>
    const int uu = tid & 31, part = tid >> 5, u = u0 + uu;
    float dW1u = 0.f, db0u = 0.f;
    if (u < h) {
      const float w1 = W1[u];
      for (int b = part; b < B; b += 8) {
        const float av = aw[(int64_t)b * h + u];
        dW1u += dyl[b] * av;
        db0u += av > 0.f ? dyl[b] * w1 : 0.f;
      }
    }
    __syncthreads();
    rA[tid] = dW1u;
    rB[tid] = db0u;
    __syncthreads();
    if (tid < 32 && u0 + tid < h) {
      float g1 = 0.f, g0 = 0.f;
      for (int s = 0; s < 8; ++s) {
        g1 += rA[s * 32 + tid];
        g0 += rB[s * 32 + tid];
      }
      rc_update(c, P, PM, PV, GF, c.fo.b0 + (int64_t)kj * h + u0 + tid, g0, as);
      rc_update(c, P, PM, PV, GF, c.fo.W1 + (int64_t)kj * h + u0 + tid, g1, as);
    }
  }
  if (tid == 0) rc_update(c, P, PM, PV, GF, c.fo.b1 + kj, db1, as);
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 23);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_MIX, 1);
}

// ------------------------------------------------------------------------------------------
// dW0 GEMM + adjacency-L1 term + Adam.  NBW column blocks (network kj, 32-unit block ub) per
// workgroup and QT = 256 / NBW dW0 columns: grid (ceil(K*p*nUB/NBW), ceil(Q/QT), R).
// NBW = 2 (long contractions, QT = 128): wave w owns block 2*bx + (w&1) and columns
// [q0 + 64*(w>>1), +64); NBW = 4 (p*L <= 64, QT = 64): wave w owns block 4*bx + w and all 64
// columns -- two 32x32 accumulators either way (rows = the block's hidden units).  The batch is
// the contraction: chunks of 32 windows, dZ built on the fly from dL/dy and the W1 snapshot.
//
// NBW = 4 (mf_recompute): the hidden activations are RECOMPUTED per chunk instead of read back
// from the forward -- the same v_mfma_f32_32x32x2f32 sequence as k_fac_fwd_mfma (windows as rows,
// the block's units as columns, q ascending in steps of 2 over rc_qpad(d), bias, ReLU), so the
// same bits (checked element by element against the stored activations with -DRC_RECOMP_DEBUG)
// -- and this workgroup also forms the output-layer / hidden-bias gradients dW1, db0
// (k_fac_mix's order: per unit, 8 partial sums over windows b = part (mod 8) in ascending order,
// combined in part order) and their Adam step.  The forward then stores no activations and the
// mixing kernel reads none (R = 32 D4IC grid: 3 x 65 MB per step less traffic).
template <int NBW>
__global__ __launch_bounds__(RC_BLOCK) __attribute__((amdgpu_waves_per_eu(NBW == 4 ? RC_FB_WAVES4 : RC_FB_WAVES, 8))) void k_fac_bwd_mfma(StepCtx c) {
  constexpr int QT = 256 / NBW, Q4 = QT / 4;
  constexpr bool RECOMP = NBW == 4;
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.z);
  const int cb0 = blockIdx.x * NBW, q0 = blockIdx.y * QT;
  const int p = d.p, h = d.h, K = d.K, Q = p * d.L, Qp = rc_qpad(d), KP = K * p, B = c.B, nUB = mf_nub(d);
  const int NB = KP * nUB;
  float* P = c.fac + r * c.fs;
  float* PM = c.facM + r * c.fs;
  float* PV = c.facV + r * c.fs;
  float* GF = c.gF + r * c.fs;
  const float* ws = c.ws + r * c.wss;
  const float* Xw = ws + c.wo.xw;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  __shared__ float Zs[NBW][MB_BC][33];  // dZ[blk][b][u]
  __shared__ float Xs[MB_BC][QT + 4];    // Xw[b][q0 + .]
  __shared__ float w1s[NBW * 32];
  __shared__ float Dys[RECOMP ? NBW : 1][MB_BC];  // dL/dy of the chunk's windows (recompute path)

  if (tid < NBW * 32) {
    const int cb = cb0 + (tid >> 5), kj = cb / nUB, u = (cb - kj * nUB) * 32 + (tid & 31);
    w1s[tid] = (cb < NB && u < h) ? ws[c.wo.w1 + (int64_t)kj * h + u] : 0.f;
  }
  // staging maps: dZ NBW x 32 x 32 (4 NBW per thread: blk, b, u) or, recomputing, dL/dy NBW x 32;
  // X 32 x QT (QT / 32 float4 per thread)
  float zr[RECOMP ? 1 : 4 * NBW];
  float4 xr[QT / 32];
  auto load = [&](int bb0) {
    if constexpr (RECOMP) {
      if (tid < NBW * MB_BC) {
        const int cb = cb0 + (tid >> 5), kj = cb / nUB, b = bb0 + (tid & 31);
        zr[0] = (cb < NB && b < B) ? ws[c.wo.dyl + (int64_t)kj * d.Bmax + b] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4 * NBW; ++i) {
        const int e = tid + i * RC_BLOCK, net = e >> 10, bb = (e >> 5) & 31;
        const int cb = cb0 + net, kj = cb / nUB, u = (cb - kj * nUB) * 32 + (e & 31), b = bb0 + bb;
        float v = 0.f;
        if (cb < NB && u < h && b < B) {
          const float av = ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u];
          const float dy = ws[c.wo.dyl + (int64_t)kj * d.Bmax + b];
          v = av > 0.f ? dy : 0.f;
        }
        zr[i] = v;  // times w1[u] at store time
      }
    }
#pragma unroll
    for (int i = 0; i < QT / 32; ++i) {
      const int e = tid + i * RC_BLOCK, bb = e / Q4, c4 = (e % Q4) * 4;
      const int b = bb0 + bb, q = q0 + c4;
      xr[i] = (b < B && q < Qp) ? ld4(Xw + (int64_t)b * Qp + q) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&]() {
    if constexpr (RECOMP) {
      if (tid < NBW * MB_BC) Dys[tid >> 5][tid & 31] = zr[0];
    } else {
#pragma unroll
      for (int i = 0; i < 4 * NBW; ++i) {
        const int e = tid + i * RC_BLOCK, net = e >> 10, bb = (e >> 5) & 31, u = e & 31;
        Zs[net][bb][u] = zr[i] * w1s[net * 32 + u];
      }
    }
#pragma unroll
    for (int i = 0; i < QT / 32; ++i) {
      const int e = tid + i * RC_BLOCK, bb = e / Q4, c4 = (e % Q4) * 4;
      Xs[bb][c4] = xr[i].x;
      Xs[bb][c4 + 1] = xr[i].y;
      Xs[bb][c4 + 2] = xr[i].z;
      Xs[bb][c4 + 3] = xr[i].w;
    }
  };

  // The epilogue's operands (W0, Adam moments, adjacency-L1 terms): RC_FB_PREFETCH=1 loads half
  // 0's before the contraction (latency overlap at 2 waves per SIMD); the default loads them
  // after it, which frees the registers for a third wave (see RC_FB_WAVES).
  const int net = NBW == 2 ? (wv & 1) : wv, qh = NBW == 2 ? 64 * (wv >> 1) : 0, kh = lane >> 5, l31 = lane & 31;
  const int cbw = cb0 + net, kin = cbw < NB;
  const int kj = kin ? cbw / nUB : 0, ub0 = kin ? (cbw - kj * nUB) * 32 : 0;
  const bool adj_grad = (c.flags & RC_LOSS_ADJ) && ((c.flags & RC_STEP_B) || (c.flags & RC_STEP_A));
  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  const bool adam = !(c.flags & RC_GRAD_ONLY);
  float* W0 = P + c.fo.W0 + (int64_t)(kin ? kj : 0) * h * Q;
  float* M0 = PM + c.fo.W0 + (int64_t)(kin ? kj : 0) * h * Q;
  float* V0 = PV + c.fo.W0 + (int64_t)(kin ? kj : 0) * h * Q;
  float* G0w = GF + c.fo.W0 + (int64_t)(kin ? kj : 0) * h * Q;
  // one 32-column half of the lane's outputs at a time: half 0's operands are loaded before
  // the contraction (their latency overlaps the matrix-core work), half 1's after it
  float dg, gn, pw[16], pm[16], pv[16];
  auto epi_load = [&](int half) {
    const int q = q0 + qh + 32 * half + l31;
    const bool qin = kin && q < Q;
    dg = (adj_grad && qin) ? ws[c.wo.dgs + (int64_t)kj * Q + q] : 0.f;
    gn = (adj_grad && qin) ? ws[c.wo.G + (int64_t)kj * Q + q] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int u = ub0 + mf_row(reg, lane);
      const bool in = qin && u < h;
      const int64_t idx = (int64_t)u * Q + q;
      pw[reg] = (in && (adam || adj_grad)) ? W0[idx] : 0.f;
      pm[reg] = (in && adam) ? M0[idx] : 0.f;
      pv[reg] = (in && adam) ? V0[idx] : 0.f;
    }
  };
  auto epi_store = [&](int half, const f32x16& acc) {
    const int q = q0 + qh + 32 * half + l31;
    if (!kin || q >= Q) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int u = ub0 + mf_row(reg, lane);
      if (u >= h) continue;
      const int64_t idx = (int64_t)u * Q + q;
      float g = acc[reg];
      if (adj_grad && gn > 0.f) g += dg * (pw[reg] / gn);
      if (!adam) {
        G0w[idx] = g;
      } else {
        rc_adam(pw[reg], pm[reg], pv[reg], g, as);
        W0[idx] = pw[reg];
        M0[idx] = pm[reg];
        V0[idx] = pv[reg];
      }
    }
  };
#if RC_FB_PREFETCH
  epi_load(0);
#endif

  // recompute path: the lane's layer-0 operand column W0[ub0 + l31][2 kk + kh] (the forward's B
  // operand), its bias, and the partial output-layer gradients of windows b = part (mod 8),
  // part = (reg & 3) + 4 kh (the rows mf_row puts in this lane)
  const int uR = ub0 + l31;
  const bool uvR = RECOMP && kin && uR < h;
  float wB[RECOMP ? 32 : 1], buR = 0.f, w1R = 0.f, pa[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RECOMP) {
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) {
      const int q = 2 * kk + kh;
      wB[kk] = (uvR && q < Q) ? W0[(int64_t)uR * Q + q] : 0.f;
    }
    buR = uvR ? P[c.fo.b0 + (int64_t)kj * h + uR] : 0.f;
  }

  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; }
  load(0);
  for (int bb0 = 0; bb0 < B; bb0 += MB_BC) {
    __syncthreads();
    store();
    __syncthreads();
    if (bb0 + MB_BC < B) load(bb0 + MB_BC);
    if constexpr (RECOMP) {
      // Z[b][u] of this chunk, exactly as k_fac_fwd_mfma forms it
      f32x16 zc;
#pragma unroll
      for (int i = 0; i < 16; ++i) zc[i] = 0.f;
      const int nk = (Q + 1) >> 1;  // the forward's k-steps (up to Q, not the padding to Qp)
#pragma unroll
      for (int kk = 0; kk < 32; ++kk) {
        if (kk < nk) zc = __builtin_amdgcn_mfma_f32_32x32x2f32(Xs[l31][2 * kk + kh], wB[kk], zc, 0, 0, 0);
      }
      w1R = w1s[net * 32 + l31];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int reg = 4 * g4 + m, bl = mf_row(reg, lane), b = bb0 + bl;
          const float a = uvR ? fmaxf(zc[reg] + buR, 0.f) : 0.f;
#ifdef RC_RECOMP_DEBUG
          if (uvR && b < B) {
            const float st = ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + uR];
            if (st != a)
              printf("RECOMP kj=%d b=%d u=%d stored=%.9g recomputed=%.9g z=%.9g bias=%.9g\n", kj, b, uR, st, a,
                     zc[reg], buR);
          }
#endif
          const float dy = Dys[net][bl];
          Zs[net][bl][l31] = (a > 0.f ? dy : 0.f) * w1R;
          if (uvR && b < B) {
            // k_fac_mix's operations exactly: a rounded product added to each running sum (that
            // loop compiles to v_mul + v_pk_add, no fma), db0's product only where a > 0
#pragma clang fp contract(off)
            pa[m] = pa[m] + dy * a;
            pb[m] = pb[m] + (a > 0.f ? dy * w1R : 0.f);
          }
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int k0 = 0; k0 < MB_BC; k0 += 2) {
      const float a = Zs[net][k0 + kh][l31];  // A[i = u][k = b]
      const float x0 = Xs[k0 + kh][qh + l31];  // B[k = b][j = q]
      const float x1 = Xs[k0 + kh][qh + 32 + l31];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, x0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, x1, acc1, 0, 0, 0);
    }
  }
  if constexpr (RECOMP) {
    // dW1[u], db0[u]: parts 0..3 live in lane l31, parts 4..7 in lane l31 + 32; summed in part order
    float hi_a[4], hi_b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      hi_a[m] = __shfl(pa[m], l31 + 32, 64);
      hi_b[m] = __shfl(pb[m], l31 + 32, 64);
    }
    if (kh == 0 && uvR) {
      float g1 = 0.f, g0 = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        g1 += pa[m];
        g0 += pb[m];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        g1 += hi_a[m];
        g0 += hi_b[m];
      }
      rc_update(c, P, PM, PV, GF, c.fo.b0 + (int64_t)kj * h + uR, g0, as);
      rc_update(c, P, PM, PV, GF, c.fo.W1 + (int64_t)kj * h + uR, g1, as);
    }
  }
  // ---- epilogue: + adjacency term through the group norms, then Adam (or store the gradient)
#if !RC_FB_PREFETCH
  epi_load(0);
#endif
  epi_store(0, acc0);
  epi_load(1);
  epi_store(1, acc1);
}

// ------------------------------------------------------------------------------------------
// Short contractions (p*L <= 64, mf_recompute; the D4IC grid): layer 0 forward and backward on
// v_mfma_f32_16x16x4_f32 with 16-UNIT blocks (h = 100 pads to 112 units, not 128).  A workgroup
// stages its replica's batch of windows ONCE in LDS, straight from X (no k_xwin, no Xw round trip):
// window b's columns q = c*L + t start at b*S + ms_sh(b), row stride S = Qp16 + 4 (S = 4 mod 16)
// plus a 2-float shift of rows 8..15 of every 16, so that both operand reads below are
// bank-conflict free (ds_read_b32: lanes 0-31 and 32-63 each hit 32 distinct banks) -- the
// recompute / forward read rows l15 x columns (g, g + 4s) (rows l15 and l15 + 8 would share banks
// without the shift), the dW0 product rows 4g + reg x 16 consecutive columns (4S = 16 mod 32 puts
// g and g + 1 on opposite bank halves);
// then each wave works through `bpw` 16-unit blocks cb = bx * 4 bpw + 4 i + w with no further
// barrier.  Lane l: l15 = l & 15, group g = l >> 4; D rows 4 g + reg, column l15.
//
// The k-step count NK4 = ceil(p*L / 4) is a template parameter (1..16): operand arrays live in
// registers, the row stride is a constant, the loops unroll.  A block's parameters are one
// contiguous run of W0 (its 16 rows of p*L weights), read and written lane-linearly through
// buffer descriptors whose range ends at the last real unit (loads past it return 0, stores past
// it are dropped), so the loads take immediate offsets and no address arithmetic or branches; the
// weights pass through a wave-private LDS tile to the MFMA operand layout, and the backward's
// gradient tile comes back through the same LDS.  The windows' dL/dy of the networks a
// workgroup covers is staged in LDS next to the window tile, so the tile loop touches no global
// memory.  Everything except the address arithmetic is the previous kernels' arithmetic in the
// same order.
//
// The hidden pre-activations are q-ascending k-ordered fmaf chains in both kernels (the forward
// as z[u][b] with W0 rows as the A operand, the backward's recompute as zT[b][u] with the X rows
// as A: a product is commutative), so the backward's recompute reproduces the forward's bits.
// y and the group norms are written per 16-unit block into slots ub < ceil(h/16) (= rc_nuchunk,
// the vector path's hidden chunks; StepCtx.fslots tells k_fac_mix how many to sum).
__host__ __device__ inline int ms_qp16(const RedcliffDims& d) { return ((d.p * d.L + 15) >> 4) << 4; }
__host__ __device__ inline int ms_rows(int B) { return (B + 31) & ~31; }
__host__ __device__ inline int ms_nk4(const RedcliffDims& d) { return (d.p * d.L + 3) >> 2; }
// networks the 4*bpw consecutive blocks of one workgroup can touch
__host__ __device__ inline int ms_nnet(int bpw, int nU) { return (4 * bpw - 1) / nU + 2; }
// per-wave LDS of the backward: the weight / gradient tile (64 NK4 floats) + dL/dG and G rows
// The wave-private weight / gradient tile: 16 rows of Q floats at row stride ms_qs(Q) = Q + 2..9 with
// ms_qs = 4 mod 8 and the same 2-float shift of rows 8..15, so the operand read (rows l15, columns
// g + 4s) and the gradient write (rows 4g + reg, 16 consecutive columns) are conflict-free like Xs;
// the lane-linear store / epilogue read cross rows with at most a few 2-way conflicts.
#ifndef RC_MS_TILE_PAD
#define RC_MS_TILE_PAD 0
#endif
constexpr bool kMsTilePad = RC_MS_TILE_PAD;  // 0: the round-3 linear tile (row stride Q), for A/B
__host__ __device__ inline int ms_qs(int Q) { return Q + 2 + ((2 - Q) & 7); }
__host__ __device__ inline int ms_sh(int row) { return ((row >> 3) & 1) << 1; }
__host__ __device__ inline int ms_tile_floats(int nk4) { return 64 * nk4 + 160; }  // >= 16 ms_qs(Q) + 2, Q <= 4 nk4
__host__ __device__ inline int ms_wave_floats(int nk4) { return ms_tile_floats(nk4) + 128; }
inline size_t ms_lds(const RedcliffDims& d, int B) { return sizeof(float) * (size_t)ms_rows(B) * (ms_qp16(d) + 4); }
inline size_t ms_lds_fwd(const RedcliffDims& d, int B) {
  return ms_lds(d, B) + sizeof(float) * 4 * (size_t)ms_tile_floats(ms_nk4(d));
}
inline size_t ms_lds_bwd(const RedcliffDims& d, int B, int bpw) {
  return ms_lds(d, B) + sizeof(float) * ((size_t)ms_rows(B) * ms_nnet(bpw, (d.h + 15) >> 4) + 4 * (size_t)ms_wave_floats(ms_nk4(d)));
}

template <int NT = RC_BLOCK>
__device__ inline void ms_stage_x(const StepCtx& c, int r, float* Xs) {
  const RedcliffDims& d = c.d;
  const int p = d.p, L = d.L, Q = p * L, Qp16 = ms_qp16(d), S = Qp16 + 4, B = c.B, rows = ms_rows(B);
  const float* src = c.X + r * c.xr + (c.row0 * d.T + (c.Lmax - L)) * p;
  const RcDiv dQ(Q), dp(p);
  rc_stage<8, NT>(B * Q, [&](int e) {
    const int b = dQ.div(e);
    return src[(int64_t)b * d.T * p + (e - b * Q)];
  }, [&](int e, float v) {
    const int b = dQ.div(e), k = e - b * Q, t = dp.div(k), ch = k - t * p;
    Xs[b * S + ms_sh(b) + ch * L + t] = v;
  });
  const int pad = Qp16 - Q;  // zero columns [Q, Qp16) of the batch rows and all of rows [B, rows)
  for (int e = threadIdx.x; e < B * pad; e += NT) {
    const int b = e / pad;
    Xs[b * S + ms_sh(b) + Q + (e - b * pad)] = 0.f;
  }
  for (int e = B * S + threadIdx.x; e < rows * S; e += NT) Xs[e] = 0.f;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Buffer descriptor over n floats from p (built from wave-uniform values): loads at or past the
// end return 0, stores there are dropped.  Offsets in bytes.
#define MS_OOB 0x40000000  // a byte offset past every range
__device__ inline __amdgpu_buffer_rsrc_t ms_rsrc(const float* p, int n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, n * 4, 0x00020000);
}
// (the b32 builtins move raw 32-bit words: bit casts, not conversions)
__device__ inline float ms_ld(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ inline void ms_st(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

// row_ror:N within each 16-lane row (DPP): lane l reads lane (l -/+ N) mod 16 of its row
template <int N>
__device__ inline float ms_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + N, 0xF, 0xF, false));
}
// Sum over the 16 lanes of a row, every lane getting the same bits: the xor-8/4/2/1 butterfly
// (lane l adds lane l^o); after the step with offset o the values repeat with period o, so
// rotating by o reads the same operand as xor o.
__device__ inline float ms_row_sum(float v) {
  v += ms_ror<8>(v);
  v += ms_ror<4>(v);
  v += ms_ror<2>(v);
  v += ms_ror<1>(v);
  return v;
}

// The block's W0 rows (16 x p*L, contiguous; rows past h read as 0) lane-linearly into
// registers: element e = lane + 64 k.
template <int NK4>
__device__ inline void ms_load_tile(__amdgpu_buffer_rsrc_t r, int lane, float (&t)[NK4]) {
#pragma unroll
  for (int k = 0; k < NK4; ++k) t[k] = ms_ld(r, 4 * (lane + 64 * k));
}
// Walk over the lane-linear elements e = lane + 64 k of a block's run: row e / Q, column e % Q,
// advanced incrementally (two live integers, not one address per k); addr() is the tile address
// (-1 for rows past 15, which hold only elements past the run -- never operands)
// The start (lane / Q, lane % Q) goes through an empty asm statement, so the compiler cannot hoist
// the NK4 addresses out of the block loop into NK4 live registers (that cost the backward a wave).
struct MsTileWalk {
  int rw, cl;
  const int Q, Qs, dr, dc;
  __device__ MsTileWalk(int rw0, int cl0, int Q_, int Qs_) : rw(rw0), cl(cl0), Q(Q_), Qs(Qs_), dr(64 / Q_), dc(64 % Q_) {
    asm volatile("" : "+v"(rw), "+v"(cl));
  }
  __device__ inline int addr() const { return rw < 16 ? rw * Qs + ms_sh(rw) + cl : -1; }
  __device__ inline void next() {
    cl += dc;
    rw += dr;
    if (cl >= Q) {
      cl -= Q;
      ++rw;
    }
  }
};
// ... through the wave's LDS tile into the MFMA operand layout: w[s] = W0[u0 + l15][4 s + g]
template <int NK4>
__device__ inline void ms_tile_operands(float* Wt, const float (&t)[NK4], int lane, int l15, int g, int Q, float (&w)[NK4]) {
  const float* row;
  if constexpr (kMsTilePad) {
    const int Qs = ms_qs(Q);
    MsTileWalk tw(lane / Q, lane % Q, Q, Qs);
#pragma unroll
    for (int k = 0; k < NK4; ++k) {
      const int a = tw.addr();
      if (a >= 0) Wt[a] = t[k];
      tw.next();
    }
    row = Wt + l15 * Qs + ms_sh(l15) + g;
  } else {
#pragma unroll
    for (int k = 0; k < NK4; ++k) Wt[lane + 64 * k] = t[k];
    row = Wt + l15 * Q + g;
  }
#pragma unroll
  for (int s = 0; s < NK4; ++s) {
    const float v = row[4 * s];
    w[s] = (s + 1 < NK4 || 4 * s + g < Q) ? v : 0.f;  // only the last k-step can pass Q
  }
}

// Forward: z[u][b] = sum_q W0[u][q] X[b][q] (A = the block's W0 rows in registers, B = Xs rows),
// two 16-window tiles at a time; epilogue a = relu(z + b0), y slot ub = sum_u W1[u] a (in-lane
// over the 4 rows, then the 4 groups in order), + b1 in block 0; group norms of the block; W1
// snapshot for the backward.
template <int NK4>
__global__ __launch_bounds__(RC_BLOCK) void k_fac_fwd_s16(StepCtx c, int bpw, int xcd) {
  constexpr int S = ((NK4 + 3) / 4) * 16 + 4;  // == ms_qp16(d) + 4
  const RedcliffDims& d = c.d;
  int bx = blockIdx.x, bz = blockIdx.z;  // xcd: the replica's workgroups (its window tile) on one XCD
  if (xcd) rc_xcd_order(gridDim.x, gridDim.z, bx, bz);
  const int r = rc_rep(c, bz);
  const int p = d.p, h = d.h, K = d.K, Q = p * d.L, B = c.B, nU = (h + 15) >> 4, NB = K * p * nU, KP = K * p;
  const int rows = ms_rows(B);
  extern __shared__ float Xs[];
  const float* P = c.fac + r * c.fs;
  float* ws = c.ws + r * c.wss;
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_FWD, 0);
  ms_stage_x(c, r, Xs);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* Wt = Xs + rows * S + wv * ms_tile_floats(NK4);
  const int cbase = bx * 4 * bpw + wv;
  // lane offsets of the stores: y of window column l15 (group 0), the W1 snapshot of unit l15
  // (group 0), the group norms of k-step l15 (q = 4 l15 + g)
  const int y_off = g == 0 ? 4 * l15 : MS_OOB;
  const int w1_off = g == 0 ? 4 * l15 : MS_OOB;
  const int gq_off = l15 < NK4 ? 4 * (4 * l15 + g) : MS_OOB;
  // a block's operands: its W0 run (lane-linear), b0 / W1 of rows 4 g + reg, W1 of unit l15, b1;
  // requested one block ahead, so their latency overlaps the previous block's matrix-core work
  struct Ops {
    float wt[NK4], bu[4], w1[4], w1A, b1;
  };
  auto issue = [&](int cb, Ops& o) {
    if (cb >= NB) return;
    const int kj = cb / nU, u0 = (cb - kj * nU) * 16, nu = min(16, h - u0);
    ms_load_tile<NK4>(ms_rsrc(P + c.fo.W0 + ((int64_t)kj * h + u0) * Q, nu * Q), lane, o.wt);
    const auto rB0 = ms_rsrc(P + c.fo.b0 + (int64_t)kj * h + u0, nu);
    const auto rW1 = ms_rsrc(P + c.fo.W1 + (int64_t)kj * h + u0, nu);
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      o.bu[reg] = ms_ld(rB0, 4 * (4 * g + reg));  // 0 past h
      o.w1[reg] = ms_ld(rW1, 4 * (4 * g + reg));
    }
    o.w1A = ms_ld(rW1, 4 * l15);
    o.b1 = P[c.fo.b1 + kj];
  };
  Ops cur, nxt;
  issue(cbase, cur);
  for (int i = 0; i < bpw; ++i) {
    const int cb = cbase + 4 * i;
    if (cb >= NB) break;
    const int kj = cb / nU, ub = cb - kj * nU, u0 = ub * 16;
    const int nu = min(16, h - u0);
    float wA[NK4];
    ms_tile_operands<NK4>(Wt, cur.wt, lane, l15, g, Q, wA);
    issue(cb + 4, nxt);
    const float b1 = ub == 0 ? cur.b1 : 0.f;
    // ---- gq[ub][kj][q] = sum over the block's units of W0[u][q]^2 (pre-update weights); lane
    // (l15, g) stores the sum of k-step s = l15, q = 4 l15 + g
    float gsel = 0.f;
#pragma unroll
    for (int s = 0; s < NK4; ++s) {
      const float sq = ms_row_sum(wA[s] * wA[s]);
      gsel = l15 == s ? sq : gsel;
    }
    ms_st(ms_rsrc(ws + c.wo.gq + ((int64_t)ub * KP + kj) * Q, Q), gq_off, gsel);
    const auto rY = ms_rsrc(ws + c.wo.y + rc_y_idx(d, ub, kj, 0), B);
    for (int t0 = 0; t0 < B; t0 += 32) {
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      const float* x0 = Xs + (t0 + l15) * S + ms_sh(l15) + g;
      const float* x1 = x0 + 16 * S;
#pragma unroll
      for (int s = 0; s < NK4; ++s) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[s], x0[4 * s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[s], x1[4 * s], a1, 0, 0, 0);
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const f32x4 z = tt ? a1 : a0;
        float ys = 0.f;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) ys += cur.w1[reg] * fmaxf(z[reg] + cur.bu[reg], 0.f);  // w1 = 0 past h
        ys += __shfl_xor(ys, 16, 64);
        ys += __shfl_xor(ys, 32, 64);
        ms_st(rY, y_off + 4 * (t0 + 16 * tt), ys + b1);  // window t0 + 16 tt + l15 (dropped at or past B)
      }
    }
    ms_st(ms_rsrc(ws + c.wo.w1 + (int64_t)kj * h + u0, nu), w1_off, cur.w1A);
    cur = nxt;
  }
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_FWD, 1);
}

// Backward (RC_STEP_B): per 16-unit block,
//   recompute  zT[b][u] (A = Xs rows, B = the block's W0 rows in registers; the forward's bits);
//   dZ[b][u] = [relu(z + b0) > 0] dL/dy[b] W1[u] in registers: lane (u = l15, g) holds the windows
//              b = t0 + 4 g + reg of the tile;
//   dW0[u][q] += sum_b dZ[b][u] X[b][q]: k-step `reg` of a tile takes windows t0 + 4 g + reg from
//              lane group g -- the A operand IS the dZ register; B = Xs[t0 + 4 g + reg][16 qt + l15];
//   dW1[u] = sum_b dy a, db0[u] = sum_b [a > 0] dy W1[u]: per lane over its windows, then the four
//              groups in order, and their Adam step;
//   epilogue (lane-linear over the block's W0 run, the gradient tile through LDS): + the
//              adjacency-L1 term through the group norms, Adam (or the gradient).
// A block costs one memory round trip: its W0 run, Adam moments, adjacency rows and output-layer
// state are requested together at its start; dL/dy comes from the workgroup's LDS copy.
// RC_S16_BWD_WAVES: the minimum waves per SIMD the register allocation must allow.  3 (168
// registers, 16 of them spilled to scratch) instead of the compiler's 2 (176 VGPRs + 28 AGPRs): the
// R = 128 grid's k_fac_bwd_s16 200.7-204.5 -> 193.7-196.1 us, whole packed fits bit-identical
// (0 / 27931 arrays, gpurun_out r5m).  0: the compiler's choice.
#ifndef RC_S16_BWD_WAVES
#define RC_S16_BWD_WAVES 3
#endif
// RC_S16_EXP (timing experiments only, wrong results): bit 0 replaces the epilogue's Adam by one
// multiply-add (loads and stores unchanged), bit 1 skips the recompute / dW0 matrix-core passes.
#ifndef RC_S16_EXP
#define RC_S16_EXP 0
#endif
#if RC_S16_BWD_WAVES > 0
#define RC_S16_BWD_BOUNDS __launch_bounds__(RC_BLOCK, RC_S16_BWD_WAVES)
#else
#define RC_S16_BWD_BOUNDS __launch_bounds__(RC_BLOCK)
#endif
template <int NK4>
__global__ RC_S16_BWD_BOUNDS void k_fac_bwd_s16(StepCtx c, int bpw, int xcd) {
  constexpr int S = ((NK4 + 3) / 4) * 16 + 4, NQT = (NK4 + 3) / 4;
  const RedcliffDims& d = c.d;
  int bx = blockIdx.x, bz = blockIdx.z;  // xcd: the replica's workgroups (its window tile) on one XCD
  if (xcd) rc_xcd_order(gridDim.x, gridDim.z, bx, bz);
  const int r = rc_rep(c, bz);
  const int p = d.p, h = d.h, K = d.K, Q = p * d.L, B = c.B, nU = (h + 15) >> 4, NB = K * p * nU;
  const int rows = ms_rows(B);
  extern __shared__ float Xs[];
  float* P = c.fac + r * c.fs;
  float* PM = c.facM + r * c.fs;
  float* PV = c.facV + r * c.fs;
  float* GF = c.gF + r * c.fs;
  const float* ws = c.ws + r * c.wss;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const RcAdamScalars as = rc_adam_scalars(hy.B, c.tB);
  const bool adam = !(c.flags & RC_GRAD_ONLY);
  const bool adj_grad = (c.flags & RC_LOSS_ADJ) && ((c.flags & RC_STEP_B) || (c.flags & RC_STEP_A));
  // the Adam moments are read only when they exist (RC_GRAD_ONLY steps may run without them)
  float* PMr = adam ? PM : P;
  float* PVr = adam ? PV : P;
  const int cb_lo = bx * 4 * bpw, cb_hi = min(NB, cb_lo + 4 * bpw) - 1;
  const int kjlo = cb_lo / nU, nnet = cb_hi / nU - kjlo + 1;
  float* Dys = Xs + rows * S;
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_BWD, 0);
  {  // dL/dy of the workgroup's networks (zero past B), then the window tile
    const RcDiv drow(rows);
    const float* dyg = ws + c.wo.dyl;
    rc_stage<4>(nnet * rows, [&](int e) {
      const int n_ = drow.div(e), b = e - n_ * rows;
      return b < B ? dyg[(int64_t)(kjlo + n_) * d.Bmax + b] : 0.f;
    }, [&](int e, float v) { Dys[e] = v; });
  }
  ms_stage_x(c, r, Xs);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* Wt = Dys + ms_nnet(bpw, nU) * rows + wv * ms_wave_floats(NK4);  // weight, then gradient tile
  float* Dg = Wt + ms_tile_floats(NK4);  // dL/dG row of the network (adjacency L1), then its group norms G
  float* Gn = Dg + 64;
  const int u_off = g == 0 ? 4 * l15 : MS_OOB;  // output-layer updates: group 0, unit l15
  // lane-linear epilogue elements e = lane + 64 k of the block's run: column q = e % Q
  const int q0 = lane % Q, dq = 64 % Q;
  // the recompute operands of a block (its W0 run, b0 and the W1 snapshot of unit l15), requested
  // one block ahead so their latency overlaps the previous block's matrix-core work
  struct Ops {
    float wt[NK4], bu, w1;
  };
  auto issue = [&](int cb, Ops& o) {
    if (cb >= NB) return;
    const int kj = cb / nU, u0 = (cb - kj * nU) * 16, nu = min(16, h - u0);
    ms_load_tile<NK4>(ms_rsrc(P + c.fo.W0 + ((int64_t)kj * h + u0) * Q, nu * Q), lane, o.wt);
    o.bu = ms_ld(ms_rsrc(P + c.fo.b0 + (int64_t)kj * h + u0, nu), 4 * l15);              // 0 past h
    o.w1 = ms_ld(ms_rsrc(ws + c.wo.w1 + (int64_t)kj * h + u0, nu), 4 * l15);             // pre-update snapshot
  };
  Ops cur, nxt;
  issue(cb_lo + wv, cur);
  for (int i = 0; i < bpw; ++i) {
    const int cb = cb_lo + 4 * i + wv;
    if (cb >= NB) break;
    const int kj = cb / nU, u0 = (cb - kj * nU) * 16;
    const int nu = min(16, h - u0);
    const int64_t wofs = c.fo.W0 + ((int64_t)kj * h + u0) * Q;
    const auto rW = ms_rsrc(P + wofs, nu * Q);
    const auto rB0 = ms_rsrc(P + c.fo.b0 + (int64_t)kj * h + u0, nu);
    const auto rW1 = ms_rsrc(P + c.fo.W1 + (int64_t)kj * h + u0, nu);
    float wB[NK4], mt[NK4], vt[NK4];
    ms_tile_operands<NK4>(Wt, cur.wt, lane, l15, g, Q, wB);
    // this block's epilogue operands (Adam moments of the run, adjacency rows, output-layer
    // state), then the next block's recompute operands: issue order = arrival order
    ms_load_tile<NK4>(ms_rsrc(PMr + wofs, nu * Q), lane, mt);
    ms_load_tile<NK4>(ms_rsrc(PVr + wofs, nu * Q), lane, vt);
    const float dgv = ms_ld(ms_rsrc(ws + c.wo.dgs + (int64_t)kj * Q, Q), 4 * lane);
    const float gnv = ms_ld(ms_rsrc(ws + c.wo.G + (int64_t)kj * Q, Q), 4 * lane);
    const auto rMb = ms_rsrc(PMr + c.fo.b0 + (int64_t)kj * h + u0, nu), rVb = ms_rsrc(PVr + c.fo.b0 + (int64_t)kj * h + u0, nu);
    const auto rMw = ms_rsrc(PMr + c.fo.W1 + (int64_t)kj * h + u0, nu), rVw = ms_rsrc(PVr + c.fo.W1 + (int64_t)kj * h + u0, nu);
    float sb[6] = {cur.bu, ms_ld(rMb, 4 * l15), ms_ld(rVb, 4 * l15), ms_ld(rW1, 4 * l15), ms_ld(rMw, 4 * l15), ms_ld(rVw, 4 * l15)};
    issue(cb + 4, nxt);
    const float bu = cur.bu, w1 = cur.w1;  // 0 past h
    f32x4 acc[NQT];
#pragma unroll
    for (int t = 0; t < NQT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float pa = 0.f, pb = 0.f;
    const float* dyn = Dys + (kj - kjlo) * rows + 4 * g;
    // two 16-window tiles per pass (independent recompute chains); rows past B are zero windows
    // with zero dL/dy, which add exact zeros, and the tile pairs run to a multiple of 32 <= rows
    for (int t0 = 0; t0 < ((RC_S16_EXP & 2) ? 0 : B); t0 += 32) {
      f32x4 z[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      const float* xr = Xs + (t0 + l15) * S + ms_sh(l15) + g;
#pragma unroll
      for (int s = 0; s < NK4; ++s) {
        z[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[4 * s], wB[s], z[0], 0, 0, 0);
        z[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[16 * S + 4 * s], wB[s], z[1], 0, 0, 0);
      }
      float dz[2][4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const f32x4 dy = *reinterpret_cast<const f32x4*>(dyn + t0 + 16 * tt);  // windows t0 + 16 tt + 4 g + reg
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
#pragma clang fp contract(off)
          const float a = fmaxf(z[tt][reg] + bu, 0.f);
          // dZ = [a > 0] dL/dy W1; the output-layer sums take the same rounded product (a zero
          // dZ adds nothing whatever its sign)
          dz[tt][reg] = a > 0.f ? dy[reg] * w1 : 0.f;
          pa = pa + dy[reg] * a;
          pb = pb + dz[tt][reg];
        }
      }
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const float* xq = Xs + (t0 + 16 * tt + 4 * g) * S + ms_sh(4 * g) + l15;  // rows 4g + reg: shift of row 4g
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt)
            acc[qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(dz[tt][reg], xq[reg * S + 16 * qt], acc[qt], 0, 0, 0);
      }
    }
    {  // output layer / hidden bias of the lane's unit: the four groups' partial sums in order
      const float a1 = __shfl(pa, l15 + 16, 64), a2 = __shfl(pa, l15 + 32, 64), a3 = __shfl(pa, l15 + 48, 64);
      const float b1 = __shfl(pb, l15 + 16, 64), b2 = __shfl(pb, l15 + 32, 64), b3 = __shfl(pb, l15 + 48, 64);
      const float g0 = ((pb + b1) + b2) + b3, g1 = ((pa + a1) + a2) + a3;
      if (!adam) {  // group 0 stores, rows past h dropped
        ms_st(ms_rsrc(GF + c.fo.b0 + (int64_t)kj * h + u0, nu), u_off, g0);
        ms_st(ms_rsrc(GF + c.fo.W1 + (int64_t)kj * h + u0, nu), u_off, g1);
      } else {
        rc_adam(sb[0], sb[1], sb[2], g0, as);
        rc_adam(sb[3], sb[4], sb[5], g1, as);
        ms_st(rB0, u_off, sb[0]);
        ms_st(rMb, u_off, sb[1]);
        ms_st(rVb, u_off, sb[2]);
        ms_st(rW1, u_off, sb[3]);
        ms_st(rMw, u_off, sb[4]);
        ms_st(rVw, u_off, sb[5]);
      }
    }
    // ---- gradient tile (the tile layout) into the wave's LDS tile: the weight operands were read
    // from it before the tile loop; the pre-update weights stay in cur.wt
    Dg[lane] = dgv;
    Gn[lane] = gnv;
    const int Qs = kMsTilePad ? ms_qs(Q) : Q, sh4g = kMsTilePad ? ms_sh(4 * g) : 0;
#pragma unroll
    for (int qt = 0; qt < NQT; ++qt) {
      const int q = 16 * qt + l15;
      if (qt + 1 < NQT || q < Q)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) Wt[(4 * g + reg) * Qs + sh4g + q] = acc[qt][reg];
    }
    MsTileWalk tw(lane / Q, lane % Q, Q, Qs);
    // ---- epilogue, lane-linear: + the adjacency term through the group norms, then Adam (or the
    // gradient); elements past the block's run are computed on zeros and their stores dropped
    const auto rM = ms_rsrc(PMr + wofs, nu * Q), rV = ms_rsrc(PVr + wofs, nu * Q), rG = ms_rsrc(GF + wofs, nu * Q);
    int q = q0;
#pragma unroll
    for (int k = 0; k < NK4; ++k) {
      const int e = lane + 64 * k;  // gradient tile element (row e / Q, column q = e % Q)
      float gr;
      if constexpr (kMsTilePad) {
        const int ta = tw.addr();
        tw.next();
        gr = Wt[ta >= 0 ? ta : 0];  // rows past 15: past the run, the stores are dropped
      } else {
        gr = Wt[e];
      }
      const float dg = Dg[q], gn = Gn[q], pw = cur.wt[k];
      if (adj_grad && gn > 0.f) gr += dg * (pw / gn);
      if (!adam) {
        ms_st(rG, 4 * e, gr);
      } else {
        float pp = pw, mm = mt[k], vv = vt[k];
        if constexpr ((RC_S16_EXP & 1) != 0)
          pp = fmaf(-1e-3f, gr, pp);
        else
          rc_adam(pp, mm, vv, gr, as);
        ms_st(rW, 4 * e, pp);
        ms_st(rM, 4 * e, mm);
        ms_st(rV, 4 * e, vv);
      }
      q += dq;
      q = q >= Q ? q - Q : q;
    }
    cur = nxt;
  }
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_BWD, 1);
}

// k_fac_mix's workgroup threads where it may be narrower than 256 (64 / 128)
#ifndef RC_MIX_NT
#define RC_MIX_NT 128
#endif
// k_fac_mix's workgroup: 128 threads when B <= 128 (one window per thread, so the per-thread
// window sums and the block sums of the loss value and the output-bias gradient see the same
// operands in the same order as at 256 threads, whose upper waves held zeros) and the hidden-layer
// gradients come from the dW0 kernel (mf_recompute: the 32-units-by-8-slices pass is not run).
static int fac_mix_nt(const RedcliffDims& d, int B) {
  const char* v = getenv("REDCLIFF_MIX_NT");  // read per launch (A/B)
  const int want = v ? atoi(v) : RC_MIX_NT;
  if (!(B <= 128 && mf_recompute(d))) return RC_BLOCK;
  return want == 64 || want == 128 ? want : RC_BLOCK;
}

size_t fac_mix_lds(const RedcliffDims& d, int Ls) {
  const int Q = d.p * d.L;
  return sizeof(float) * (size_t)(2 * d.Bmax + 2 * Q + d.p + d.L + 16 + d.p * Ls + d.Bmax * d.K + 2 * RC_BLOCK + d.Bmax);
}

}  // namespace

// Path choice: the matrix-core path (32-unit hidden blocks, h <= 128) pays off once the
// contraction is long (the stress config) or many replicas share the launch (packed grid
// search: D4IC R = 32 runs 4.2 M -> 5.5 M windows/s, while a single D4IC fit is faster on the
// latency-shaped vector kernels, 1.31 M vs 0.92 M).  REDCLIFF_FAC_PATH=mfma|vector overrides
// (tests, tuning).
bool rc_fac_vector_fits(const RedcliffDims& d);  // rc_factor.hip

bool rc_fac_use_mfma(const RedcliffDims& d) {
  const char* v = getenv("REDCLIFF_FAC_PATH");  // read per call: tests switch paths in-process
  const int env = !v ? 0 : (!strcmp(v, "mfma") ? 1 : (!strcmp(v, "vector") ? 2 : 0));
  if (d.h > 128) return false;
  if (env == 1) return true;
  if (env == 2) return false;
  return (d.p * d.L >= 256 && d.h <= 32) || d.R >= 8 || !rc_fac_vector_fits(d);
}

// Short-contraction kernels (k_fac_fwd_s16 / k_fac_bwd_s16) for p*L <= 64; REDCLIFF_FAC_SHORT=0
// runs the 32-unit tiled kernels there instead (tuning, A/B).  Read per call like the path choice.
bool rc_fac_short(const RedcliffDims& d) {
  const char* v = getenv("REDCLIFF_FAC_SHORT");
  return mf_recompute(d) && !(v && !strcmp(v, "0"));
}
// y / group-norm slots the forward writes (k_fac_mix sums them): 16- or 32-unit blocks
int rc_fac_slots(const RedcliffDims& d) { return rc_fac_short(d) ? (d.h + 15) / 16 : mf_nub(d); }

// Launch of the short-contraction kernels: the k-step count picks the instantiation, and the
// blocks per wave are chosen from the resident workgroups (the occupancy the runtime computes
// from the kernel's registers and this launch's LDS, times the CUs).  REDCLIFF_FAC_BPW=n (backward) /
// REDCLIFF_FAC_BPW_FWD=n (forward) override.
typedef void (*MsKern)(StepCtx, int, int);
template <int N>
struct MsTab {
  static void fill(MsKern* f, MsKern* b) {
    f[N - 1] = k_fac_fwd_s16<N>;
    b[N - 1] = k_fac_bwd_s16<N>;
    MsTab<N - 1>::fill(f, b);
  }
};
template <>
struct MsTab<0> {
  static void fill(MsKern*, MsKern*) {}
};

static int ms_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return v;
  }();
  return n;
}

static int ms_occupancy(MsKern k, size_t lds) {
  struct Ent { MsKern k; size_t lds; int occ; };
  static thread_local Ent cache[32];
  static thread_local int n = 0;
  for (int i = 0; i < n; ++i)
    if (cache[i].k == k && cache[i].lds == lds) return cache[i].occ;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, RC_BLOCK, lds) != hipSuccess) nb = 0;
  cache[n < 32 ? n++ : 31] = Ent{k, lds, nb};
  return nb;
}

static int ms_launch(bool bwd, const StepCtx& c, hipStream_t s) {
  static MsKern tf[16], tb[16];
  static const bool init = (MsTab<16>::fill(tf, tb), true);
  (void)init;
  const RedcliffDims& d = c.d;
  const char* what = bwd ? "k_fac_bwd_s16" : "k_fac_fwd_s16";
  const int nk4 = ms_nk4(d);
  if (nk4 < 1 || nk4 > 16) { rc_set_error("%s: p*L = %d outside the short-contraction kernels", what, d.p * d.L); return REDCLIFF_ELIMIT; }
  MsKern k = bwd ? tb[nk4 - 1] : tf[nk4 - 1];
  const int NB = d.K * d.p * ((d.h + 15) / 16);
  const size_t cap = RC_LDS_MAX_FLOATS * sizeof(float);
  size_t lds = bwd ? ms_lds_bwd(d, c.B, 1) : ms_lds_fwd(d, c.B);
  if (lds > cap) { rc_set_error("%s: %d windows do not fit in LDS", what, c.B); return REDCLIFF_ELIMIT; }
  int bpw = 1;
  const char* env = getenv(bwd ? "REDCLIFF_FAC_BPW" : "REDCLIFF_FAC_BPW_FWD");
  if (env && atoi(env) > 0) {
    bpw = atoi(env);
  } else {
    static bool optin[2][16];
    if (!optin[bwd][nk4 - 1]) {  // the occupancy query of a launch past 64 KiB needs the opt-in
      const int e = rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)cap), what);
      if (e) return e;
      optin[bwd][nk4 - 1] = true;
    }
    const int64_t slots = (int64_t)ms_occupancy(k, lds) * ms_cus();
    if (slots > 0) {
      // the backward as one round of resident workgroups, the forward (short blocks, a staging
      // prologue per workgroup) as about two: R = 128 D4IC grid, bpw 4 / 8 / 16 -> forward 114 /
      // 140 / 145 us, backward 228 / 236 / 266 us against 205 us at one round (12)
      const int64_t rounds = bwd ? 1 : 2;
      const int64_t blocks = (int64_t)NB * c.nrep, want = (blocks + 4 * rounds * slots - 1) / (4 * rounds * slots);
      bpw = (int)(want < 1 ? 1 : (want > 16 ? 16 : want));
    }
  }
  if (bwd)
    while (bpw > 1 && ms_lds_bwd(d, c.B, bpw) > cap) --bpw;
  if (bwd) lds = ms_lds_bwd(d, c.B, bpw);
  if (lds > cap) { rc_set_error("%s: %d windows do not fit in LDS", what, c.B); return REDCLIFF_ELIMIT; }
  if (lds > RC_LDS_LIMIT_FLOATS * sizeof(float)) {
    const int e = rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), what);
    if (e) return e;
  }
  const char* xe = getenv("REDCLIFF_S16_XCD");  // read per launch (A/B); default on
  hipLaunchKernelGGL(k, dim3((NB + 4 * bpw - 1) / (4 * bpw), 1, c.nrep), dim3(RC_BLOCK), lds, s, c, bpw, (int)!(xe && xe[0] == '0'));
  return rc_check(hipGetLastError(), what);
}

int rc_launch_fac_fwd_mfma(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  if (c.fslots != rc_fac_slots(d)) { rc_set_error("factor forward: slot layout changed within a step"); return REDCLIFF_EINVAL; }
  if (rc_fac_short(d)) return ms_launch(false, c, s);
  const int KP = d.K * d.p;
  const int nxw = (c.B * rc_qpad(d) + XW_PER * RC_BLOCK - 1) / (XW_PER * RC_BLOCK);
  hipLaunchKernelGGL(k_xwin, dim3(nxw, c.nrep), dim3(RC_BLOCK), 0, s, c);
  int e = rc_check(hipGetLastError(), "k_xwin");
  if (e) return e;
  const int NB = KP * ((d.h + 31) / 32);
  hipLaunchKernelGGL(k_fac_fwd_mfma, dim3((NB + 1) / 2, (c.B + MF_BT - 1) / MF_BT, c.nrep), dim3(RC_BLOCK), 0, s, c);
  return rc_check(hipGetLastError(), "k_fac_fwd_mfma");
}

int rc_launch_fac_mix(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int KP = d.K * d.p;
  const size_t lds = fac_mix_lds(d, c.Ls);
  if (lds > RC_LDS_LIMIT_FLOATS * sizeof(float)) { rc_set_error("factor mixing: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  const char* xe = getenv("REDCLIFF_MIX_XCD");  // read per launch (A/B); default on
  // 128-thread workgroups where every window has its own thread and the output-layer sums run in
  // the dW0 kernel: twice the resident workgroups for a kernel whose time is its workgroups'
  // chains of dependent memory rounds, the same bits (every sum keeps its order: fac_mix_nt).
  // REDCLIFF_MIX_NT=256 keeps the full workgroups (A/B).
  const int nt = fac_mix_nt(d, c.B);
  if (nt == 64)
    hipLaunchKernelGGL(k_fac_mix<64>, dim3(KP, c.nrep), dim3(64), lds, s, c, (int)!(xe && xe[0] == '0'));
  else if (nt == 128)
    hipLaunchKernelGGL(k_fac_mix<128>, dim3(KP, c.nrep), dim3(128), lds, s, c, (int)!(xe && xe[0] == '0'));
  else
    hipLaunchKernelGGL(k_fac_mix<RC_BLOCK>, dim3(KP, c.nrep), dim3(RC_BLOCK), lds, s, c, (int)!(xe && xe[0] == '0'));
  return rc_check(hipGetLastError(), "k_fac_mix");
}

int rc_launch_fac_dw0(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  if (!(c.flags & RC_STEP_B)) return 0;
  const int NB = d.K * d.p * ((d.h + 31) / 32), Q = d.p * d.L;
  if (rc_fac_short(d)) return ms_launch(true, c, s);
  if (Q <= 64)  // short contraction rows: four column blocks share one 64-column X tile
    hipLaunchKernelGGL(k_fac_bwd_mfma<4>, dim3((NB + 3) / 4, 1, c.nrep), dim3(RC_BLOCK), 0, s, c);
  else
    hipLaunchKernelGGL(k_fac_bwd_mfma<2>, dim3((NB + 1) / 2, (Q + 127) / 128, c.nrep), dim3(RC_BLOCK), 0, s, c);
  return rc_check(hipGetLastError(), "k_fac_bwd_mfma");
}
