// rc_embed_gemm.hip -- the DGCNN factor-score embedder as a chain of GEMMs, for large node
// counts / feature windows (the stress config p=64, F=64: p*F = 4096 per window), where the
// per-window workgroups of rc_forward.hip / rc_embed.hip would re-read every window once per
// (node, column chunk) block and run out of LDS.
//
// Reference: models/redcliff_factor_score_embedders.py:335-392, models/dgcnn.py:15-64 and the
// torcheeg 1.1.3 DGCNN (restated in oracle/torcheeg_dgcnn.py).  Layout: T[b][c][i][f]
// (T_0 = x_bn), so the graph convolution over all windows and nodes is ONE product
//   Z[(b,c)][h] = sum_{(i,f)} T[(b,c)][(i,f)] gcW[(i,f)][h]      (B*p x n*F x H)
// because the packed graph-conv weights gcW[n][F][H] are exactly that (n*F) x H matrix.
//
// forward:  prep (x_bn)  ->  T_i = S_i x_bn (per window, i >= 1)  ->  R = relu(T gcW)
//           ->  fc1 split-K partials  ->  head (f1, relu, fc2 -> w)
// backward: dhead (dL/dw_raw, dL/df1, fc2 / fc1-bias gradients)  ->  dfc1W = df1^T R
//           ->  dZ = [R > 0] df1 fc1W  ->  dW = T^T dZ (p split-K slices, summed by the final
//           kernel)  ->  dT = dZ gcW^T  ->  dx_bn = sum_i S_i^T dT_i  ->  dS_i = sum_b dT_i x_bn^T
//           (window-group slices)  ->  BatchNorm affine partials.  The final kernel (rc_embed.hip,
//           k_emb_final) applies Adam, the Chebyshev / normalize_A backward and the BN running stats.
// The window-sized products of small node counts (p < 32: T_i, dx_bn, dS_i, BN partials) run in
// the windowed kernels k_lemb_prep_win / k_lemb_win_bwd instead; every other contraction is the
// shared GEMM core (rc_gemm.h), one launch per product for all replicas.
#include <cstdlib>
#include <cstring>

#include "rc_gemm.h"

namespace {

// windows per k_lemb_dhead workgroup: 64 (window, factor) items of 4 lanes each (K <= 16)
__host__ __device__ inline int lemb_wpw(const RedcliffDims& d) { return 64 / d.K; }
// k_lemb_dhead: fc2W (via LDS), f1, w and the labels requested before the dL/dw sums (1) or where used (0)
#ifndef RC_DHEAD_EARLY
#define RC_DHEAD_EARLY 1
#endif

// x_bn[b][c][0][f] = X[row0 + b][Lmax - F + f][c] * alpha_f + beta_f    grid (B, R)
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_prep(StepCtx c) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), b = blockIdx.x;
  const int p = d.p, F = d.F, n = d.n;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr + ((c.row0 + b) * d.T + (c.Lmax - F)) * p;
  __shared__ float alpha[64], beta[64];
  const int tid = threadIdx.x;
  if (tid < F) {
    const bool train = c.flags & RC_BN_TRAIN;
    float mean, inv;
    if (train) {
      mean = (float)c.bns[r * c.bnsr + tid];
      inv = (float)(1.0 / sqrt(c.bns[r * c.bnsr + F + tid] + c.hyp[r].bn_eps));
    } else {
      mean = c.rm[r * F + tid];
      inv = 1.0f / sqrtf(c.rv[r * F + tid] + (float)c.hyp[r].bn_eps);
    }
    const float a = inv * E[c.eo.bnw + tid];
    alpha[tid] = a;
    beta[tid] = E[c.eo.bnb + tid] - mean * a;
  }
  __syncthreads();
  float* T = ws + c.wo.T + (int64_t)b * p * n * F;
  const RcDiv dp(p);
  // read (f, c) contiguous, write [c][0][f]; every load of a round issued before its stores
  for (int e0 = 0; e0 < p * F; e0 += 16 * RC_BLOCK) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = e0 + u * RC_BLOCK + tid;
      v[u] = e < p * F ? X[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = e0 + u * RC_BLOCK + tid;
      if (e < p * F) {
        const int f = dp.div(e), ch = e - f * p;
        T[(int64_t)ch * n * F + f] = v[u] * alpha[f] + beta[f];
      }
    }
  }
}

// f1 = sum of the split-K partials + bias; w = fc2(relu(f1)).  grid (ceil(B / 4), R): one window
// per wave, lane m sums the partials in 4 interleaved chains, combined in fixed order; lane k forms
// w[k] from the wave's relu(f1) (no LDS, no barrier).  Every load is issued before the first use:
// the partials four at a time (clamped indices, no branch per load) and lane k's fc2 row into
// registers 32 terms at a time; relu(f1[m]) is read with v_readlane.  (The previous form -- a branch per partial and a
// global load per fc2 term inside the chain -- compiled to 68 serial load round trips per wave.)
// W windows per wave (grid (ceil(B / (4 W)), R)): a packed grid's one-window waves are too short to
// cover their dispatch, so each wave takes W windows, their loads requested together and their
// chains interleaved (every window keeps its own summation order: the same bits for any W).
template <int W>
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_head(StepCtx c, int nsplit) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), lane = threadIdx.x & 63;
  const int bw = (blockIdx.x * 4 + (threadIdx.x >> 6)) * W;  // the wave's first window
  if (bw >= c.B) return;
  const int M1 = d.M1, K = d.K;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const int ml = lane < M1 ? lane : M1 - 1;
  const float* part = ws + c.wo.f1p + ml;
  const int64_t pst = (int64_t)d.Bmax * M1;
  int bo[W];  // window offsets of the partials (windows past B read the last one and do not store)
#pragma unroll
  for (int w = 0; w < W; ++w) bo[w] = min(bw + w, c.B - 1) * M1;
  // lane k's fc2 row (lanes >= K read row 0 and do not store), 32 terms per round of loads
  const float* w2 = E + c.eo.fc2W + (lane < K ? lane : 0) * M1;
  float w2r[32];
#pragma unroll
  for (int u = 0; u < 32; ++u) w2r[u] = w2[min(u, M1 - 1)];
  const float fb1 = E[c.eo.fc1b + ml];
  float t4[W][4];
#pragma unroll
  for (int w = 0; w < W; ++w) t4[w][0] = t4[w][1] = t4[w][2] = t4[w][3] = 0.f;
  for (int q0 = 0; q0 < nsplit; q0 += 4) {  // nsplit <= 64; t4[q & 3] += partial q, q ascending
    float v[W][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t qo = (int64_t)min(q0 + u, nsplit - 1) * pst;
#pragma unroll
      for (int w = 0; w < W; ++w) v[w][u] = part[qo + bo[w]];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (q0 + u < nsplit) {
#pragma unroll
        for (int w = 0; w < W; ++w) t4[w][u] += v[w][u];
      }
  }
  float rv[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    float v = 0.f;
    if (lane < M1) {
      v = ((t4[w][0] + t4[w][1]) + (t4[w][2] + t4[w][3])) + fb1;
      if (bw + w < c.B) ws[c.wo.f1 + (int64_t)(bw + w) * M1 + lane] = v;
    }
    rv[w] = fmaxf(v, 0.f);
  }
  // w[k] = fc2b[k] + sum_m fc2W[k][m] relu(f1[m]), m ascending
  float a[W];
#pragma unroll
  for (int w = 0; w < W; ++w) a[w] = 0.f;
  for (int m0 = 0; m0 < M1; m0 += 32) {  // M1 <= 64
    if (m0 > 0) {
#pragma unroll
      for (int u = 0; u < 32; ++u) w2r[u] = w2[min(m0 + u, M1 - 1)];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (m0 + u < M1) {
#pragma unroll
        for (int w = 0; w < W; ++w)
          a[w] = fmaf(w2r[u], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rv[w]), m0 + u)), a[w]);
      }
  }
  if (lane < K) {
    const float b2 = E[c.eo.fc2b + lane];
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (bw + w < c.B) ws[c.wo.w + (int64_t)(bw + w) * K + lane] = a[w] + b2;
  }
}

// grid (ceil(B / WPW), R), WPW = 64 / K windows per workgroup: lanes (item = (window, k), g),
// g sums every 4th channel partial of the factor-side dL/dw (all loads in flight); then dL/df1
// of the workgroup's windows.  dr -> ws.edr, df1 -> ws.edf1.
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_dhead(StepCtx c) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y);
  const int K = d.K, M1 = d.M1, p = d.p, B = c.B;
  const int WPW = lemb_wpw(d), b0 = blockIdx.x * WPW;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  __shared__ float drs[64];
  const int tid = threadIdx.x, item = tid >> 2, g = tid & 3;
  const int s = item / K, k = item - s * K, b = b0 + s;
  const bool ok = item < WPW * K && b < B;
  const bool fac_grad = c.flags & (RC_LOSS_FORECAST | RC_LOSS_ADJ);
  const bool lab_on = (c.flags & RC_LOSS_FACTOR) && d.nsup > 0;
  const float* f1 = ws + c.wo.f1;
#if RC_DHEAD_EARLY
  // everything the workgroup reads that does not depend on dL/dw is requested up front: fc2W
  // (K x M1 <= 1024 floats) into LDS, the first four dL/df1 elements' f1 values, and the items'
  // w / label values -- the dL/dw partial sums below then overlap them
  __shared__ float w2s[1024];
  for (int e = tid; e < K * M1; e += RC_BLOCK) w2s[e] = E[c.eo.fc2W + e];
  float f1p[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * RC_BLOCK, sw = e / M1, bb = min(b0 + sw, B - 1);
    f1p[u] = e < WPW * M1 ? f1[(int64_t)bb * M1 + (e - sw * M1)] : 0.f;
  }
  const float wv = ok ? ws[c.wo.w + (int64_t)b * K + k] : 0.f;
  const float yv = (ok && lab_on) ? c.lab[r * c.labr + (c.row0 + b) * K + k] : 0.f;
#endif
  float t = 0.f;
  if (ok && fac_grad) {
    // four loads in flight at a time (clamped channel indices, no branch per load), added in j order
    const float* dw = ws + c.wo.dwp + (int64_t)b * K + k;
    const int nu = (p + 3) >> 2;  // p <= 64
    for (int u0 = 0; u0 < nu; u0 += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = dw[(int64_t)min(g + 4 * (u0 + u), p - 1) * d.Bmax * K];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (g + 4 * (u0 + u) < p) t += v[u];
    }
  }
  t += __shfl_xor(t, 1);
  t += __shfl_xor(t, 2);
  if (ok && g == 0) {
#if RC_DHEAD_EARLY
    const float v = rc_emb_draw(c, r, k, wv, t, yv);
#else
    const float y = lab_on ? c.lab[r * c.labr + (c.row0 + b) * K + k] : 0.f;
    const float v = rc_emb_draw(c, r, k, ws[c.wo.w + (int64_t)b * K + k], t, y);
#endif
    drs[item] = v;
    ws[c.wo.edr + (int64_t)b * K + k] = v;
  }
  __syncthreads();
  float* df1 = ws + c.wo.edf1;
#if RC_DHEAD_EARLY
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * RC_BLOCK, sw = e / M1, m = e - sw * M1, bb = b0 + sw;
    if (e >= WPW * M1 || bb >= B) continue;
    float gg = 0.f;
    if (f1p[u] > 0.f) {
      for (int kk = 0; kk < K; ++kk) gg += drs[sw * K + kk] * w2s[kk * M1 + m];
    }
    df1[(int64_t)bb * M1 + m] = gg;
  }
  for (int e = tid + 4 * RC_BLOCK; e < WPW * M1; e += RC_BLOCK) {
    const int sw = e / M1, m = e - sw * M1, bb = b0 + sw;
    if (bb >= B) continue;
    float gg = 0.f;
    if (f1[(int64_t)bb * M1 + m] > 0.f) {
      for (int kk = 0; kk < K; ++kk) gg += drs[sw * K + kk] * w2s[kk * M1 + m];
    }
    df1[(int64_t)bb * M1 + m] = gg;
  }
#else
  for (int e = tid; e < WPW * M1; e += RC_BLOCK) {
    const int sw = e / M1, m = e - sw * M1, bb = b0 + sw;
    if (bb >= B) continue;
    float w2[16];  // K <= 16: fc2W[.][m] requested together, not once per term of the chain
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) w2[kk] = E[c.eo.fc2W + min(kk, K - 1) * M1 + m];
    float gg = 0.f;
    if (f1[(int64_t)bb * M1 + m] > 0.f) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        if (kk < K) gg += drs[sw * K + kk] * w2[kk];
    }
    df1[(int64_t)bb * M1 + m] = gg;
  }
#endif
}

// Workgroups [0, ngfc): fc2 weight / fc2 bias / fc1 bias gradients, 64 outputs per workgroup,
// lanes (output, g) over every 4th window, fixed-order combine:
//   dfc2W[k][m] = sum_b dr[b][k] relu(f1[b][m]); dfc2b[k] = sum_b dr[b][k]; dfc1b[m] = sum_b df1[b][m]
// Workgroups [ngfc, ...): Af[c][c'*n + i] = S_i[c'][c] ([S_0^T | S_1^T | ...] interleaved, for
// dx_bn = sum_i S_i^T dT_i).  grid (ngfc + ceil(p*p*n / 256), R)
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_gfc(StepCtx c, int ngfc) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), K = d.K, M1 = d.M1, B = c.B, p = d.p, n = d.n;
  float* ws = c.ws + r * c.wss;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ngfc) {
    const int e = ((int)blockIdx.x - ngfc) * RC_BLOCK + tid;
    if (e >= p * p * n) return;
    const int cc = e / (p * n), rem = e - cc * p * n, cp = rem / n, i = rem - cp * n;
    ws[c.wo.eAf + e] = ws[c.wo.S + ((int64_t)i * p + cp) * p + cc];
    return;
  }
  const int nout = K * M1 + K + M1;
  const int e = blockIdx.x * 64 + (tid >> 2), g = tid & 3;
  const float* dr = ws + c.wo.edr;
  const float* f1 = ws + c.wo.f1;
  const float* df1 = ws + c.wo.edf1;
  float t = 0.f;
  if (e < K * M1) {
    const int k = e / M1, m = e - k * M1;
#pragma unroll 8
    for (int b = g; b < B; b += 4) t += dr[(int64_t)b * K + k] * fmaxf(f1[(int64_t)b * M1 + m], 0.f);
  } else if (e < K * M1 + K) {
    const int k = e - K * M1;
#pragma unroll 8
    for (int b = g; b < B; b += 4) t += dr[(int64_t)b * K + k];
  } else if (e < nout) {
    const int m = e - K * M1 - K;
#pragma unroll 8
    for (int b = g; b < B; b += 4) t += df1[(int64_t)b * M1 + m];
  }
  t += __shfl_xor(t, 1);
  t += __shfl_xor(t, 2);
  if (e < nout && g == 0) ws[c.wo.gfc + e] = t;
}

// BatchNorm affine partials: slot s of c.dgN sums rows (b, c) [s*rows, (s+1)*rows) of
//   dgamma[f] = sum dx_bn[b][c][f] * xhat[b][c][f],  dbeta[f] = sum dx_bn[b][c][f].  grid (dgN, R)
__device__ __forceinline__ void lemb_bn_body(const StepCtx& c, int s) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y);
  const int p = d.p, F = d.F;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const int nrows = c.B * p, per = (nrows + c.dgN - 1) / c.dgN;
  const int r0 = s * per, r1 = min(nrows, r0 + per);
  const int tid = threadIdx.x, f = tid % F, sl = tid / F, nsl = RC_BLOCK / F;
  __shared__ float red[2][RC_BLOCK];
  const bool train = c.flags & RC_BN_TRAIN;
  float mean = 0.f, inv = 0.f;
  if (sl < nsl) {
    if (train) {
      mean = (float)c.bns[r * c.bnsr + f];
      inv = (float)(1.0 / sqrt(c.bns[r * c.bnsr + F + f] + c.hyp[r].bn_eps));
    } else {
      mean = c.rm[r * F + f];
      inv = 1.0f / sqrtf(c.rv[r * F + f] + (float)c.hyp[r].bn_eps);
    }
  }
  float ag = 0.f, ab = 0.f;
  if (sl < nsl)
#pragma unroll 8
    for (int row = r0 + sl; row < r1; row += nsl) {
      const int b = row / p, cc = row - b * p;
      const float dx = ws[c.wo.edX + (int64_t)row * F + f];
      const float x = X[((c.row0 + b) * d.T + (c.Lmax - F + f)) * p + cc];
      ag += dx * ((x - mean) * inv);
      ab += dx;
    }
  red[0][tid] = ag;
  red[1][tid] = ab;
  __syncthreads();
  if (tid < F) {
    float g = 0.f, bb = 0.f;
    for (int q = 0; q < nsl; ++q) {
      g += red[0][q * F + tid];
      bb += red[1][q * F + tid];
    }
    ws[c.wo.dgb + ((int64_t)s * 2) * F + tid] = g;
    ws[c.wo.dgb + ((int64_t)s * 2 + 1) * F + tid] = bb;
  }
}

// dS_i slices -> slot 0 (fixed order), so the final kernel's adjacency workgroup reads one record.
// block bx of ceil((n-1) p^2 / 256)
__device__ __forceinline__ void lemb_dsred_body(const StepCtx& c, int nds, int bx) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), p = d.p, n = d.n;
  const int64_t pp2 = (int64_t)p * p;
  const int e = bx * RC_BLOCK + threadIdx.x;
  if (e >= (n - 1) * pp2) return;
  float* dS = c.ws + r * c.wss + c.wo.dS + pp2 + e;  // rows i >= 1 of slot 0
  const int64_t ss = (int64_t)n * pp2;
  float t4[4] = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 3 < nds; s += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) t4[u] += dS[(s + u) * ss];
  for (; s < nds; ++s) t4[0] += dS[s * ss];
  dS[0] = (t4[0] + t4[1]) + (t4[2] + t4[3]);
}

// The two independent ends of the GEMM-embedder backward in one launch: workgroups [0, ndr) reduce
// the dS_i slices (lemb_dsred_body), workgroups [ndr, ndr + dgN) the BatchNorm affine partials
// (lemb_bn_body).  grid (ndr + dgN, R)
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_bwd_ends(StepCtx c, int nds, int ndr) {
  rc_critical_priority();
  const int bx = blockIdx.x;
  if (bx < ndr) lemb_dsred_body(c, nds, bx);
  else lemb_bn_body(c, bx - ndr);
}

// ---- small-node windowed kernels (p < 32): the per-window products T_i = S_i x_bn (forward) and
// dx_bn = sum_i S_i^T dT_i, dS_i = sum_b dT_i x_bn^T and the BatchNorm affine partials (backward)
// are p x p x F per window -- 2000 multiply-adds at D4IC, a 5 % corner of one 64 x 64 matrix-core
// tile.  As batched GEMMs they cost one latency-bound workgroup per (window, replica) (R = 128:
// 16384 workgroups, 75 us per product); here one workgroup stages `wb` windows of one replica in
// LDS with every load in flight and runs the products as fmaf chains in the GEMM's k-order.
#define RC_LEMB_LDS 12288  // LDS floats for the staged windows of one workgroup (48 KiB)

// dynamic LDS bytes of the two windowed kernels
__host__ __device__ inline int lemb_win_lds_fwd(const RedcliffDims& d, int wb) {
  return 4 * (128 + (d.n - 1) * d.p * d.p + wb * d.p * d.F);
}
__host__ __device__ inline int lemb_win_lds_bwd(const RedcliffDims& d, int wb) {
  return 4 * (d.n * d.p * d.p + wb * d.p * d.F * (d.n + 2) + 2 * RC_BLOCK);
}

// windows per workgroup, 0 when the node count or batch needs the GEMM products (p >= 32, or
// more than 64 window groups: the dS / BN partial regions hold 64 slots)
__host__ __device__ inline int lemb_win(const RedcliffDims& d, int B) {
  if (d.p >= 32 || B < 1) return 0;
  const int fit = RC_LEMB_LDS / (d.p * (d.n + 2) * d.F);  // windows whose tiles fit the LDS budget
  // few windows per workgroup (many workgroups: the per-window chains are latency-bound; R = 128
  // D4IC: 16 windows per workgroup ran 71 us), but at most 64 groups (the partial slots)
  int wb = (B + 63) / 64;
  if (wb < 4) wb = B < 4 ? B : 4;
  if (wb > fit) return 0;
  if (lemb_win_lds_bwd(d, wb) > 65536) return 0;  // default dynamic LDS limit
  return wb;
}

// x_bn and T_i (i >= 1) of windows [b0, b0 + wb) of replica r.  grid (ceil(B / wb), R)
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_prep_win(StepCtx c, int wb) {
  rc_critical_priority();
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FWD, 0);
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 8);
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), b0 = blockIdx.x * wb;
  const int p = d.p, F = d.F, n = d.n, pF = p * F, pp2 = p * p;
  const int nw = min(wb, c.B - b0), tot = nw * pF;  // tot <= RC_LEMB_LDS / 3 = 16 * RC_BLOCK
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr + ((c.row0 + b0) * d.T + (c.Lmax - F)) * p;
  extern __shared__ float sm[];
  float* alpha = sm;             // [64]
  float* beta = alpha + 64;      // [64]
  float* S = beta + 64;          // S_1 .. S_{n-1}
  float* xb = S + (n - 1) * pp2; // [w][c][f]
  const int tid = threadIdx.x;
  const RcDiv dpf(pF), dp(p);
  float v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {  // window w's F rows of X are contiguous ([t][c])
    const int e = u * RC_BLOCK + tid;
    v[u] = 0.f;
    if (e < tot) {
      const int w = dpf.div(e);
      v[u] = X[(int64_t)w * d.T * p + (e - w * pF)];
    }
  }
  for (int e = tid; e < (n - 1) * pp2; e += RC_BLOCK) S[e] = ws[c.wo.S + pp2 + e];
  if (tid < F) {
    const bool train = c.flags & RC_BN_TRAIN;
    float mean, inv;
    if (train) {
      mean = (float)c.bns[r * c.bnsr + tid];
      inv = (float)(1.0 / sqrt(c.bns[r * c.bnsr + F + tid] + c.hyp[r].bn_eps));
    } else {
      mean = c.rm[r * F + tid];
      inv = 1.0f / sqrtf(c.rv[r * F + tid] + (float)c.hyp[r].bn_eps);
    }
    const float a = inv * E[c.eo.bnw + tid];
    alpha[tid] = a;
    beta[tid] = E[c.eo.bnb + tid] - mean * a;
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 9);
  const int64_t pnF = (int64_t)pF * n, nF = (int64_t)n * F;
  float* T = ws + c.wo.T + (int64_t)b0 * pnF;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = u * RC_BLOCK + tid;
    if (e < tot) {
      const int w = dpf.div(e), rem = e - w * pF, f = dp.div(rem), ch = rem - f * p;
      const float x = v[u] * alpha[f] + beta[f];
      xb[w * pF + ch * F + f] = x;
      T[w * pnF + ch * nF + f] = x;
    }
  }
  if (n == 1) {
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FWD, 1);
    return;
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 10);
  // T_i[w][ch][f] = sum_{c'} S_i[ch][c'] x_bn[w][c'][f]  (c' in order), items (i, w, ch, f)
  const RcDiv dF(F);
  for (int e = tid; e < (n - 1) * tot; e += RC_BLOCK) {
    const int i1 = dpf.div(e) / nw, q = e - i1 * tot;  // q = (w, ch, f)
    const int w = dpf.div(q), rem = q - w * pF, ch = dF.div(rem), f = rem - ch * F;
    const float* Si = S + i1 * pp2 + ch * p;
    const float* xw = xb + w * pF + f;
    float t = 0.f;
#pragma unroll 4
    for (int cp = 0; cp < p; ++cp) t = fmaf(Si[cp], xw[cp * F], t);
    T[w * pnF + ch * nF + (i1 + 1) * F + f] = t;
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 11);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FWD, 1);
}

// Backward of the per-window products for windows [g * wb, g * wb + wb) of replica r: dx_bn
// (never stored), its BatchNorm affine partials into ws.dgb slot g and the dS_i partials into
// ws.dS slot g (summed by k_emb_final's adjacency workgroup, c.dsN = c.dgN = ceil(B / wb)).
// grid (ceil(B / wb), R)
__global__ __launch_bounds__(RC_BLOCK) void k_lemb_win_bwd(StepCtx c, int wb) {
  rc_critical_priority();
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 0);
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 0);
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), g = blockIdx.x, b0 = g * wb;
  const int p = d.p, F = d.F, n = d.n, pF = p * F, pp2 = p * p;
  const int nw = min(wb, c.B - b0);
  const int64_t pnF = (int64_t)pF * n, nF = (int64_t)n * F;
  float* ws = c.ws + r * c.wss;
  extern __shared__ float sm[];
  float* S = sm;                    // S_0 .. S_{n-1}
  float* dT = S + n * pp2;          // [w][c'][i][f]
  float* x0 = dT + nw * pnF;        // x_bn [w][c][f]
  float* xr = x0 + nw * pF;         // raw X [w][f][c]
  float* red = xr + nw * pF;        // [2][RC_BLOCK]
  const int tid = threadIdx.x;
  const float* X = c.X + r * c.xr + ((c.row0 + b0) * d.T + (c.Lmax - F)) * p;
  const float* dTg = ws + c.wo.edT + (int64_t)b0 * pnF;
  const float* Tg = ws + c.wo.T + (int64_t)b0 * pnF;
  const RcDiv dpf(pF), dF(F);
  // stage (every segment's loads in flight together): dT (contiguous over the group's windows),
  // x_bn = the T_0 rows, raw X, S
  rc_stage_all(rc_seg<8>(nw * (int)pnF, [&](int e) { return dTg[e]; }, [&](int e, float v) { dT[e] = v; }),
               rc_seg<4>(nw * pF, [&](int e) {
                 const int w = dpf.div(e), rem = e - w * pF, ch = dF.div(rem);
                 return Tg[w * pnF + ch * nF + (rem - ch * F)];
               }, [&](int e, float v) { x0[e] = v; }),
               rc_seg<4>(nw * pF, [&](int e) {
                 const int w = dpf.div(e);
                 return X[(int64_t)w * d.T * p + (e - w * pF)];
               }, [&](int e, float v) { xr[e] = v; }),
               rc_seg<2>(n * pp2, [&](int e) { return ws[c.wo.S + e]; }, [&](int e, float v) { S[e] = v; }));
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 1);
  const int f = tid % F, sl = tid / F, nsl = RC_BLOCK / F;
  float mean = 0.f, inv = 0.f;
  if (sl < nsl) {
    if (c.flags & RC_BN_TRAIN) {
      mean = (float)c.bns[r * c.bnsr + f];
      inv = (float)(1.0 / sqrt(c.bns[r * c.bnsr + F + f] + c.hyp[r].bn_eps));
    } else {
      mean = c.rm[r * F + f];
      inv = 1.0f / sqrtf(c.rv[r * F + f] + (float)c.hyp[r].bn_eps);
    }
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 2);
  // dx_bn[w][ch][f] = sum_{c'} sum_i S_i[c'][ch] dT[w][c'][i][f]  (k = c' n + i, the GEMM's order);
  // lanes (f, slot) over rows (w, ch): dgamma[f] += dx xhat, dbeta[f] += dx
  // (a thread's rows sl, sl + nsl, ... run four at a time as interleaved chains; each row's chain and
  // the row order of the dgamma / dbeta sums are unchanged)
  float ag = 0.f, ab = 0.f;
  if (sl < nsl)
    for (int r0 = sl; r0 < nw * p; r0 += 4 * nsl) {
      int chj[4], dtj[4];  // the row's channel and the LDS offset of its window's dT column f
      float dx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = min(r0 + j * nsl, nw * p - 1);  // past the end: a repeat of the last row, not summed
        const int w = row / p;
        chj[j] = row - w * p;
        dtj[j] = w * (int)pnF + f;
        dx[j] = 0.f;
      }
      for (int cp = 0; cp < p; ++cp)
        for (int i = 0; i < n; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) dx[j] = fmaf(S[i * pp2 + cp * p + chj[j]], dT[dtj[j] + cp * (int)nF + i * F], dx[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = r0 + j * nsl;
        if (row < nw * p) {
          const int w = row / p, ch = row - w * p;
          const float x = xr[w * pF + f * p + ch];
          ag += dx[j] * ((x - mean) * inv);
          ab += dx[j];
        }
      }
    }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 3);
  red[tid] = ag;
  red[RC_BLOCK + tid] = ab;
  // dS_i[ch][c'] partial = sum_w sum_f dT[w][ch][i][f] x_bn[w][c'][f]   (w outer, f inner), i >= 1
  float* dS = ws + c.wo.dS + (int64_t)g * c.dsS;
  for (int e = tid; e < (n - 1) * pp2; e += RC_BLOCK) {
    const int i = 1 + e / pp2, rem = e - (i - 1) * pp2, ch = rem / p, cp = rem - ch * p;
    float t = 0.f;
    for (int w = 0; w < nw; ++w) {
      const float* a = dT + w * pnF + ch * nF + i * F;
      const float* bq = x0 + w * pF + cp * F;
#pragma unroll 4
      for (int ff = 0; ff < F; ++ff) t = fmaf(a[ff], bq[ff], t);
    }
    dS[i * pp2 + rem] = t;
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 4);
  __syncthreads();
  if (tid < F) {
    float ga = 0.f, gb = 0.f;
    for (int q = 0; q < nsl; ++q) {
      ga += red[q * F + tid];
      gb += red[RC_BLOCK + q * F + tid];
    }
    ws[c.wo.dgb + ((int64_t)g * 2) * F + tid] = ga;
    ws[c.wo.dgb + ((int64_t)g * 2 + 1) * F + tid] = gb;
  }
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 5);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 1);
}

// splits of the fc1 contraction (p*H): largest divisor of p*H that is <= 64 with >= 64 terms each
int fc1_splits(const RedcliffDims& d) {
  const int pH = d.p * d.H;
  for (int s = 64; s > 1; --s)
    if (pH % s == 0 && pH / s >= 64) return s;
  return 1;
}

// window groups of the dS product: a power-of-two divisor of B, at most 64
int ds_splits(int B) {
  int s = 64;
  while (s > 1 && B % s) s >>= 1;
  return s;
}

}  // namespace

// GEMM-shaped embedder: large p (C5), or a packed grid search of >= RC_EMB_GEMM_R replicas, whose
// products batched over the replicas keep the matrix cores busy where the fused node-chunk
// kernels' per-workgroup latency chains set the time.  REDCLIFF_EMB_PATH=gemm|fused overrides; the
// round-4 value "batched" (the replica-batched embedder, removed in round 5) is no longer accepted
// and, like any other value, leaves the default choice.
#ifndef RC_EMB_GEMM_R
#define RC_EMB_GEMM_R 16
#endif
bool rc_emb_use_gemm(const RedcliffDims& d) {
  const char* v = getenv("REDCLIFF_EMB_PATH");  // read per call: tests switch paths in-process
  if (v && !strcmp(v, "gemm")) return d.F <= 64 && d.M1 <= 64;
  if (v && !strcmp(v, "fused")) return false;
  return (d.p >= 32 || d.R >= RC_EMB_GEMM_R) && d.F <= 64 && d.M1 <= 64;
}

// windows per workgroup of the windowed kernels for this step (0: the GEMM products);
// REDCLIFF_EMB_WIN=0 forces the GEMM products (tests, tuning)
static int lemb_win_step(const StepCtx& c) {
  const char* v = getenv("REDCLIFF_EMB_WIN");
  if (v && !strcmp(v, "0")) return 0;
  return lemb_win(c.d, c.B);
}

void rc_emb_partial_layout(StepCtx& c, bool gemm) {
  const RedcliffDims& d = c.d;
  const int nch = rc_nchunk(d), n = d.n, p = d.p;
  c.dwN = p;
  const int wb = gemm ? lemb_win_step(c) : 0;
  if (wb) {  // k_lemb_win_bwd: one dS / BN record [s][i][cc][c'] / [s][2][F] per window group
    c.dsN = c.dgN = (c.B + wb - 1) / wb;
    c.dsCC = p;
    c.dsS = (int64_t)n * p * p;
    c.dsI = (int64_t)p * p;
  } else if (gemm) {  // dS partials [s][i][cc][c'] over window groups, reduced into slot 0; BN partials over row slices
    c.dsN = 1;
    c.dsCC = p;
    c.dsS = (int64_t)n * p * p;
    c.dsI = (int64_t)p * p;
    c.dgN = p * nch < 64 ? p * nch : 64;
  } else {  // node-chunk kernel: [node][chunk][i][c'] and one BN record per (node, chunk)
    c.dsN = nch;
    c.dsCC = (int64_t)nch * n * p;
    c.dsS = (int64_t)n * p;
    c.dsI = p;
    c.dgN = p * nch;
  }
}

// Products of the GEMM-shaped embedder: one launch per product for ALL replicas of the step (the
// replica axis of rc_gemm.h: operands of replica r at r * c.wss in the workspace and r * c.es in
// the embedder parameters), so a packed grid search runs the same launch chain as one fit.  Each
// output keeps the in-order fmaf chain of the one-replica launch, so packed and single fits agree
// bit for bit.
int rc_launch_emb_fwd_gemm(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int p = d.p, F = d.F, n = d.n, H = d.H, M1 = d.M1, B = c.B;
  const int64_t pnF = (int64_t)p * n * F, nF = (int64_t)n * F;
  if (F > 64 || M1 > 64) { rc_set_error("GEMM embedder: F <= 64 and M1 <= 64 required"); return REDCLIFF_ELIMIT; }
  const int wb = lemb_win_step(c);
  int e;
  if (wb) {
    hipLaunchKernelGGL(k_lemb_prep_win, dim3((B + wb - 1) / wb, c.nrep), dim3(RC_BLOCK), lemb_win_lds_fwd(d, wb), s, c,
                       wb);
    e = rc_check(hipGetLastError(), "k_lemb_prep_win");
  } else {
    hipLaunchKernelGGL(k_lemb_prep, dim3(B, c.nrep), dim3(RC_BLOCK), 0, s, c);
    e = rc_check(hipGetLastError(), "k_lemb_prep");
  }
  const int nsp = fc1_splits(d), Ks = p * H / nsp;
  float* ws = c.ws;  // replica 0's slice; the replica axis adds r * c.wss
  const float* E = c.emb;
  float* T = ws + c.wo.T;
  // T_i[b] = S_i x_bn[b]  (p x p x F per window), the n - 1 products independent: up to three per launch
  for (int i0 = 1; i0 < n && !e && !wb; i0 += RC_GEMM_SET_MAX) {
    RcGemm gs[RC_GEMM_SET_MAX];
    int bs[RC_GEMM_SET_MAX], ng = 0;
    for (int i = i0; i < n && ng < RC_GEMM_SET_MAX; ++i, ++ng) {
      gs[ng] = rc_gemm_args(0, 0, p, F, p, ws + c.wo.S + (int64_t)i * p * p, p, 0, T, nF, pnF, T + i * F, nF, pnF);
      rc_gemm_reps(gs[ng], c, c.wss, c.wss, c.wss);
      bs[ng] = B;
    }
    e = rc_gemm_launch_set(gs, bs, ng, s, "emb T_i");
  }
  if (!e) {  // R = relu(T gcW): (B*p) x (n*F) x H
    RcGemm g = rc_gemm_args(0, 0, B * p, H, (int)nF, T, nF, 0, E + c.eo.gcW, H, 0, ws + c.wo.R, H, 0);
    g.epi = RC_EPI_RELU;
    rc_gemm_reps(g, c, c.wss, c.es, c.wss);
    e = rc_gemm_launch(g, 1, s, "emb graph conv");
  }
  if (!e) {  // fc1 partials over nsp slices of the p*H contraction
    RcGemm g = rc_gemm_args(0, 1, B, M1, Ks, ws + c.wo.R, (int64_t)p * H, Ks, E + c.eo.fc1W, (int64_t)p * H, Ks,
                            ws + c.wo.f1p, M1, (int64_t)d.Bmax * M1);
    rc_gemm_reps(g, c, c.wss, c.es, c.wss);
    e = rc_gemm_launch(g, nsp, s, "emb fc1");
  }
  if (e) return e;
  // windows per wave: 4 for packs of >= 8 replicas (REDCLIFF_HEAD_WPW=1|2|4 overrides), else 1
  const char* hv = getenv("REDCLIFF_HEAD_WPW");
  const int hw = hv ? atoi(hv) : (c.nrep >= 8 ? 4 : 1);
  if (hw == 4)
    hipLaunchKernelGGL(k_lemb_head<4>, dim3((B + 15) / 16, c.nrep), dim3(RC_BLOCK), 0, s, c, nsp);
  else if (hw == 2)
    hipLaunchKernelGGL(k_lemb_head<2>, dim3((B + 7) / 8, c.nrep), dim3(RC_BLOCK), 0, s, c, nsp);
  else
    hipLaunchKernelGGL(k_lemb_head<1>, dim3((B + 3) / 4, c.nrep), dim3(RC_BLOCK), 0, s, c, nsp);
  return rc_check(hipGetLastError(), "k_lemb_head");
}

int rc_launch_emb_bwd_gemm(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int p = d.p, F = d.F, n = d.n, H = d.H, M1 = d.M1, B = c.B;
  const int64_t pnF = (int64_t)p * n * F, nF = (int64_t)n * F, pH = (int64_t)p * H;
  hipLaunchKernelGGL(k_lemb_dhead, dim3((B + lemb_wpw(d) - 1) / lemb_wpw(d), c.nrep), dim3(RC_BLOCK), 0, s, c);
  int e = rc_check(hipGetLastError(), "k_lemb_dhead");
  const int wb = lemb_win_step(c);
  if (wb && c.dsN != (B + wb - 1) / wb) {
    rc_set_error("windowed embedder backward: partial layout of %d groups, %d expected", c.dsN, (B + wb - 1) / wb);
    return REDCLIFF_EINVAL;
  }
  if (!e) {
    const int ngfc = (d.K * M1 + d.K + M1 + 63) / 64, naf = wb ? 0 : (p * p * n + RC_BLOCK - 1) / RC_BLOCK;
    hipLaunchKernelGGL(k_lemb_gfc, dim3(ngfc + naf, c.nrep), dim3(RC_BLOCK), 0, s, c, ngfc);
    e = rc_check(hipGetLastError(), "k_lemb_gfc");
  }
  const int nds = ds_splits(B), wps = B / nds;
  float* ws = c.ws;  // replica 0's slice; the replica axis adds r * c.wss
  const float* E = c.emb;
  const float* T = ws + c.wo.T;
  const float* df1 = ws + c.wo.edf1;
  // (pairs of products that do not depend on each other share a launch where the LDS-tiled core runs
  // them, rc_gemm_launch_set: dfc1W and dZ both read df1; dW and dT both read dZ)
  if (!e) {
    RcGemm gs[2];
    const int bs[2] = {1, 1};
    // dfc1W = df1^T R   (M1 x B x p*H), applied by the final kernel's Adam
    gs[0] = rc_gemm_args(1, 0, M1, (int)pH, B, df1, M1, 0, ws + c.wo.R, pH, 0, ws + c.wo.gfc1, pH, 0);
    rc_gemm_reps(gs[0], c, c.wss, c.wss, c.wss);
    // dZ = [R > 0] (df1 fc1W)   (B x M1 x p*H)
    gs[1] = rc_gemm_args(0, 0, B, (int)pH, M1, df1, M1, 0, E + c.eo.fc1W, pH, 0, ws + c.wo.dZ, pH, 0);
    gs[1].epi = RC_EPI_MASK;
    gs[1].aux = ws + c.wo.R;
    gs[1].ldaux = pH;
    rc_gemm_reps(gs[1], c, c.wss, c.es, c.wss, c.wss);
    e = rc_gemm_launch_set(gs, bs, 2, s, "emb dfc1W + dZ");
  }
  if (!e) {
    RcGemm gs[2];
    const int bs[2] = {p, 1};
    // dW slices: dWi[s] = T[rows s]^T dZ[rows s], p slices of B rows of the (b, c) axis
    gs[0] = rc_gemm_args(1, 0, (int)nF, H, B, T, nF, (int64_t)B * nF, ws + c.wo.dZ, H, (int64_t)B * H, ws + c.wo.dWi,
                         H, nF * H);
    rc_gemm_reps(gs[0], c, c.wss, c.wss, c.wss);
    // dT = dZ gcW^T   ((B*p) x H x n*F)
    gs[1] = rc_gemm_args(0, 1, B * p, (int)nF, H, ws + c.wo.dZ, H, 0, E + c.eo.gcW, H, 0, ws + c.wo.edT, nF, 0);
    rc_gemm_reps(gs[1], c, c.wss, c.es, c.wss);
    e = rc_gemm_launch_set(gs, bs, 2, s, "emb dW + dT");
  }
  if (wb) {  // dx_bn, its BatchNorm partials and the dS_i partials, wb windows per workgroup
    if (e) return e;
    hipLaunchKernelGGL(k_lemb_win_bwd, dim3(c.dsN, c.nrep), dim3(RC_BLOCK), lemb_win_lds_bwd(d, wb), s, c, wb);
    return rc_check(hipGetLastError(), "k_lemb_win_bwd");
  }
  // dx_bn[b] = Af dT[b] (p x p*n x F per window) and the dS_i slices (sum over the windows of group z of
  // dT_i[b] x_bn[b]^T, p x wps*F x p): independent products, up to three per launch
  {
    RcGemm gs[RC_GEMM_SET_MAX];
    int bs[RC_GEMM_SET_MAX], ng = 0;
    gs[0] = rc_gemm_args(0, 0, p, F, p * n, ws + c.wo.eAf, (int64_t)p * n, 0, ws + c.wo.edT, F, pnF, ws + c.wo.edX,
                         F, (int64_t)p * F);
    rc_gemm_reps(gs[0], c, c.wss, c.wss, c.wss);
    bs[0] = B;
    ng = 1;
    for (int i = 1; i < n && !e; ++i) {
      RcGemm q = rc_gemm_args(0, 1, p, p, wps * F, ws + c.wo.edT + i * F, nF, (int64_t)wps * pnF, T, nF,
                              (int64_t)wps * pnF, ws + c.wo.dS + (int64_t)i * p * p, p, c.dsS);
      q.Kblk = F;
      q.rA = pnF;
      q.rB = pnF;
      rc_gemm_reps(q, c, c.wss, c.wss, c.wss);
      if (ng == RC_GEMM_SET_MAX) {
        e = rc_gemm_launch_set(gs, bs, ng, s, "emb dx_bn + dS");
        ng = 0;
      }
      gs[ng] = q;
      bs[ng++] = nds;
    }
    if (!e && ng) e = rc_gemm_launch_set(gs, bs, ng, s, "emb dx_bn + dS");
  }
  if (e) return e;
  const int ndr = n > 1 ? (int)(((int64_t)(n - 1) * p * p + RC_BLOCK - 1) / RC_BLOCK) : 0;
  hipLaunchKernelGGL(k_lemb_bwd_ends, dim3(ndr + c.dgN, c.nrep), dim3(RC_BLOCK), 0, s, c, nds, ndr);
  return rc_check(hipGetLastError(), "k_lemb_bwd_ends");
}
