// rc_embed_batched.hip -- the DGCNN factor-score embedder of a packed grid search as three
// replica-batched kernels (round 4).  One 256-thread workgroup per (replica, 16-window tile) runs
// the forward, one the backward, with every intermediate of its tile in LDS (no HBM round trip
// between the products of a tile); a third kernel, one workgroup per replica, forms the weight
// gradients that sum over the whole batch (dfc1W = df1^T R and the fc2 / bias gradients).  It
// replaces the GEMM chain of rc_embed_gemm.hip (about ten launches per step whose intermediates
// T, R, f1, dZ, dT went through HBM between launches) for small node counts, where each per-tile
// product is a handful of 16x16 matrix-core tiles.
//
// Reference: models/redcliff_factor_score_embedders.py:335-392 (DGCNN_Embedder) ->
// models/dgcnn.py:15-64 -> torcheeg 1.1.3 DGCNN (oracle/torcheeg_dgcnn.py): BatchNorm1d over the F
// features, Chebyshev supports S_i of normalize_A(A), graph convolution sum_i S_i x W_i, ReLU,
// fc1 (p*H -> M1), ReLU, fc2 (M1 -> K).  The three embedder evaluations of a reference step
// (:844-856) are one here.
//
// Tile layouts (LDS; the MFMA is v_mfma_f32_16x16x4_f32, lane l: l15 = l & 15, g = l >> 4,
// D rows 4g + reg, column l15):
//   Ts  [c][w][nFs]  T = [x_bn | S_1 x_bn | ...] node-major, so M-tile c of the graph convolution
//                    is node c's 16 windows; row stride nFs = 2 mod 4 (A reads: 16 rows x 2 k-slots
//                    on 32 distinct banks), node stride 16 nFs + 1 (per-node loops over c in lockstep
//                    -- the dS product, the staging stores -- hit distinct banks)
//   Rs  [w][pHs]     relu(T gcW) window-major, the fc1 A operand (pHs = 2 mod 4)
//   DZs [c][w][Hs]   dL/dZ = [R > 0] dL/dR, node-major, same strides as Ts
//   DTs [c][w][nFs]  dL/dT
// Every output is an fmaf chain in a fixed order (k ascending within an MFMA tile; cross-wave and
// cross-tile partials added in index order), so a replica's bits do not depend on the pack it runs
// in: a pack equals its fits run one by one on this path (tests/test_gpu_replicas.py).
//
// The forward writes the workspace regions the GEMM chain writes (T [b][c][nF], R [b][c][H],
// f1 [b][M1], w [b][K]), so the factor mixing, the head workgroup and validation read the same
// records.  The backward writes one partial record per tile for the final kernel (dW_i -> ws.dWi
// slot t, c.dwN tiles; BatchNorm affine -> ws.dgb slot t; dS_i -> ws.dS slot t) plus dr / df1 for
// k_gemb_dfc1, which writes dfc1W -> ws.gfc1 and fc2 / fc2-bias / fc1-bias -> ws.gfc; k_emb_final
// applies Adam as for the other paths.
#include <cstdlib>
#include <cstring>

#include "rc_common.h"

#define GB_THREADS 256
#define GB_WAVES (GB_THREADS / 64)
#define GB_WT 16       // windows per tile
#define GB_MAXKF 96    // fc1 k-steps (p*H <= 384)
#define GB_MAXNQ 5     // fc1 column tiles per wave in the backward (p*H <= 4 * 5 * 16 = 320)
#define GB_MAXNT 3     // column tiles of the n*F axis (n*F <= 48)
#define GB_MAXKH 8     // k-steps of the H axis (H <= 32)
#define GB_DFC_THREADS 512

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline f32x4 gb_mfma(float a, float b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

// padded row stride 2 mod 4 (A-operand reads of 16 rows x 2 k-slots hit 32 distinct banks)
__host__ __device__ inline int gb_s2(int x) { return x + ((2 - x) & 3); }

struct GbShape {
  int p, F, n, H, M1, K, nF, pH, nFs, pHs, Hs, NSt, NSz, M1h, nkz, nkf, nqt, ntt, nkh;
  __host__ __device__ explicit GbShape(const RedcliffDims& d)
      : p(d.p), F(d.F), n(d.n), H(d.H), M1(d.M1), K(d.K), nF(d.n * d.F), pH(d.p * d.H) {
    nkz = (nF + 3) / 4;   // k-steps of the graph convolution (over n*F)
    nkf = (pH + 3) / 4;   // k-steps of fc1 (over p*H)
    nqt = (pH + 15) / 16; // column tiles of dR (over p*H)
    ntt = (nF + 15) / 16; // column tiles of dT (over n*F)
    nkh = (H + 3) / 4;    // k-steps of dT (over H)
    nFs = gb_s2(4 * nkz > 16 * ntt ? 4 * nkz : 16 * ntt);  // the last k-step / column tile stays in the row
    pHs = gb_s2(4 * nkf);
    Hs = gb_s2(4 * nkh > 32 ? 4 * nkh : 32);               // dW_i reads columns up to 31
    NSt = 16 * nFs + 1;
    NSz = 16 * Hs + 1;
    M1h = M1 + 1;         // f1 rows for the head: windows on distinct banks
  }
};

__host__ __device__ inline int gb_lds_fwd(const GbShape& s) {
  return s.p * s.NSt + GB_WT * s.pHs + GB_WT * s.M1h + (s.n - 1) * s.p * s.p + 128;
}
__host__ __device__ inline int gb_lds_bwd(const GbShape& s) {
  return 2 * s.p * s.NSt + GB_WT * s.pHs + s.p * s.NSz + GB_WT * gb_s2(s.M1) + GB_WT * s.F * s.p + s.K * s.M1 +
         GB_WT * 16 + s.n * s.p * s.p + 16 * GB_MAXNT * s.Hs + 2 * GB_THREADS;
}
__host__ __device__ inline int gb_ntiles(int B) { return (B + GB_WT - 1) / GB_WT; }

// BatchNorm scale / shift of feature f: train mode from the batch statistics, eval mode from the
// running statistics (torch BatchNorm1d; the GEMM chain's k_lemb_prep_win)
__device__ inline void gb_bn(const StepCtx& c, int r, int f, float& mean, float& inv) {
  if (c.flags & RC_BN_TRAIN) {
    mean = (float)c.bns[r * c.bnsr + f];
    inv = (float)(1.0 / sqrt(c.bns[r * c.bnsr + c.d.F + f] + c.hyp[r].bn_eps));
  } else {
    mean = c.rm[r * c.d.F + f];
    inv = 1.0f / sqrtf(c.rv[r * c.d.F + f] + (float)c.hyp[r].bn_eps);
  }
}

// zero the padding columns [from, stride) of `rows` rows (read by the last k-step / column tile of a
// product: LDS garbage could be NaN, and 0 * NaN is NaN); row r at (r / 16) * ns + (r % 16) * stride
__device__ inline void gb_zero_pad(float* base, int rows, int from, int stride, int ns) {
  const int w = stride - from;
  for (int e = threadIdx.x; e < rows * w; e += GB_THREADS) {
    const int r = e / w;
    base[(r >> 4) * ns + (r & 15) * stride + from + (e - r * w)] = 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// Forward.  grid (tiles, nrep), 256 threads.  x_bn and T_i into Ts (vector), the graph convolution
// Z = T gcW as p x 2 output tiles (wave w: column tile w & 1, nodes w >> 1, +2, ...; gcW in
// registers), R = relu(Z) into Rs, fc1 as 4 column tiles (wave w: m = 16 w + l15, fc1W in
// registers), the head (fc2) per window; T, R, f1, w to the workspace.
__global__ __launch_bounds__(GB_THREADS) void k_gemb_fwd(StepCtx c) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const GbShape s(d);
  const int r = rc_rep(c, blockIdx.y), b0 = blockIdx.x * GB_WT;
  if (b0 >= c.B) return;
  const int nw = min(GB_WT, c.B - b0);
  const int p = s.p, F = s.F, n = s.n, H = s.H, M1 = s.M1, K = s.K, nF = s.nF, pH = s.pH;
  const int nFs = s.nFs, pHs = s.pHs, NSt = s.NSt, M1h = s.M1h;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  extern __shared__ float sm[];
  float* Ts = sm;                          // [p][16][nFs], node stride NSt
  float* Rs = Ts + p * NSt;                // [16][pHs]
  float* F1s = Rs + GB_WT * pHs;           // [16][M1h]
  float* Ss = F1s + GB_WT * M1h;           // S_1 .. S_{n-1}
  float* alpha = Ss + (n - 1) * p * p;     // [64]
  float* beta = alpha + 64;                // [64]
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pF = p * F;
  // register operands: graph conv B = gcW[(i,f)][h] (column tile wv & 1); fc1 B = fc1W[m][q] (m = 16 wv + l15)
  const int hz = 16 * (wv & 1) + l15;
  float gB[16];
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + g;
    gB[ks] = (ks < s.nkz && k < nF && hz < H) ? E[c.eo.gcW + k * H + hz] : 0.f;
  }
  const int mf = 16 * wv + l15;
  float fB[GB_MAXKF];
#pragma unroll
  for (int ks = 0; ks < GB_MAXKF; ++ks) {
    const int q = 4 * ks + g;
    fB[ks] = (ks < s.nkf && q < pH && mf < M1) ? E[c.eo.fc1W + (int64_t)mf * pH + q] : 0.f;
  }
  if (tid < F) {
    float mean, inv;
    gb_bn(c, r, tid, mean, inv);
    const float a = inv * E[c.eo.bnw + tid];
    alpha[tid] = a;
    beta[tid] = E[c.eo.bnb + tid] - mean * a;
  }
  for (int e = tid; e < (n - 1) * p * p; e += GB_THREADS) Ss[e] = ws[c.wo.S + p * p + e];
  gb_zero_pad(Ts, 16 * p, nF, nFs, NSt);
  gb_zero_pad(Rs, GB_WT, pH, pHs, GB_WT * pHs);
  __syncthreads();
  // ---- x_bn (T_0) of the tile (X[row0 + b][Lmax - F + f][c], contiguous (f, c) per window; 8 loads
  // in flight per thread): consecutive threads take consecutive channels, i.e. consecutive nodes,
  // whose rows are one bank apart (node stride NSt = 1 mod 32)
  const float* Xg = c.X + r * c.xr + ((c.row0 + b0) * d.T + (c.Lmax - F)) * p;
  rc_stage<8>(GB_WT * pF, [&](int e) {
    const int w = e / pF;
    return w < nw ? Xg[(int64_t)w * d.T * p + (e - w * pF)] : 0.f;
  }, [&](int e, float v) {
    const int w = e / pF, rem = e - w * pF, f = rem / p, ch = rem - f * p;
    Ts[ch * NSt + w * nFs + f] = w < nw ? v * alpha[f] + beta[f] : 0.f;
  });
  __syncthreads();
  // ---- T_i = S_i x_bn (i >= 1), c' ascending
  for (int e = tid; e < (n - 1) * p * 16 * F; e += GB_THREADS) {
    const int i1 = e / (p * 16 * F), rem = e - i1 * p * 16 * F, ch = rem / (16 * F), r2 = rem - ch * 16 * F;
    const int w = r2 / F, f = r2 - w * F;
    const float* Si = Ss + (i1 * p + ch) * p;
    float t = 0.f;
    for (int cp = 0; cp < p; ++cp) t = fmaf(Si[cp], Ts[cp * NSt + w * nFs + f], t);
    Ts[ch * NSt + w * nFs + (i1 + 1) * F + f] = w < nw ? t : 0.f;
  }
  __syncthreads();
  // ---- T to the workspace ([b][c][nF]) for the backward; the graph convolution
  for (int e = tid; e < nw * p * nF; e += GB_THREADS) {
    const int w = e / (p * nF), rem = e - w * p * nF, ch = rem / nF, col = rem - ch * nF;
    ws[c.wo.T + (int64_t)(b0 + w) * p * nF + rem] = Ts[ch * NSt + w * nFs + col];
  }
  for (int ch = wv >> 1; ch < p; ch += GB_WAVES / 2) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* a = Ts + ch * NSt + l15 * nFs + g;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      if (ks < s.nkz) acc = gb_mfma(a[4 * ks], gB[ks], acc);
    if (hz < H)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) Rs[(4 * g + reg) * pHs + ch * H + hz] = fmaxf(acc[reg], 0.f);
  }
  __syncthreads();
  for (int e = tid; e < nw * pH; e += GB_THREADS) {
    const int w = e / pH;
    ws[c.wo.R + (int64_t)(b0 + w) * pH + (e - w * pH)] = Rs[w * pHs + (e - w * pH)];
  }
  // ---- fc1: f1[w][m] = fc1b[m] + sum_q R[w][q] fc1W[m][q] (q ascending)
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* a = Rs + l15 * pHs + g;
#pragma unroll
    for (int ks = 0; ks < GB_MAXKF; ++ks)
      if (ks < s.nkf) acc = gb_mfma(a[4 * ks], fB[ks], acc);
    if (mf < M1) {
      const float bias = E[c.eo.fc1b + mf];
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int w = 4 * g + reg;
        const float v = acc[reg] + bias;
        F1s[w * M1h + mf] = v;
        if (w < nw) ws[c.wo.f1 + (int64_t)(b0 + w) * M1 + mf] = v;
      }
    }
  }
  __syncthreads();
  // ---- head: w[k] = fc2b[k] + sum_m fc2W[k][m] relu(f1[m]), m ascending
  for (int e = tid; e < nw * K; e += GB_THREADS) {
    const int w = e / K, k = e - w * K;
    const float* w2 = E + c.eo.fc2W + k * M1;
    float a = 0.f;
    for (int m = 0; m < M1; ++m) a = fmaf(w2[m], fmaxf(F1s[w * M1h + m], 0.f), a);
    ws[c.wo.w + (int64_t)(b0 + w) * K + k] = a + E[c.eo.fc2b + k];
  }
}

// ------------------------------------------------------------------------------------------
// Backward.  grid (tiles, nrep), 256 threads.  Per tile:
//   dr = dL/d(raw embedder output) (the factor side's per-channel partials summed in channel
//        order, the label and fw-L1 terms: rc_emb_draw) -> ws.edr;
//   df1 = [f1 > 0] dr fc2W -> ws.edf1 (k_gemb_dfc1 forms dfc1W and the fc2 / bias gradients);
//   dR = df1 fc1W (column tiles over the waves, fc1W in registers), dZ = [R > 0] dR into DZs;
//   dT = dZ gcW^T (node tiles over the waves), dW_i = T^T dZ (per-wave partials over the wave's
//        nodes, added in wave order) -> ws.dWi slot t;
//   dx_bn = sum_i S_i^T dT_i -> BatchNorm affine partials -> ws.dgb slot t; dS_i = dT_i x_bn^T ->
//        ws.dS slot t.
__global__ __launch_bounds__(GB_THREADS) void k_gemb_bwd(StepCtx c) {
  rc_critical_priority();
  const RedcliffDims& d = c.d;
  const GbShape s(d);
  const int r = rc_rep(c, blockIdx.y), tile = blockIdx.x, b0 = tile * GB_WT;
  if (b0 >= c.B) return;
  const int nw = min(GB_WT, c.B - b0);
  const int p = s.p, F = s.F, n = s.n, H = s.H, M1 = s.M1, K = s.K, nF = s.nF, pH = s.pH;
  const int nFs = s.nFs, pHs = s.pHs, Hs = s.Hs, NSt = s.NSt, NSz = s.NSz, M1s = gb_s2(M1);
  const int pp2 = p * p, pF = p * F;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  extern __shared__ float sm[];
  float* Ts = sm;                          // [p][16][nFs], node stride NSt
  float* DTs = Ts + p * NSt;               // [p][16][nFs], node stride NSt
  float* Rs = DTs + p * NSt;               // [16][pHs]
  float* DZs = Rs + GB_WT * pHs;           // [p][16][Hs], node stride NSz
  float* DF1 = DZs + p * NSz;              // [16][M1s]: f1, then dL/df1 in place
  float* Xs = DF1 + GB_WT * M1s;           // raw x [16][F][p]
  float* W2s = Xs + GB_WT * pF;            // fc2W [K][M1]
  float* DR = W2s + K * M1;                // [16][16] dr (K <= 16)
  float* Ss = DR + GB_WT * 16;             // S_0 .. S_{n-1}
  float* Gs = Ss + n * pp2;                // gcW[(i,f)][h], row stride Hs (the dT B operand)
  float* red = Gs + 16 * GB_MAXNT * Hs;    // [2][GB_THREADS]
  float* xw = Rs;  // [GB_WAVES][GB_MAXNT * 2][256] dW_i partials, over Rs + DZs once both are dead
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool fac_grad = c.flags & (RC_LOSS_FORECAST | RC_LOSS_ADJ);
  const bool lab_on = (c.flags & RC_LOSS_FACTOR) && d.nsup > 0;
  // ---- register operands of dR (fc1W B[k = m][col = q], column tiles nq = wv + 4 j), requested
  // first so that their latency overlaps the staging
  float fR[GB_MAXNQ][16];
#pragma unroll
  for (int j = 0; j < GB_MAXNQ; ++j) {
    const int q = 16 * (wv + GB_WAVES * j) + l15;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const int m = 4 * ks + g;
      fR[j][ks] = (q < pH && m < M1) ? E[c.eo.fc1W + (int64_t)m * pH + q] : 0.f;
    }
  }
  // ---- stage the tile: T (node-major), R, raw x, S, gcW; zero past the batch
  const float* Tg = ws + c.wo.T + (int64_t)b0 * p * nF;
  const float* Rg = ws + c.wo.R + (int64_t)b0 * pH;
  const float* Xg = c.X + r * c.xr + ((c.row0 + b0) * d.T + (c.Lmax - F)) * p;
  const int pnF = p * nF;
  rc_stage_all(
      rc_seg<8>(GB_WT * pnF, [&](int e) { return e < nw * pnF ? Tg[e] : 0.f; },
                [&](int e, float v) {
                  const int w = e / pnF, rem = e - w * pnF, ch = rem / nF, col = rem - ch * nF;
                  Ts[ch * NSt + w * nFs + col] = v;
                }),
      rc_seg<8>(GB_WT * pH, [&](int e) { return e < nw * pH ? Rg[e] : 0.f; },
                [&](int e, float v) {
                  const int w = e / pH;
                  Rs[w * pHs + (e - w * pH)] = v;
                }),
      rc_seg<4>(GB_WT * pF, [&](int e) {
        const int w = e / pF;
        return w < nw ? Xg[(int64_t)w * d.T * p + (e - w * pF)] : 0.f;
      }, [&](int e, float v) { Xs[e] = v; }),
      rc_seg<4>(GB_WT * M1, [&](int e) {
        const int w = e / M1;
        return w < nw ? ws[c.wo.f1 + (int64_t)(b0 + w) * M1 + (e - w * M1)] : 0.f;
      }, [&](int e, float v) {
        const int w = e / M1;
        DF1[w * M1s + (e - w * M1)] = v;
      }),
      rc_seg<2>(K * M1, [&](int e) { return E[c.eo.fc2W + e]; }, [&](int e, float v) { W2s[e] = v; }),
      rc_seg<2>(n * pp2, [&](int e) { return ws[c.wo.S + e]; }, [&](int e, float v) { Ss[e] = v; }),
      rc_seg<4>(16 * GB_MAXNT * Hs, [&](int e) {
        const int col = e / Hs, h = e - col * Hs;
        return (col < nF && h < H) ? E[c.eo.gcW + col * H + h] : 0.f;
      }, [&](int e, float v) { Gs[e] = v; }));
  gb_zero_pad(DZs, 16 * p, H, Hs, NSz);
  gb_zero_pad(Ts, 16 * p, nF, nFs, NSt);
  // ---- dr (one thread per (window, factor)): channel partials in channel order
  if (tid < GB_WT * K) {
    const int w = tid / K, k = tid - w * K, b = b0 + w;
    float v = 0.f;
    if (w < nw) {
      float t = 0.f;
      if (fac_grad)
        for (int j = 0; j < p; ++j) t += ws[c.wo.dwp + ((int64_t)j * d.Bmax + b) * K + k];
      const float y = lab_on ? c.lab[r * c.labr + (c.row0 + b) * K + k] : 0.f;
      v = rc_emb_draw(c, r, k, ws[c.wo.w + (int64_t)b * K + k], t, y);
      ws[c.wo.edr + (int64_t)b * K + k] = v;
    }
    DR[w * 16 + k] = v;
  }
  __syncthreads();
  // ---- df1 = [f1 > 0] dr fc2W (k ascending), in place over f1
  for (int e = tid; e < GB_WT * M1; e += GB_THREADS) {
    const int w = e / M1, m = e - w * M1;
    float gg = 0.f;
    for (int k = 0; k < K; ++k) gg = fmaf(DR[w * 16 + k], W2s[k * M1 + m], gg);
    gg = DF1[w * M1s + m] > 0.f ? gg : 0.f;
    DF1[w * M1s + m] = gg;
    if (w < nw) ws[c.wo.edf1 + (int64_t)(b0 + w) * M1 + m] = gg;
  }
  __syncthreads();
  // ---- dR = df1 fc1W, dZ = [R > 0] dR (node-major)
#pragma unroll
  for (int j = 0; j < GB_MAXNQ; ++j) {
    const int nq = wv + GB_WAVES * j;
    if (nq < s.nqt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* a = DF1 + l15 * M1s + g;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) acc = gb_mfma(a[4 * ks], fR[j][ks], acc);
      const int q = 16 * nq + l15;
      if (q < pH) {
        const int ch = q / H, h = q - ch * H;
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int w = 4 * g + reg;
          DZs[ch * NSz + w * Hs + h] = Rs[w * pHs + q] > 0.f ? acc[reg] : 0.f;
        }
      }
    }
  }
  __syncthreads();
  // ---- dT = dZ gcW^T for the wave's nodes; dW_i partial = T^T dZ over the same rows
  f32x4 aW[GB_MAXNT][2];
#pragma unroll
  for (int i = 0; i < GB_MAXNT; ++i) aW[i][0] = aW[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ch = wv; ch < p; ch += GB_WAVES) {
#pragma unroll
    for (int nt = 0; nt < GB_MAXNT; ++nt) {
      if (nt < s.ntt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* a = DZs + ch * NSz + l15 * Hs + g;
        const float* bg = Gs + (16 * nt + l15) * Hs + g;  // B[k = h][col = (i,f)] = gcW[(i,f)][h]
#pragma unroll
        for (int ks = 0; ks < GB_MAXKH; ++ks)
          if (ks < s.nkh) acc = gb_mfma(a[4 * ks], bg[4 * ks], acc);
        const int col = 16 * nt + l15;
        if (col < nF)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) DTs[ch * NSt + (4 * g + reg) * nFs + col] = acc[reg];
      }
    }
#pragma unroll
    for (int mi = 0; mi < GB_MAXNT; ++mi) {
      if (mi < s.ntt) {
        const float* aa = Ts + ch * NSt + g * nFs + 16 * mi + l15;  // A = T^T: rows (i,f), k = windows
#pragma unroll
        for (int hj = 0; hj < 2; ++hj) {
          const float* bb = DZs + ch * NSz + g * Hs + 16 * hj + l15;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) aW[mi][hj] = gb_mfma(aa[4 * ks * nFs], bb[4 * ks * Hs], aW[mi][hj]);
        }
      }
    }
  }
  __syncthreads();  // every wave is done with Rs / DZs: xw takes their place
#pragma unroll
  for (int mi = 0; mi < GB_MAXNT; ++mi)
#pragma unroll
    for (int hj = 0; hj < 2; ++hj)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) xw[((wv * GB_MAXNT + mi) * 2 + hj) * 256 + reg * 64 + lane] = aW[mi][hj][reg];
  __syncthreads();
  // ---- dW_i slot `tile`: the waves' partials added in wave order
  const int nFH = nF * H;
  for (int e = tid; e < GB_MAXNT * 2 * 256; e += GB_THREADS) {
    const int tl = e >> 8, reg = (e >> 6) & 3, ln = e & 63, mi = tl >> 1, hj = tl & 1;
    const int row = 16 * mi + 4 * (ln >> 4) + reg, h = 16 * hj + (ln & 15);  // row = (i, f)
    if (row < nF && h < H) {
      float t = 0.f;
      for (int w = 0; w < GB_WAVES; ++w) t += xw[((w * GB_MAXNT + mi) * 2 + hj) * 256 + reg * 64 + ln];
      ws[c.wo.dWi + (int64_t)tile * nFH + row * H + h] = t;
    }
  }
  // ---- dx_bn = dT_0 + sum_{i>=1} S_i^T dT_i (c' ascending, then i); BatchNorm affine partials over
  // the tile's (node, window) rows, threads (f, slot), slots added in order
  const int bf = tid % F, bsl = tid / F, nbsl = GB_THREADS / F;
  float ag = 0.f, ab = 0.f;
  if (bsl < nbsl) {
    float bmean, binv;
    gb_bn(c, r, bf, bmean, binv);
    for (int row = bsl; row < p * GB_WT; row += nbsl) {
      const int ch = row / GB_WT, w = row - ch * GB_WT;
      float dx = DTs[ch * NSt + w * nFs + bf];
      for (int i = 1; i < n; ++i)
        for (int cp = 0; cp < p; ++cp) dx = fmaf(Ss[(i * p + cp) * p + ch], DTs[cp * NSt + w * nFs + i * F + bf], dx);
      const float x = Xs[(w * F + bf) * p + ch];
      if (w < nw) {  // windows past the batch have dT = 0: skipped, so their (x - mean) terms add nothing
        ag += dx * ((x - bmean) * binv);
        ab += dx;
      }
    }
  }
  red[tid] = ag;
  red[GB_THREADS + tid] = ab;
  // ---- dS_i[ch][c'] slot `tile` = sum_w sum_f dT_i[ch][w][f] x_bn[c'][w][f] on the matrix cores: one
  // 16 x 16 tile per power (A = dT_i rows ch, B = x_bn^T columns c', k = (w, f), F % 4 == 0), wave wv
  // over windows 4 wv .. 4 wv + 3 (w, then f ascending), the four waves' partials added in wave order
  {
    const int chA = l15 < p ? l15 : p - 1;
    const float ma = l15 < p ? 1.f : 0.f;
    float* dsx = DZs;  // [GB_WAVES][n - 1][256], DZs is dead now
    for (int i = 1; i < n; ++i) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int w = 4 * wv; w < 4 * wv + 4; ++w) {
        const float* a = DTs + chA * NSt + w * nFs + i * F + g;
        const float* bq = Ts + chA * NSt + w * nFs + g;
        for (int j = 0; j < F / 4; ++j) acc = gb_mfma(ma * a[4 * j], ma * bq[4 * j], acc);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) dsx[(wv * (n - 1) + (i - 1)) * 256 + reg * 64 + lane] = acc[reg];
    }
  }
  __syncthreads();
  for (int e = tid; e < (n - 1) * 256; e += GB_THREADS) {
    const int i1 = e >> 8, reg = (e >> 6) & 3, ln = e & 63;
    const int ch = 4 * (ln >> 4) + reg, cp = ln & 15;
    if (ch < p && cp < p) {
      float t = 0.f;
      for (int w = 0; w < GB_WAVES; ++w) t += DZs[(w * (n - 1) + i1) * 256 + reg * 64 + ln];
      ws[c.wo.dS + (int64_t)tile * c.dsS + pp2 + i1 * pp2 + ch * p + cp] = t;
    }
  }
  if (tid < F) {
    float ga = 0.f, gb = 0.f;
    for (int q = 0; q < nbsl; ++q) {
      ga += red[q * F + tid];
      gb += red[GB_THREADS + q * F + tid];
    }
    ws[c.wo.dgb + ((int64_t)tile * 2) * F + tid] = ga;
    ws[c.wo.dgb + ((int64_t)tile * 2 + 1) * F + tid] = gb;
  }
}

// ------------------------------------------------------------------------------------------
// Weight gradients over the whole batch, one 512-thread workgroup per replica (windows ascending):
//   dfc1W[m][q] = sum_b df1[b][m] R[b][q]: wave wv owns the q tiles wv + 8 j and all four m tiles
//   (accumulated over the batch in registers), operands read from the workspace (L2) one
//   16-window chunk ahead of the matrix-core work;
//   dfc2W[k][m] = sum_b dr[b][k] relu(f1[b][m]), dfc2b[k] = sum_b dr[b][k], dfc1b[m] = sum_b df1[b][m].
#define GB_DFC_WAVES (GB_DFC_THREADS / 64)
#define GB_DFC_NQ 3  // p*H <= 8 * 3 * 16 = 384
__global__ __launch_bounds__(GB_DFC_THREADS) void k_gemb_dfc1(StepCtx c) {
  rc_critical_priority();
  const GbShape s(c.d);
  const int r = rc_rep(c, blockIdx.y);
  const int M1 = s.M1, pH = s.pH, K = s.K, B = c.B;
  float* ws = c.ws + r * c.wss;
  const float* df1 = ws + c.wo.edf1;
  const float* R = ws + c.wo.R;
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  f32x4 acc[4][GB_DFC_NQ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < GB_DFC_NQ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // operands of one 16-window chunk: A = df1^T (rows m = 16 mi + l15, k = window b0 + 4 ks + g),
  // B = R (k = window, column q = 16 nq + l15); windows past B read as 0
  struct Chunk {
    float a[4][4], b[4][GB_DFC_NQ];
  };
  auto load = [&](int b0, Chunk& ch) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int b = b0 + 4 * ks + g;
      const bool in = b < B;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) ch.a[ks][mi] = in ? df1[(int64_t)b * M1 + 16 * mi + l15] : 0.f;
#pragma unroll
      for (int j = 0; j < GB_DFC_NQ; ++j) {
        const int q = 16 * (wv + GB_DFC_WAVES * j) + l15;
        ch.b[ks][j] = (in && q < pH) ? R[(int64_t)b * pH + q] : 0.f;
      }
    }
  };
  Chunk cur, nxt;
  load(0, cur);
  for (int b0 = 0; b0 < B; b0 += GB_WT) {
    if (b0 + GB_WT < B) load(b0 + GB_WT, nxt);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int j = 0; j < GB_DFC_NQ; ++j)
        if (wv + GB_DFC_WAVES * j < s.nqt)
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) acc[mi][j] = gb_mfma(cur.a[ks][mi], cur.b[ks][j], acc[mi][j]);
    cur = nxt;
  }
#pragma unroll
  for (int j = 0; j < GB_DFC_NQ; ++j) {
    const int q = 16 * (wv + GB_DFC_WAVES * j) + l15;
    if (q < pH)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) ws[c.wo.gfc1 + (int64_t)(16 * mi + 4 * g + reg) * pH + q] = acc[mi][j][reg];
  }
  // fc2 / fc2-bias / fc1-bias, windows ascending, through 32-window chunks staged in LDS
  const float* dr = ws + c.wo.edr;
  const float* f1 = ws + c.wo.f1;
  const int nfc = K * M1 + K + M1;
  __shared__ float cdr[32 * 16], cf1[32 * 64], cdf[32 * 64];
  float t0 = 0.f, t1 = 0.f, t2 = 0.f;  // outputs tid, tid + 512, tid + 1024 (nfc <= 16 * 64 + 80)
  auto acc_out = [&](int e, int nb, float& t) {
    if (e >= nfc) return;
    if (e < K * M1) {
      const int k = e / M1, m = e - k * M1;
      for (int b = 0; b < nb; ++b) t = fmaf(cdr[b * 16 + k], cf1[b * 64 + m], t);
    } else if (e < K * M1 + K) {
      const int k = e - K * M1;
      for (int b = 0; b < nb; ++b) t += cdr[b * 16 + k];
    } else {
      const int m = e - K * M1 - K;
      for (int b = 0; b < nb; ++b) t += cdf[b * 64 + m];
    }
  };
  for (int b0 = 0; b0 < B; b0 += 32) {
    const int nb = min(32, B - b0);
    __syncthreads();
    for (int e = tid; e < nb * K; e += GB_DFC_THREADS) cdr[(e / K) * 16 + e % K] = dr[(int64_t)b0 * K + e];
    for (int e = tid; e < nb * M1; e += GB_DFC_THREADS) {
      cf1[(e / M1) * 64 + e % M1] = fmaxf(f1[(int64_t)b0 * M1 + e], 0.f);
      cdf[(e / M1) * 64 + e % M1] = df1[(int64_t)b0 * M1 + e];
    }
    __syncthreads();
    acc_out(tid, nb, t0);
    acc_out(tid + GB_DFC_THREADS, nb, t1);
    acc_out(tid + 2 * GB_DFC_THREADS, nb, t2);
  }
  if (tid < nfc) ws[c.wo.gfc + tid] = t0;
  if (tid + GB_DFC_THREADS < nfc) ws[c.wo.gfc + tid + GB_DFC_THREADS] = t1;
  if (tid + 2 * GB_DFC_THREADS < nfc) ws[c.wo.gfc + tid + 2 * GB_DFC_THREADS] = t2;
}

}  // namespace

// The batched kernels take a packed grid's embedder when its shapes fit them: small node counts
// and widths (the D4IC-shaped grid: p = 10, n*F = 40, H = 30, p*H = 300).  REDCLIFF_EMB_PATH=batched
// forces them (tests: single fits on the same path as a pack), =gemm / =fused the other paths.
bool rc_emb_batched_fits(const RedcliffDims& d) {
  const GbShape s(d);
  return d.p <= 16 && d.M1 == 64 && d.K <= 16 && s.nF <= 16 * GB_MAXNT && d.H <= 4 * GB_MAXKH &&
         s.nqt <= GB_WAVES * GB_MAXNQ && s.nqt <= GB_DFC_WAVES * GB_DFC_NQ && s.nkf <= GB_MAXKF && d.F <= GB_THREADS &&
         gb_ntiles(d.Bmax) <= 64 && (int64_t)gb_lds_bwd(s) <= RC_LDS_MAX_FLOATS && d.F % 4 == 0 &&
         (d.n - 1) * 256 * GB_WAVES <= d.p * s.NSz &&  // dS partials over DZs
         GB_WAVES * GB_MAXNT * 2 * 256 <= GB_WT * s.pHs + s.p * s.NSz &&  // xw over Rs + DZs
         (int64_t)gb_lds_fwd(s) <= RC_LDS_MAX_FLOATS;
}

// record slots of the final kernel's sums (rc_emb_partial_layout)
int rc_emb_batched_slots(int B) { return gb_ntiles(B); }

#ifndef RC_EMB_BATCHED_R
#define RC_EMB_BATCHED_R 0  // default off until measured faster than the GEMM chain (REDCLIFF_EMB_PATH=batched)
#endif
bool rc_emb_use_batched(const RedcliffDims& d) {
  const char* v = getenv("REDCLIFF_EMB_PATH");
  if (v && !strcmp(v, "batched")) return rc_emb_batched_fits(d);
  if (v && (!strcmp(v, "gemm") || !strcmp(v, "fused"))) return false;
  return RC_EMB_BATCHED_R > 0 && d.R >= RC_EMB_BATCHED_R && rc_emb_batched_fits(d);
}

int rc_launch_emb_fwd_batched(const StepCtx& c, hipStream_t s) {
  const GbShape sh(c.d);
  const size_t lds = sizeof(float) * (size_t)gb_lds_fwd(sh);
  int e = rc_lds_optin(k_gemb_fwd, lds, "k_gemb_fwd LDS");
  if (e) return e;
  hipLaunchKernelGGL(k_gemb_fwd, dim3(gb_ntiles(c.B), c.nrep), dim3(GB_THREADS), lds, s, c);
  return rc_check(hipGetLastError(), "k_gemb_fwd");
}

int rc_launch_emb_bwd_batched(const StepCtx& c, hipStream_t s) {
  const GbShape sh(c.d);
  const int nt = gb_ntiles(c.B);
  if (c.dwN != nt || c.dsN != nt || c.dgN != nt) {
    rc_set_error("batched embedder backward: partial layout of %d / %d / %d slots, %d expected", c.dwN, c.dsN, c.dgN, nt);
    return REDCLIFF_EINVAL;
  }
  const size_t lds = sizeof(float) * (size_t)gb_lds_bwd(sh);
  int e = rc_lds_optin(k_gemb_bwd, lds, "k_gemb_bwd LDS");
  if (e) return e;
  hipLaunchKernelGGL(k_gemb_bwd, dim3(nt, c.nrep), dim3(GB_THREADS), lds, s, c);
  if ((e = rc_check(hipGetLastError(), "k_gemb_bwd"))) return e;
  hipLaunchKernelGGL(k_gemb_dfc1, dim3(1, c.nrep), dim3(GB_DFC_THREADS), 0, s, c);
  return rc_check(hipGetLastError(), "k_gemb_dfc1");
}
