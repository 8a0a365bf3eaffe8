// rc_embed.hip -- DGCNN factor-score embedder on gfx950: forward, backward, optimizer
// finalisation, Chebyshev supports and BatchNorm batch statistics.
//
// Reference: models/redcliff_factor_score_embedders.py:335-392 (DGCNN_Embedder),
// models/dgcnn.py:15-64 (DGCNN_Model) and the torcheeg 1.1.3 DGCNN it wraps
// (restated in oracle/torcheeg_dgcnn.py):
//   x_bn = BN1(x)                      BatchNorm1d over F features, stats over (B, p)
//   L    = D^-1/2 relu(A) D^-1/2       normalize_A
//   Z_b  = sum_i (S_i x_bn_b) W_i      S = [I, L, L^2, ...]  (Chebynet)
//   w_b  = fc2(relu(fc1(vec(relu(Z_b)))))
// One batch_update runs the embedder 3x on the same window (forward + two GC calls,
// ...withStateSmoothing.py:844-856); the math is identical, so it is evaluated once,
// the three upstream gradients are summed, and the BatchNorm running statistics are
// advanced n_bn_updates (=3) times.
#include <cstdlib>
#include <cstring>

#include "rc_common.h"
#include "rc_fac_bwd.h"

#ifndef RC_MERGED_LEAD_SPLIT
#define RC_MERGED_LEAD_SPLIT 1  // k_bwd_merged: the factor leads' update parts as their own workgroups
#endif

namespace {

// BatchNorm scale/shift exactly as torch's CPU kernel forms them
// (batch_norm_cpu_collect_linear_and_constant_terms): y = x*alpha + beta.
// BatchNorm affine of feature f (F <= 64 < RC_BLOCK: thread f): bn_affine_load requests the
// operands, bn_affine_store forms alpha / beta (and the mean / invstd the backward needs) once
// they are in -- split so that the node workgroup's staging loads go out in between.
struct BnOperands {
  double m, v;
  float g, b;
};
__device__ inline void bn_affine_load(const StepCtx& c, int r, const float* E, int f, BnOperands& q) {
  const RedcliffDims& d = c.d;
  if (c.flags & RC_BN_TRAIN) {
    const double* st = c.bns + r * c.bnsr;
    q.m = st[f];
    q.v = st[d.F + f];
  } else {
    q.m = c.rm[r * d.F + f];
    q.v = c.rv[r * d.F + f];
  }
  q.g = E[c.eo.bnw + f];
  q.b = E[c.eo.bnb + f];
}
__device__ inline void bn_affine_store(const StepCtx& c, int r, int f, const BnOperands& q, float* alpha, float* beta,
                                       float* mean_out, float* inv_out) {
  float mean, inv;
  if (c.flags & RC_BN_TRAIN) {
    mean = (float)q.m;
    inv = (float)(1.0 / sqrt(q.v + c.hyp[r].bn_eps));
  } else {
    mean = (float)q.m;
    inv = 1.0f / sqrtf((float)q.v + (float)c.hyp[r].bn_eps);
  }
  const float a = inv * q.g;
  alpha[f] = a;
  beta[f] = q.b - mean * a;
  if (mean_out) mean_out[f] = mean;
  if (inv_out) inv_out[f] = inv;
}

// dL/d(raw embedder output) of one window / factor: the factor-side gradient gw (sum of
// the per-channel partials written by the factor kernel) plus the supervised-score MSE and
// factor-weight L1 terms, through the optional sigmoid (compute_loss, :633-666).
__device__ inline float draw_value(const StepCtx& c, int r, int k, float raw, float gw, float y) {
  const RedcliffDims& d = c.d;
  const int K = d.K, nsup = d.nsup;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const int ncol = nsup > 0 ? nsup : K;  // columns of factor_scores[0] (state_label_preds)
  const float weff = sig ? rc_sigmoid(ecc * raw) : raw;
  float graw = sig ? gw * ecc * weff * (1.f - weff) : gw;
  if (k < ncol) {
    // score used by the factor MSE and the L1: class logits when supervised, else w
    const float sl = nsup > 0 ? (sig ? rc_sigmoid(raw) : raw) : weff;
    float gsl = 0.f;
    if ((c.flags & RC_LOSS_FACTOR) && nsup > 0) gsl += hy.c_factor * (2.f / (float)(c.Bg * nsup)) * (sl - y);
    if (c.flags & RC_LOSS_FWL1) gsl += hy.c_fwl1 * rc_sign(sl);
    if (nsup > 0)
      graw += sig ? gsl * sl * (1.f - sl) : gsl;
    else
      graw += sig ? gsl * ecc * weff * (1.f - weff) : gsl;
  }
  return graw;
}

// ------------------------------------------------------------------------------------------
// Cosine similarity of the lag-free conditional GC estimates (metrics.py:342-381), a value
// only (the reference's torch.Tensor(list) drops its gradient):
//   v_bk[r][c] = w_bk * G0[k][r][c] + A[c][r] - I[r][c],  cosb[b] = sum_{k1<k2} cos(v_bk1, v_bk2)
// grid (ceil(B / COS_WPW), R), one WAVE per COS_WPV windows: the workgroup stages the replica's
// G0 stack and A^T in LDS once (K p^2 + p^2 floats; read from global memory when they do not
// fit), then each wave runs its windows with no further barrier.  The arithmetic is that of a 256-thread
// workgroup per window: virtual thread (vw, lane) sums the elements e = 64 vw + lane + 256 i,
// each virtual wave's sum is lane 0's butterfly sum, the four are added in order, the pairs'
// cosines in order in double -- bit for bit the one-window-per-workgroup form.
#define COS_WPV 1                             // windows per wave (2: no faster at R = 128 D4IC)
#define COS_WPW (COS_WPV * (RC_BLOCK / 64))  // windows per workgroup
#define COS_LDS 8192  // staged floats
__global__ __launch_bounds__(RC_BLOCK) void k_cos_values(StepCtx c) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y), K = d.K, p = d.p, pp2 = p * p;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* G0g = ws + c.wo.G0;
  const float* A = E + c.eo.A;
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const int npair = K * (K - 1) / 2;
  extern __shared__ float st[];  // (K + 1) p^2 floats when staged (rc_launch_cos_values)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool staged = (K + 1) * pp2 <= COS_LDS;
  const float* G0 = staged ? st : G0g;
  float* At = st + K * pp2;  // At[e] = A[c][r] for e = r * p + c (staged)
  if (staged) {
    for (int e = tid; e < K * pp2; e += RC_BLOCK) st[e] = G0g[e];
    for (int e = tid; e < pp2; e += RC_BLOCK) {
      const int rr = e / p, cc = e - rr * p;
      At[e] = A[cc * p + rr];
    }
  }
  __syncthreads();
  // virtual waves holding elements (the others add exact +0 sums: one +0.f stands for them)
  const int nvw = (pp2 + 63) / 64 < RC_BLOCK / 64 ? (pp2 + 63) / 64 : RC_BLOCK / 64;
  // p^2 <= RC_BLOCK: one element per virtual thread, its pair-independent terms kept in registers
  const bool one = pp2 <= RC_BLOCK;
  float atv[RC_BLOCK / 64], eyev[RC_BLOCK / 64];
#pragma unroll
  for (int vw = 0; vw < RC_BLOCK / 64; ++vw) {
    const int e = vw * 64 + lane;
    atv[vw] = 0.f;
    eyev[vw] = 0.f;
    if (one && e < pp2) {
      const int rr = e / p, cc = e - rr * p;
      atv[vw] = staged ? At[e] : A[cc * p + rr];
      eyev[vw] = (rr == cc ? 1.f : 0.f);
    }
  }
  for (int b = (blockIdx.x * (RC_BLOCK / 64) + wv) * COS_WPV, bend = min(c.B, b + COS_WPV); b < bend; ++b) {
    float wl = 0.f;  // lane k < K: w_bk
    if (lane < K) {
      const float raw = ws[c.wo.w + (int64_t)b * K + lane];
      wl = sig ? rc_sigmoid(ecc * raw) : raw;
    }
    double t = 0.0;
    for (int q = 0; q < npair; ++q) {
      int k1 = 0, rem = q;
      while (rem >= K - 1 - k1) { rem -= K - 1 - k1; ++k1; }
      const int k2 = k1 + 1 + rem;
      const float w1 = __shfl(wl, k1, 64), w2 = __shfl(wl, k2, 64);
      const float* g1 = G0 + (int64_t)k1 * pp2;
      const float* g2 = G0 + (int64_t)k2 * pp2;
      float dot = 0.f, n1 = 0.f, n2 = 0.f;
#pragma unroll
      for (int vw = 0; vw < RC_BLOCK / 64; ++vw) {
        if (vw >= nvw) break;
        float pd = 0.f, p1 = 0.f, p2 = 0.f;
        if (one) {
          const int e = vw * 64 + lane;
          if (e < pp2) {
            const float v1 = (w1 * g1[e] + atv[vw]) - eyev[vw];
            const float v2 = (w2 * g2[e] + atv[vw]) - eyev[vw];
            pd += v1 * v2;  // fmaf onto +0, as the strided loop's first step (not a bare product)
            p1 += v1 * v1;
            p2 += v2 * v2;
          }
        } else {
          for (int e = vw * 64 + lane; e < pp2; e += RC_BLOCK) {
            const int rr = e / p, cc = e - rr * p;
            const float at = staged ? At[e] : A[cc * p + rr];
            const float eye = (rr == cc ? 1.f : 0.f);
            const float v1 = (w1 * g1[e] + at) - eye;
            const float v2 = (w2 * g2[e] + at) - eye;
            pd += v1 * v2;
            p1 += v1 * v1;
            p2 += v2 * v2;
          }
        }
        dot += __shfl(rc_wave_sum(pd), 0, 64);
        n1 += __shfl(rc_wave_sum(p1), 0, 64);
        n2 += __shfl(rc_wave_sum(p2), 0, 64);
      }
      if (nvw < RC_BLOCK / 64) {
        dot += 0.f;
        n1 += 0.f;
        n2 += 0.f;
      }
      const float eps2 = 1e-16f;
      t += (double)(dot / sqrtf(fmaxf(n1, eps2) * fmaxf(n2, eps2)));
    }
    if (lane == 0) reinterpret_cast<double*>(ws + c.wo.cosb)[b] = t;
  }
}

// ------------------------------------------------------------------------------------------
// K3 head workgroup (launched only for loss values / the confusion matrix): the
// coefficient-normalised loss terms of validate_training and the factor-score confusion.
__device__ __forceinline__ void emb_bwd_head(const StepCtx& c, int r, float* sm) {
  const RedcliffDims& d = c.d;
  const int K = d.K, B = c.B, p = d.p, nsup = d.nsup;
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int tid = threadIdx.x;
  float* red = sm;                                        // [8]
  double* dred = reinterpret_cast<double*>(sm + 8);       // [8]
  int* hist = reinterpret_cast<int*>(sm + 32);            // [nsup][nsup]
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const float* wraw = ws + c.wo.w;
  const int ncol = nsup > 0 ? nsup : K;
  if (c.flags & RC_VALUES) {
    // supervised MSE and factor-weight L1 (values)
    double fsum = 0.0, l1 = 0.0;
    for (int e = tid; e < B * K; e += RC_BLOCK) {
      const int b = e / K, k = e - b * K;
      if (k >= ncol) continue;
      const float raw = wraw[(int64_t)b * K + k];
      const float sl = nsup > 0 ? (sig ? rc_sigmoid(raw) : raw) : (sig ? rc_sigmoid(ecc * raw) : raw);
      l1 += fabsf(sl);
      if (nsup > 0) {
        const float y = c.lab[r * c.labr + (c.row0 + b) * K + k];
        fsum += (double)(sl - y) * (double)(sl - y);
      }
    }
    fsum = rc_block_sum_d(fsum, dred);
    l1 = rc_block_sum_d(l1, dred);
    // cosine-similarity penalty: per-window sums from k_cos_values (ws.cosb), summed here
    double cs = 0.0;
    if (K > 1) {
      const double* cb = reinterpret_cast<const double*>(ws + c.wo.cosb);
      for (int b = tid; b < B; b += RC_BLOCK) cs += cb[b];
    }
    cs = (K > 1) ? rc_block_sum_d(cs, dred) : 0.0;
    if (tid == 0) {
      const float* lp = ws + c.wo.lossp;
      double fore = 0.0;
      for (int j = 0; j < p; ++j) fore += (double)lp[j] / (double)c.Bg;
      fore *= hy.c_forecast;
      double adj = 0.0;
      for (int e = 0; e < K * p; ++e) adj += lp[p + e];
      const double factor = nsup > 0 ? hy.c_factor * fsum / (double)(c.Bg * nsup) : 0.0;
      const double fwl1 = hy.c_fwl1 * (l1 - 1.0);
      const double cosv = hy.c_cos * cs;
      const double smooth = 0.0;  // num_sims == 1
      const double combo = fore + factor + fwl1 + smooth + adj + (K > 1 ? cosv : 0.0);
      double* acc = c.acc + r * 8;
      acc[ACC_FORECAST] += hy.c_forecast > 0.f ? fore / hy.c_forecast : fore;
      acc[ACC_FACTOR] += hy.c_factor > 0.f ? factor / hy.c_factor : factor;
      acc[ACC_COS] += (K > 1) ? (hy.c_cos > 0.f ? cosv / hy.c_cos : cosv) : 0.0;
      acc[ACC_FWL1] += hy.c_fwl1 > 0.f ? fwl1 / hy.c_fwl1 : fwl1;
      acc[ACC_SMOOTH] += 0.0;
      acc[ACC_ADJ] += hy.c_adj > 0.f ? adj / hy.c_adj : adj;
      acc[ACC_COMBO] += combo;
      acc[ACC_BATCHES] += 1.0;
    }
  }
  if ((c.flags & RC_CONFUSION) && nsup > 0) {
    // np.argmax (first maximum) of state_label_preds[0] and of the labels (:801-803);
    // integer counts, so the LDS atomics are order-independent
    for (int e = tid; e < nsup * nsup; e += RC_BLOCK) hist[e] = 0;
    __syncthreads();
    for (int b = tid; b < B; b += RC_BLOCK) {
      int pred = 0, lab = 0;
      float best = 0.f, bestl = 0.f;
      for (int k = 0; k < nsup; ++k) {
        const float raw = wraw[(int64_t)b * K + k];
        const float sl = sig ? rc_sigmoid(raw) : raw;
        const float y = c.lab[r * c.labr + (c.row0 + b) * K + k];
        if (k == 0 || sl > best) { best = sl; pred = k; }
        if (k == 0 || y > bestl) { bestl = y; lab = k; }
      }
      atomicAdd(&hist[lab * nsup + pred], 1);
    }
    __syncthreads();
    int* conf = c.conf + (int64_t)r * nsup * nsup;
    for (int e = tid; e < nsup * nsup; e += RC_BLOCK) conf[e] += hist[e];
  }
}

// K3 node workgroup (node c, hidden columns [h0, h0+HC), windows [wb*WPB, wb*WPB+WPB)):
// dL/dw_raw of its windows, dL/dfc1 of the chunk's columns, graph-conv output gradient dZ,
// and partial sums over its windows of dfc1W, dW_i, dS_i[c][:], the BatchNorm affine
// gradients and (node 0, chunk 0) the fc2 / fc1-bias gradients.  The windows are walked in
// LDS sub-blocks of BC (register accumulators carry over), so large p*F windows keep the
// partial records few.  The partials of the nbw window blocks of one (node, chunk) are
// combined in fixed order by k_emb_combine (c.defer == 1, the default), by k_emb_final in
// place (2), or by the block that arrives last (0: agent-scope release / ticket / acquire,
// cdna_hip_programming.md §6 Guideline 16).  The first sub-block's inputs and the
// fixed operands are staged by one multi-segment pass (one memory latency for everything).
template <bool MULTI, bool LATE = false>
__device__ __forceinline__ void emb_bwd_node(const StepCtx& c, int r, int node, int ch, int wb, int BC, int WPB, float* sm,
                             const unsigned* wait_cnt = nullptr, unsigned wait_target = 0) {
  const RedcliffDims& d = c.d;
  const int K = d.K, M1 = d.M1, B = c.B, p = d.p, H = d.H, F = d.F, n = d.n;
  const int pH = p * H, pF = p * F, nF = n * F, HC = EMB_HC, HP = EMB_HC + 1;
  const int h0 = ch * HC, hc = min(HC, H - h0);
  const int nch = rc_nchunk(d);
  // (the host's window blocking in the single-sub-block kernels; the multi-sub-block merged kernel
  // keeps the divisions -- the two more live scalars there cost it a wave per SIMD: 244 -> 256 VGPRs)
  const int nbw = (!MULTI && WPB == c.ewpb) ? c.enbw : (B + WPB - 1) / WPB, nbw_max = MULTI ? rc_emb_nbw(d) : c.enbwm;
  const int wend = min(B, (wb + 1) * WPB);
  const int grp = node * nch + ch;
  const bool head_grads = (grp == 0);  // fc2 / fc1-bias partials ride on group 0
  float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const int tid = threadIdx.x;

  float* dr = sm;                        // [BC][K]
  float* wrl = dr + BC * K;              // [BC][K]   raw embedder output
  float* labl = wrl + BC * K;            // [BC][K]   labels
  float* dwl = labl + BC * K;            // [BC][K]   factor-side dL/dw (sum over channels)
  float* fc2s = dwl + BC * K;            // [K][M1]
  float* FW = fc2s + K * M1;             // [M1][HC]  fc1 columns of the chunk
  float* WiC = FW + M1 * HC;             // [n][F][HC+1]
  float* Srow = WiC + nF * HP;           // [n][p]    row `node` of each support
  float* rs = Srow + n * p;              // [4]       row sums
  int* tk = reinterpret_cast<int*>(rs + 4);  // [4]   arrival ticket broadcast
  float* alpha = rs + 8;                 // [F]
  float* beta = alpha + F;               // [F]
  float* mean = beta + F;                // [F]
  float* inv = mean + F;                 // [F]
  float* red = inv + F;                  // [RC_BLOCK]
  float* f1r = red + RC_BLOCK;           // [BC][M1]  fc1 pre-activations
  float* df1c = f1r + BC * M1;           // [BC][M1]
  float* Rc = df1c + BC * M1;            // [BC][HC]
  float* dZc = Rc + BC * HC;             // [BC][HC]
  float* Tc = dZc + BC * HC;             // [BC][n][F]   T_i row `node`
  float* dTc = Tc + BC * nF;             // [BC][n][F]
  const bool late_x = LATE && rc_emb_late_x(d);
  float* xc = late_x ? f1r : dTc + BC * nF;  // [BC][p][F] raw window (late: over f1r .. Tc)

  const RcDiv32 dF(F, c.mg[RC_MG_F]), dp(p, c.mg[RC_MG_P]), dpF(pF, c.mg[RC_MG_PF]), dnF(nF, c.mg[RC_MG_NF]),
      dK(K, c.mg[RC_MG_K]), dM1(M1, c.mg[RC_MG_M1]);
  // trace builds: the node workgroup's own index (inside the merged launch the factor leads come first)
  const int pbx = wait_cnt ? (int)blockIdx.x - d.K * d.p : (int)blockIdx.x;
  (void)pbx;
  RC_PHASE(c.ws, c.wo.total, pbx, 33);
  // (single sub-block: the BatchNorm operands are requested here and stored after the staging
  // pass; the multi-sub-block kernel, at 256 registers, stores them at once -- six more live
  // registers there spilled into accumulation registers and cost it half its occupancy)
  BnOperands bnq{0.0, 0.0, 0.f, 0.f};
  if (tid < F) {
    bn_affine_load(c, r, E, tid, bnq);
    if (MULTI) bn_affine_store(c, r, tid, bnq, alpha, beta, mean, inv);
  }
  const bool fac_grad = c.flags & (RC_LOSS_FORECAST | RC_LOSS_ADJ);
  const bool lab_on = (c.flags & RC_LOSS_FACTOR) && d.nsup > 0;
  const float* f1 = ws + c.wo.f1;
  const float* Rg = ws + c.wo.R;
  const float* Tg = ws + c.wo.T;
  const float* S = ws + c.wo.S;
  const float* wraw = ws + c.wo.w;
  const float* dwp = ws + c.wo.dwp;

  // register accumulators over all sub-blocks of the workgroup's windows
  float afc[4] = {0.f, 0.f, 0.f, 0.f};     // dfc1W chunk: M1*HC <= 1024 -> 4 / thread
  float agf[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // group 0: dfc2W | dfc2b | dfc1b (< 5*256)
  float awi[16];                            // dW_i chunk: n*F*HC <= 4096 -> 16 / thread
#pragma unroll
  for (int k = 0; k < 16; ++k) awi[k] = 0.f;
  // Matrix-core form of the sub-block products (16-window sub-blocks, fc1 width <= 64, K <= 16,
  // n*F <= 256): df1, dZ, dT and the dfc1W / dW_i partials as v_mfma_f32_16x16x4_f32 tiles,
  // each an fmaf chain over its contraction index in ascending order; the partial-record
  // layout is the vector form's.  Lane l: l15 = l & 15, g = l >> 4; D rows 4 g + reg, column l15.
  const bool mf = !MULTI && BC == 16 && M1 <= 64 && K <= 16 && nF <= 256;  // single-sub-block workgroups
  const int lane = tid & 63, l15 = lane & 15, lg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (the matrix-core accumulators live in afc (dfc1W rows m in [16 wv, 16 wv + 16)) and awi
  // (dW_i row tiles wv + 4 i, 4 registers each): one register set for either form)
  const int nwi = (nF * HC + RC_BLOCK - 1) / RC_BLOCK;
  const int nout = K * M1 + K + M1;
  const int nS = (n - 1) * p;
  const int nslS = nS > 0 ? RC_BLOCK / nS : 0, oS = nS > 0 ? tid % nS : 0, slS = nS > 0 ? tid / nS : 1;
  const int nslF = RC_BLOCK / F, oF = tid % F, slF = tid / F;
  float aS = 0.f, aG = 0.f, aB = 0.f;

  // MULTI = false: one sub-block per workgroup (WPB == BC), the loop folds away
  const int nsub = MULTI ? (wend - wb * WPB + BC - 1) / BC : 1;
  for (int it = 0; it < nsub; ++it) {
    const int bw0 = wb * WPB + it * BC;
    const int nbc = min(BC, wend - bw0);
    // ---- stage the sub-block's windows (with the fixed operands on the first pass)
    auto sR = rc_seg<1>(nbc * HC, [&](int e) {
      const int s = e / HC, hh = e - s * HC;
      return hh < hc ? Rg[(int64_t)(bw0 + s) * pH + node * H + h0 + hh] : 0.f;
    }, [&](int e, float v) { Rc[e] = v; });
    auto sT = rc_seg<4>(nbc * nF, [&](int e) {
      const int s = dnF.div(e), rem = e - s * nF, i = dF.div(rem), f = rem - i * F;
      return Tg[(int64_t)(bw0 + s) * n * pF + i * pF + node * F + f];
    }, [&](int e, float v) { Tc[e] = v; });
    auto x_ld = [&](int e) {
      const int s = dpF.div(e), rem = e - s * pF;  // rem = f * p + cc (contiguous in the window row)
      return X[(c.row0 + bw0 + s) * d.T * p + (int64_t)(c.Lmax - F) * p + rem];
    };
    auto x_st = [&](int e, float v) {
      const int s = dpF.div(e), rem = e - s * pF, f = dp.div(rem), cc = rem - f * p;
      xc[s * pF + cc * F + f] = v;
    };
    auto sX = rc_seg<16>(late_x ? 0 : nbc * pF, x_ld, x_st);
    auto sF1 = rc_seg<4>(nbc * M1, [&](int e) { return f1[(int64_t)bw0 * M1 + e]; }, [&](int e, float v) { f1r[e] = v; });
    auto sW = rc_seg<1>(nbc * K, [&](int e) { return wraw[(int64_t)bw0 * K + e]; }, [&](int e, float v) { wrl[e] = v; });
    auto sL = rc_seg<1>(nbc * K, [&](int e) { return lab_on ? c.lab[r * c.labr + (c.row0 + bw0) * K + e] : 0.f; },
                        [&](int e, float v) { labl[e] = v; });
    // factor-side dL/dw of the sub-block's windows (sum of the p channel partials): four lanes
    // per (window, factor) item over every 4th channel; the first 64 items' loads are issued
    // here and summed after the staging pass, so the two latencies overlap
    const int ditem = tid >> 2, dg = tid & 3, nitem = nbc * K;
    float dv[16];
    auto dw_load = [&](int i0) {
      const int it2 = i0 + ditem, sw = dK.div(it2), kk = it2 - sw * K;
#pragma unroll
      for (int u = 0; u < 16; ++u) {  // p <= 64
        const int j = dg + 4 * u;
        const float* q = dwp + ((int64_t)j * d.Bmax + bw0 + sw) * K + kk;
        dv[u] = (fac_grad && it2 < nitem && j < p) ? (wait_cnt ? rc_load_sc1(q) : *q) : 0.f;
      }
    };
    auto dw_store = [&](int i0) {
      float t = 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) t += dv[u];
      t += __shfl_xor(t, 1);
      t += __shfl_xor(t, 2);
      if (dg == 0 && i0 + ditem < nitem) dwl[i0 + ditem] = t;
    };
    // the rounds after the first (nitem > 64: K > 4 at 16-window sub-blocks).  With p <= 16 four
    // channel slots per lane cover every channel, so all the remaining rounds' loads are in flight
    // together (one memory latency instead of one per round); same terms, same order, same sums
    auto dw_rest = [&]() {
      if (nitem <= RC_BLOCK / 4) return;
      if (!MULTI && p <= 16 && nitem <= RC_BLOCK) {  // (not at the multi-sub-block kernel's 256 registers)
        float dr4[3][4];
#pragma unroll
        for (int rd = 0; rd < 3; ++rd) {
          const int it2 = (rd + 1) * (RC_BLOCK / 4) + ditem, sw = dK.div(it2), kk = it2 - sw * K;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = dg + 4 * u;
            const float* q = dwp + ((int64_t)j * d.Bmax + bw0 + sw) * K + kk;
            dr4[rd][u] = (fac_grad && it2 < nitem && j < p) ? (wait_cnt ? rc_load_sc1(q) : *q) : 0.f;
          }
        }
#pragma unroll
        for (int rd = 0; rd < 3; ++rd) {
          const int it2 = (rd + 1) * (RC_BLOCK / 4) + ditem;
          float t = 0.f;
#pragma unroll
          for (int u = 0; u < 4; ++u) t += dr4[rd][u];
          t += __shfl_xor(t, 1);
          t += __shfl_xor(t, 2);
          if (dg == 0 && it2 < nitem) dwl[it2] = t;
        }
      } else {
        for (int i0 = RC_BLOCK / 4; i0 < nitem; i0 += RC_BLOCK / 4) {
          dw_load(i0);
          dw_store(i0);
        }
      }
    };
    // merged launch: the factor-side partials come from the same launch's factor-lead workgroups;
    // stage everything else first, then wait for them
    const bool wait_now = wait_cnt != nullptr && it == 0;
    if (!wait_now) dw_load(0);
    __syncthreads();  // the previous sub-block is done with the LDS tiles
    if (it == 0) {
      rc_stage_all(
          // (K M1 <= 1,024: one round; with one load per thread TST's 576 took three.  The
          // multi-sub-block kernel keeps one: its registers are at the limit)
          rc_seg<MULTI ? 1 : 4>(K * M1, [&](int e) { return E[c.eo.fc2W + e]; }, [&](int e, float v) { fc2s[e] = v; }),
          rc_seg<4>(M1 * HC, [&](int e) {
            const int m = e / HC, hh = e - m * HC;
            return hh < hc ? E[c.eo.fc1W + (int64_t)m * pH + node * H + h0 + hh] : 0.f;
          }, [&](int e, float v) { FW[e] = v; }),
          rc_seg<4>(nF * HC, [&](int e) {
            const int eh = e >> 4, i = dF.div(eh), f = eh - i * F, hh = e & 15;  // HC == 16
            return hh < hc ? E[c.eo.gcW + ((int64_t)i * F + f) * H + h0 + hh] : 0.f;
          }, [&](int e, float v) { WiC[(e / HC) * HP + e % HC] = v; }),
          rc_seg<1>(n * p, [&](int e) {
            const int i = dp.div(e), cc = e - i * p;
            return S[((int64_t)i * p + node) * p + cc];
          }, [&](int e, float v) { Srow[e] = v; }),
          sR, sT, sX, sF1, sW, sL);
  RC_PHASE(c.ws, c.wo.total, pbx, 44);  // (trace builds: the staging pass's loads are in)
#ifdef RC_STAGE_TWICE
      // timing experiment (trace builds): the window operands staged again -- warm caches and TLB
      rc_stage_all(sR, sT, sX, sF1, sW, sL);
  RC_PHASE(c.ws, c.wo.total, pbx, 47);
#endif
      if (!MULTI && tid < F) bn_affine_store(c, r, tid, bnq, alpha, beta, mean, inv);
      if (wait_now) {
        rc_wait_leads(c, c.ws + r * c.wss, wait_cnt, wait_target);
        RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_WAIT, 0);
        dw_load(0);
      }
      dw_store(0);
  RC_PHASE(c.ws, c.wo.total, pbx, 45);  // the first dL/dw round is in
      dw_rest();
  RC_PHASE(c.ws, c.wo.total, pbx, 46);
      __syncthreads();
      if (tid < n) {
        float t = 0.f;
        for (int cc = 0; cc < p; ++cc) t += Srow[tid * p + cc];
        rs[tid] = t;
      }
    } else {
      rc_stage_all(sR, sT, sX, sF1, sW, sL);
      dw_store(0);
      dw_rest();
      __syncthreads();
    }
  RC_PHASE(c.ws, c.wo.total, pbx, 34);
    for (int e = tid; e < nbc * K; e += RC_BLOCK) dr[e] = draw_value(c, r, dK.mod(e), wrl[e], dwl[e], labl[e]);
    if (mf) {
      // rows [nbc, 16) of the window tiles the products read are zero windows
      for (int e = nbc * K + tid; e < 16 * K; e += RC_BLOCK) dr[e] = 0.f;
      for (int e = nbc * HC + tid; e < 16 * HC; e += RC_BLOCK) Rc[e] = 0.f;
      for (int e = nbc * nF + tid; e < 16 * nF; e += RC_BLOCK) Tc[e] = 0.f;
      __syncthreads();
      // df1[s][m] = [f1 > 0] sum_k dr[s][k] fc2W[k][m]: wave w, columns m in [16 w, 16 w + 16)
      if (16 * wv < M1) {
        const int m = 16 * wv + l15;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < K; k0 += 4) {
          const int k = k0 + lg;
          const float av = k < K ? dr[l15 * K + k] : 0.f;
          const float bv = (k < K && m < M1) ? fc2s[k * M1 + m] : 0.f;
          a = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, a, 0, 0, 0);
        }
        if (m < M1)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int sw = 4 * lg + reg;
            df1c[sw * M1 + m] = (sw < nbc && f1r[sw * M1 + m] > 0.f) ? a[reg] : 0.f;
          }
      }
      __syncthreads();
  RC_PHASE(c.ws, c.wo.total, pbx, 35);
      // dZ[s][hh] = [R > 0] sum_m df1[s][m] fc1W[m][hh]: wave 0
      if (wv == 0) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        for (int m0 = 0; m0 < M1; m0 += 4) {
          const int m = m0 + lg;
          const float av = m < M1 ? df1c[l15 * M1 + m] : 0.f;
          const float bv = m < M1 ? FW[m * HC + l15] : 0.f;
          a = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, a, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int e = (4 * lg + reg) * HC + l15;
          dZc[e] = Rc[e] > 0.f ? a[reg] : 0.f;
        }
      }
      // dfc1W chunk partial: afc[m][hh] += sum_s df1[s][m] R[s][hh]: wave w, rows m in [16 w, 16 w + 16)
      if (16 * wv < M1) {
        const int m = 16 * wv + l15;
        f32x4 accA = {afc[0], afc[1], afc[2], afc[3]};
#pragma unroll
        for (int s0 = 0; s0 < 16; s0 += 4) {
          const int sw = s0 + lg;
          const float av = m < M1 ? df1c[sw * M1 + m] : 0.f;
          accA = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Rc[sw * HC + l15], accA, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) afc[reg] = accA[reg];
      }
      // group 0: dfc2W[k][m] += sum_s dr[s][k] relu(f1[s][m]); dfc2b[k] += sum_s dr[s][k]; dfc1b[m] += sum_s df1[s][m]
      if (head_grads) {
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) {
          const int e = tid + kk * RC_BLOCK;
          if (e >= nout) continue;
          float g = agf[kk];
          if (e < K * M1) {
            const int k = dM1.div(e), m = e - k * M1;
            for (int s = 0; s < nbc; ++s) g += dr[s * K + k] * fmaxf(f1r[s * M1 + m], 0.f);
          } else if (e < K * M1 + K) {
            const int k = e - K * M1;
            for (int s = 0; s < nbc; ++s) g += dr[s * K + k];
          } else {
            const int m = e - K * M1 - K;
            for (int s = 0; s < nbc; ++s) g += df1c[s * M1 + m];
          }
          agf[kk] = g;
        }
      }
      __syncthreads();
  RC_PHASE(c.ws, c.wo.total, pbx, 36);
      // dW_i chunk partial: awi[q][hh] += sum_s T[s][q] dZ[s][hh], q = (i, f); dT[s][q] =
      // sum_hh dZ[s][hh] W[q][hh]: wave w, 16-row tiles qt = w + 4 i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qt = wv + 4 * i;
        if (16 * qt >= nF) break;
        const int q = 16 * qt + l15;
        f32x4 accW = {awi[4 * i], awi[4 * i + 1], awi[4 * i + 2], awi[4 * i + 3]};
#pragma unroll
        for (int s0 = 0; s0 < 16; s0 += 4) {
          const int sw = s0 + lg;
          const float av = q < nF ? Tc[sw * nF + q] : 0.f;
          accW = __builtin_amdgcn_mfma_f32_16x16x4f32(av, dZc[sw * HC + l15], accW, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) awi[4 * i + reg] = accW[reg];
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int hq = 0; hq < 16; hq += 4) {
          const int hh = hq + lg;
          const float bv = q < nF ? WiC[q * HP + hh] : 0.f;
          a = __builtin_amdgcn_mfma_f32_16x16x4f32(dZc[l15 * HC + hh], bv, a, 0, 0, 0);
        }
        if (q < nF)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) dTc[(4 * lg + reg) * nF + q] = a[reg];
      }
      __syncthreads();
    } else {
      __syncthreads();
      // df1[s][m] = [f1 > 0] sum_k dr[s][k] fc2W[k][m]
      for (int e = tid; e < nbc * M1; e += RC_BLOCK) {
        const int s = dM1.div(e), m = e - s * M1;
        float g = 0.f;
        if (f1r[e] > 0.f)
          for (int k = 0; k < K; ++k) g += dr[s * K + k] * fc2s[k * M1 + m];
        df1c[e] = g;
      }
      __syncthreads();
  RC_PHASE(c.ws, c.wo.total, pbx, 35);
      // dZ[s][hh] = [R > 0] sum_m df1[s][m] fc1W[m][hh]   (4 independent partial sums)
      for (int e = tid; e < nbc * HC; e += RC_BLOCK) {
        const int s = e / HC, hh = e - s * HC;
        const float* dfr = df1c + s * M1;
        float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f;
        int m = 0;
        for (; m + 3 < M1; m += 4) {
          g0 += dfr[m] * FW[m * HC + hh];
          g1 += dfr[m + 1] * FW[(m + 1) * HC + hh];
          g2 += dfr[m + 2] * FW[(m + 2) * HC + hh];
          g3 += dfr[m + 3] * FW[(m + 3) * HC + hh];
        }
        for (; m < M1; ++m) g0 += dfr[m] * FW[m * HC + hh];
        const float g = (g0 + g1) + (g2 + g3);
        dZc[e] = Rc[e] > 0.f ? g : 0.f;
      }
      // dfc1W chunk partial: afc[m][hh] += sum_s df1[s][m] R[s][hh]
      for (int s = 0; s < nbc; ++s) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = tid + k * RC_BLOCK;
          if (e < M1 * HC) afc[k] += df1c[s * M1 + e / HC] * Rc[s * HC + e % HC];
        }
      }
      // group 0: dfc2W[k][m] += sum_s dr[s][k] relu(f1[s][m]); dfc2b[k] += sum_s dr[s][k]; dfc1b[m] += sum_s df1[s][m]
      if (head_grads) {
#pragma unroll
        for (int kk = 0; kk < 5; ++kk) {
          const int e = tid + kk * RC_BLOCK;
          if (e >= nout) continue;
          float g = agf[kk];
          if (e < K * M1) {
            const int k = dM1.div(e), m = e - k * M1;
            for (int s = 0; s < nbc; ++s) g += dr[s * K + k] * fmaxf(f1r[s * M1 + m], 0.f);
          } else if (e < K * M1 + K) {
            const int k = e - K * M1;
            for (int s = 0; s < nbc; ++s) g += dr[s * K + k];
          } else {
            const int m = e - K * M1 - K;
            for (int s = 0; s < nbc; ++s) g += df1c[s * M1 + m];
          }
          agf[kk] = g;
        }
      }
      __syncthreads();
  RC_PHASE(c.ws, c.wo.total, pbx, 36);
      // dW_i chunk partial: awi[i][f][hh] += sum_s T_i[s][f] dZ[s][hh]
      for (int s = 0; s < nbc; ++s) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int e = tid + k * RC_BLOCK;
          if (k < nwi && e < nF * HC) awi[k] += Tc[s * nF + e / HC] * dZc[s * HC + e % HC];
        }
      }
      // dT_i[s][f] = sum_hh dZ[s][hh] W_i[f][hh]
      for (int e = tid; e < nbc * nF; e += RC_BLOCK) {
        const int s = dnF.div(e), rem = e - s * nF;
        const float* wr = WiC + rem * HP;
        const float* dz = dZc + s * HC;
        float t0 = 0.f, t1 = 0.f;
#pragma unroll
        for (int hh = 0; hh < HC; hh += 2) {
          t0 += dz[hh] * wr[hh];
          t1 += dz[hh + 1] * wr[hh + 1];
        }
        dTc[e] = t0 + t1;
      }
      __syncthreads();
    }
    if (late_x) {  // f1 / df1 / R / dZ / T are dead: the window tile goes there
      rc_stage_all(rc_seg<16>(nbc * pF, x_ld, x_st));
      __syncthreads();
    }
  RC_PHASE(c.ws, c.wo.total, pbx, 37);
    // dS_i[node][c'] (i >= 1) and BatchNorm affine partials, windows split over thread slices
    if (slS < nslS) {
      const int i = 1 + oS / p, cp = oS - (i - 1) * p;
      for (int s = slS; s < nbc; s += nslS) {
        const float* dt = dTc + s * nF + i * F;
        const float* xr = xc + s * pF + cp * F;
#pragma unroll 4  // (LDS reads of 4 features in flight; the same running sum)
        for (int f = 0; f < F; ++f) aS += dt[f] * (xr[f] * alpha[f] + beta[f]);
      }
    }
    if (slF < nslF) {
      const int f = oF;
      const float mu = mean[f], iv = inv[f];
      for (int s = slF; s < nbc; s += nslF) {
        const float* xs_ = xc + s * pF + f;
        for (int i = 0; i < n; ++i) {
          float u;
          if (i == 0) {
            u = (xs_[node * F] - mu) * iv;
          } else {
            u = 0.f;
#pragma unroll 4
            for (int cc = 0; cc < p; ++cc) u += Srow[i * p + cc] * ((xs_[cc * F] - mu) * iv);
          }
          const float dt = dTc[s * nF + i * F + f];
          aG += dt * u;
          aB += dt * rs[i];
        }
      }
    }
  }
  RC_PHASE(c.ws, c.wo.total, pbx, 38);
  // ---- publish this block's partials:
  //      [grp][wb][ afc M1*HC | awi nF*HC | dS nS | dgamma F | dbeta F | (group 0) dfc2W dfc2b dfc1b ]
  const int pst = rc_emb_pstride(d);
  const int ofs_w = M1 * HC, ofs_s = ofs_w + nF * HC, ofs_g = ofs_s + nS, ofs_h = ofs_g + 2 * F;
  float* part = ws + c.wo.ebp + ((int64_t)grp * nbw_max + wb) * pst;
  if (mf) {
    if (16 * wv < M1)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int m = 16 * wv + 4 * lg + reg;
        if (m < M1) part[m * HC + l15] = afc[reg];
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qt = wv + 4 * i;
      if (16 * qt >= nF) break;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int q = 16 * qt + 4 * lg + reg;
        if (q < nF) part[ofs_w + q * HC + l15] = awi[4 * i + reg];
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = tid + k * RC_BLOCK;
      if (e < M1 * HC) part[e] = afc[k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = tid + k * RC_BLOCK;
      if (k < nwi && e < nF * HC) part[ofs_w + e] = awi[k];
    }
  }
  if (head_grads) {
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const int e = tid + kk * RC_BLOCK;
      if (e < nout) part[ofs_h + e] = agf[kk];
    }
  }
  red[tid] = (slS < nslS) ? aS : 0.f;
  __syncthreads();
  if (tid < nS) {
    float t = 0.f;
#pragma unroll 4
    for (int q = 0; q < nslS; ++q) t += red[q * nS + tid];
    part[ofs_s + tid] = t;
  }
  __syncthreads();
  red[tid] = (slF < nslF) ? aG : 0.f;
  __syncthreads();
  if (tid < F) {
    float t = 0.f;
#pragma unroll 4
    for (int q = 0; q < nslF; ++q) t += red[q * F + tid];
    part[ofs_g + tid] = t;
  }
  __syncthreads();
  red[tid] = (slF < nslF) ? aB : 0.f;
  __syncthreads();
  if (tid < F) {
    float t = 0.f;
#pragma unroll 4
    for (int q = 0; q < nslF; ++q) t += red[q * F + tid];
    part[ofs_g + F + tid] = t;
  }
  RC_PHASE(c.ws, c.wo.total, pbx, 39);
  if (c.defer) {  // k_emb_combine sums the window blocks after this kernel (no ticket / fences)
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 1);
    return;
  }
  // release (every wave drains its stores, one lane publishes at agent scope), then the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* cnt = reinterpret_cast<unsigned*>(ws + c.wo.ecnt);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tk[0] = (int)__hip_atomic_fetch_add(&cnt[grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (tk[0] != nbw - 1) {
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 1);
    return;
  }
  RC_PHASE(c.ws, c.wo.total, pbx, 40);
  // ---- last arriver: acquire, then combine the nbw partials in window-block order
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const float* base = ws + c.wo.ebp + (int64_t)grp * nbw_max * pst;
  float* dWi = ws + c.wo.dWi + (int64_t)node * n * F * H;
  float* gfc1 = ws + c.wo.gfc1;
  const int64_t pout = (int64_t)node * nch + ch;
  rc_stage<8>(head_grads ? pst : ofs_h, [&](int e) {
    float t = 0.f;
    for (int w0 = 0; w0 < nbw; w0 += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = (w0 + q < nbw) ? base[(int64_t)(w0 + q) * pst + e] : 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (w0 + q < nbw) t += v[q];
    }
    return t;
  }, [&](int e, float t) {
    if (e < ofs_w) {
      const int m = e / HC, hh = e - m * HC;  // dfc1W columns of the chunk (Adam in k_emb_final)
      if (hh < hc) gfc1[(int64_t)m * pH + node * H + h0 + hh] = t;
    } else if (e < ofs_s) {
      const int q = e - ofs_w, qh = q >> 4, i = dF.div(qh), f = qh - i * F, hh = q & 15;  // HC == 16
      if (hh < hc) dWi[((int64_t)i * F + f) * H + h0 + hh] = t;
    } else if (e < ofs_g) {
      ws[c.wo.dS + pout * n * p + p + (e - ofs_s)] = t;  // layout [part][n][p], rows i >= 1
    } else if (e < ofs_h) {
      ws[c.wo.dgb + pout * 2 * F + (e - ofs_g)] = t;     // [part][2][F]: dgamma, dbeta
    } else {
      ws[c.wo.gfc + (e - ofs_h)] = t;                    // dfc2W | dfc2b | dfc1b
    }
  });
  RC_PHASE(c.ws, c.wo.total, pbx, 41);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 1);
}

// The last-arriver combine of emb_bwd_node as its own launch (c.defer): element e of
// (node, chunk) group blockIdx.y summed over the window blocks in block order and scattered
// exactly as the last arriver does, so both variants give the same bits.
// grid (ceil(pstride / RC_BLOCK), p * nchunk, R).
// (emb_combine_elem: element e of group grp of replica r; sc1: coherent stores, read inside the
// same launch by k_emb_tail's parameter workgroups)
__device__ __forceinline__ bool emb_combine_in(const StepCtx& c, int grp, int e) {
  const RedcliffDims& d = c.d;
  const int ofs_h = d.M1 * EMB_HC + d.n * d.F * EMB_HC + (d.n - 1) * d.p + 2 * d.F;
  return e < (grp == 0 ? rc_emb_pstride(d) : ofs_h);  // fc2 / fc1-bias partials ride on group 0
}
__device__ __forceinline__ float emb_combine_sum(const StepCtx& c, int r, int grp, int e) {
  const RedcliffDims& d = c.d;
  if (!emb_combine_in(c, grp, e)) return 0.f;
  const int pst = rc_emb_pstride(d), nbwm = c.enbwm, nbw = c.enbw;
  const float* base = c.ws + r * c.wss + c.wo.ebp + (int64_t)grp * nbwm * pst + e;
  float t = 0.f;
  for (int w0 = 0; w0 < nbw; w0 += 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = (w0 + q < nbw) ? base[(int64_t)(w0 + q) * pst] : 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (w0 + q < nbw) t += v[q];
  }
  return t;
}
__device__ __forceinline__ void emb_combine_store(const StepCtx& c, int r, int grp, int e, float t, bool sc1) {
  const RedcliffDims& d = c.d;
  if (!emb_combine_in(c, grp, e)) return;
  const int p = d.p, n = d.n, F = d.F, H = d.H, M1 = d.M1, HC = EMB_HC;
  const int nch = rc_nchunk(d), node = RcDiv32(nch, c.mg[RC_MG_NCH]).div(grp), ch = grp - node * nch;
  const int ofs_w = M1 * HC, ofs_s = ofs_w + n * F * HC, ofs_g = ofs_s + (n - 1) * p, ofs_h = ofs_g + 2 * F;
  float* ws = c.ws + r * c.wss;
  const int h0 = ch * HC, hc = min(HC, H - h0);
  if (e < ofs_w) {
    const int m = e / HC, hh = e - m * HC;
    if (hh < hc) rc_store_payload(ws + c.wo.gfc1 + (int64_t)m * p * H + node * H + h0 + hh, t, sc1);
  } else if (e < ofs_s) {
    const int q = e - ofs_w, qh = q >> 4, i = qh / F, f = qh - i * F, hh = q & 15;  // HC == 16
    if (hh < hc) rc_store_payload(ws + c.wo.dWi + (int64_t)node * n * F * H + ((int64_t)i * F + f) * H + h0 + hh, t, sc1);
  } else if (e < ofs_g) {
    rc_store_payload(ws + c.wo.dS + (int64_t)grp * n * p + p + (e - ofs_s), t, sc1);
  } else if (e < ofs_h) {
    rc_store_payload(ws + c.wo.dgb + (int64_t)grp * 2 * F + (e - ofs_g), t, sc1);
  } else {
    rc_store_payload(ws + c.wo.gfc + (e - ofs_h), t, sc1);
  }
}

__device__ __forceinline__ void emb_combine_elem(const StepCtx& c, int r, int grp, int e, bool sc1) {
  emb_combine_store(c, r, grp, e, emb_combine_sum(c, r, grp, e), sc1);
}

__global__ __launch_bounds__(RC_BLOCK) void k_emb_combine(StepCtx c) {
  emb_combine_elem(c, rc_rep(c, blockIdx.z), blockIdx.y, blockIdx.x * RC_BLOCK + threadIdx.x, false);
}

// Adjacency-L1 gradient of A summed over the K factors' records, in place into record 0
// (fixed order, every load in flight at once: K <= 16).
__device__ __forceinline__ void emb_bwd_dadj(const StepCtx& c, int r, int blk, bool sc1 = false) {
  const int pp2 = c.d.p * c.d.p, e = blk * RC_BLOCK + threadIdx.x;
  if (e >= pp2) return;
  float* dA = c.ws + r * c.wss + c.wo.dAadj;
  float v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k)
    v[k] = k < c.d.K ? (sc1 ? rc_load_sc1(dA + (int64_t)k * pp2 + e) : dA[(int64_t)k * pp2 + e]) : 0.f;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k < c.d.K) t += v[k];
  dA[e] = t;
}

// The embedder backward's launch without node workgroups (the GEMM-shaped embedder computes those
// products itself; validation steps compute none): the optional head workgroup and the adjacency-L1
// reduce workgroups, as a light kernel of its own -- k_emb_bwd's node-sized LDS and registers (the
// multi-sub-block instantiation: 256 VGPRs) made this launch take 32.5 us at C5 for 17 workgroups of
// trivial work (profiles/r06_kernel_stats_c5_f.csv).  The same device functions, so the same bits.
// grid (head + nred, R)
__global__ __launch_bounds__(RC_BLOCK) void k_emb_head_dadj(StepCtx c, int head) {
  __shared__ __attribute__((aligned(16))) float sm[32 + 16 * 16];  // [8] floats, [8] doubles, hist[nsup][nsup] (nsup <= K <= 16)
  const int r = rc_rep(c, blockIdx.y);
  if ((int)blockIdx.x >= head)
    emb_bwd_dadj(c, r, (int)blockIdx.x - head);
  else
    emb_bwd_head(c, r, sm);
}

// grid (p * nchunk * nbw [+ 1] [+ nred], R): workgroups [0, p*nchunk*nbw) are (node, column
// chunk, window block) blocks; then the optional head (loss values / confusion), then the
// adjacency-L1 reduce workgroups.
// The single-sub-block variant stages the window tile late (rc_emb_late_x) and runs with a floor
// of RC_EMB_WAVES waves per SIMD (0: the compiler's choice); the multi-sub-block one (256 VGPRs)
// keeps its layout and registers.
#ifndef RC_EMB_WAVES
#define RC_EMB_WAVES 0
#endif
template <bool MULTI>
__global__ __launch_bounds__(RC_BLOCK) __attribute__((amdgpu_waves_per_eu(MULTI || RC_EMB_WAVES == 0 ? 1 : RC_EMB_WAVES)))
void k_emb_bwd(StepCtx c, int nnode, int head, int BC, int WPB) {
  extern __shared__ float sm[];
  const int r = rc_rep(c, blockIdx.y);
  const int nch = rc_nchunk(c.d);
  // the host's window blocking and multipliers when WPB is the default one (always, in the step)
  const bool hb = WPB == c.ewpb;
  const RcDiv32 dnbw = hb ? RcDiv32(c.enbw, c.mg[RC_MG_ENBW]) : RcDiv32((c.B + WPB - 1) / WPB), dnch(nch, c.mg[RC_MG_NCH]);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 0);
  RC_PHASE(c.ws, c.wo.total, blockIdx.x, 32);
  if ((int)blockIdx.x >= nnode + head) {
    emb_bwd_dadj(c, r, (int)blockIdx.x - nnode - head);
  } else if ((int)blockIdx.x == nnode) {
    emb_bwd_head(c, r, sm);
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 1);
  } else {
    const int grp = dnbw.div(blockIdx.x), wb = blockIdx.x - grp * dnbw.d, node = dnch.div(grp);
    emb_bwd_node<MULTI, !MULTI>(c, r, node, grp - node * nch, wb, BC, WPB, sm);
  }
}

// Merged backward launch (vector factor path + fused embedder, training steps without loss
// values): the factor backward and the embedder backward in ONE grid instead of two dependent
// launches.  The embedder backward needs only the factor-side dL/dw partials and the
// adjacency-L1 dL/dA records, which the K*p factor-lead workgroups (mixing, forecast residual,
// adjacency L1) write early; the rest of the factor backward (dW0 / Adam) is independent of
// it.  Workgroup order: [K*p factor leads][embedder node / head / dA-reduce workgroups][the
// other factor workgroups]; node and reduce workgroups wait on the leads' published count
// (rc_wait_count), everything else runs free.  Same arithmetic in the same order as the two
// launches, so the results are bit-identical (tests/test_gpu_replicas.py).
// RC_MERGED_WAVES (experiment builds): a floor of waves per SIMD for the single-sub-block merged
// kernel (0: the compiler's choice, 217 VGPRs + 24 AGPRs = 2 waves; 3 caps it at 168 registers with
// 116 bytes of scratch per lane, and 3 workgroups per CU make C1(K=4)'s 681-workgroup grid resident)
#ifndef RC_MERGED_WAVES
#define RC_MERGED_WAVES 0
#endif
template <bool MULTI>
__global__ __launch_bounds__(RC_BLOCK) __attribute__((amdgpu_waves_per_eu(MULTI || RC_MERGED_WAVES == 0 ? 1 : RC_MERGED_WAVES)))
void k_bwd_merged(StepCtx c, int nUl, int nQ, int nnode, int head, int nred,
                                                         int BC, int WPB) {
  extern __shared__ float sm[];
  const int r = rc_rep(c, blockIdx.y);
  unsigned* cnt = rc_fac_lead_cnt(c, c.ws + r * c.wss);
  const int KP = c.d.K * c.d.p;
  const int bx = blockIdx.x;
  const int nemb = nnode + head + nred;
  const int e = bx - KP;
  if (e >= 0 && e < nemb) {
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_BWD, 0);
    if (e >= nnode + head) {
      rc_wait_leads(c, c.ws + r * c.wss, cnt, KP);
      emb_bwd_dadj(c, r, e - nnode - head, true);
    } else if (e == nnode) {
      emb_bwd_head(c, r, sm);
    } else {
      const int nch = rc_nchunk(c.d);
      const RcDiv32 dnbw = WPB == c.ewpb ? RcDiv32(c.enbw, c.mg[RC_MG_ENBW]) : RcDiv32((c.B + WPB - 1) / WPB);
      const int grp = dnbw.div(e), wb = e - grp * dnbw.d, node = RcDiv32(nch, c.mg[RC_MG_NCH]).div(grp);
      emb_bwd_node<MULTI>(c, r, node, grp - node * nch, wb, BC, WPB, sm, cnt, (unsigned)KP);
    }
    return;
  }
  // factor workgroups: the K*p leads first (ids [0, K*p)), the rest after the embedder's.  With
  // a factor step the leads only write their records (the embedder workgroups' inputs) and
  // publish; the update part of each network's (0, 0) workgroup is K*p more workgroups at the
  // end, so no workgroup carries both (the longest workgroups of the launch otherwise)
  const bool lead_split = RC_MERGED_LEAD_SPLIT && (c.flags & RC_STEP_B);
  int kj, uc = 0, qc = 0, role = RC_FB_ALL;
  if (e < 0) {
    kj = bx;
    if (lead_split) role = RC_FB_RECORDS;
  } else if (lead_split && e - nemb >= KP * (nUl * nQ - 1)) {
    kj = e - nemb - KP * (nUl * nQ - 1);
    role = RC_FB_UPDATE;
  } else {
    const int f = e - nemb, per = nUl * nQ - 1;
    int rem;
    if ((KP & 7) == 0) {
      // XCD-aware order: blocks b and b + 8 share an XCD (MI355X_MICROARCH.md, workgroup
      // dispatch; a speed hint only), and lead kj is block kj.  Deal the non-lead workgroups so
      // every workgroup of network kj lands in kj's block class: the per-network operands every
      // one of them stages (predictions, embedder outputs, targets, group-norm partials, A
      // column) are then fetched into one XCD's L2 instead of up to seven.
      const int x = (KP + nemb + f) & 7, t = f >> 3;  // f's block class; each round of 8 covers all 8
      kj = x + 8 * (t / per);
      rem = t % per + 1;
    } else {
      kj = f / per;
      rem = f - kj * per + 1;
    }
    uc = rem / nQ;
    qc = rem - uc * nQ;
  }
  fac_bwd_wg(c, nUl, nQ, kj, uc, qc, r, sm, e < 0 ? cnt : nullptr, role);
}

// ---- adjacency algebra for p <= 64 in one workgroup, operands in LDS with row stride P = p + 1

// Row sums over j < p of f(i, j), i < p: four lanes per row, each summing a strided quarter,
// combined in fixed order; out(i, s) runs on the row's first lane.
template <class Fn, class Out>
__device__ inline void lds_rowsum(int p, Fn f, Out out) {
  const int i = threadIdx.x >> 2, sub = threadIdx.x & 3;
  float s = 0.f;
  if (i < p)
    for (int j = sub; j < p; j += 4) s += f(i, j);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  if (i < p && sub == 0) out(i, s);
}

// p x p product op(X) op(Y) on the matrix cores: wave w owns the 32x32 output tile
// (w >> 1, w & 1); entries at or beyond p are zero padding.  Returns false for a wave with no
// tile; lane entry reg is row a0 + mf_row(reg, lane), column b0 + (lane & 31).
template <bool TX, bool TY>
__device__ inline bool lds_mm_tile(const float* X, const float* Y, int p, int P, f32x16& acc, int& a0, int& bj) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  a0 = 32 * (wv >> 1);
  const int b0 = 32 * (wv & 1);
  if (a0 >= p || b0 >= p) return false;
  const int l31 = lane & 31, kh = lane >> 5, ai = a0 + l31;
  bj = b0 + l31;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // four k steps' operands read before their products (one LDS round trip per four steps);
  // the steps themselves are the k0 < p ones, in order
  for (int k00 = 0; k00 < p; k00 += 8) {
    float xs[4], ys[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k00 + 2 * u + kh;
      xs[u] = (k < p && ai < p) ? (TX ? X[k * P + ai] : X[ai * P + k]) : 0.f;
      ys[u] = (k < p && bj < p) ? (TY ? Y[bj * P + k] : Y[k * P + bj]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (k00 + 2 * u < p) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[u], ys[u], acc, 0, 0, 0);
  }
  return true;
}

// out(a, b, v) receives each in-range result (one writer per entry).
template <bool TX, bool TY, class Out>
__device__ inline void lds_mm(const float* X, const float* Y, int p, int P, Out out) {
  f32x16 acc;
  int a0, bj;
  if (!lds_mm_tile<TX, TY>(X, Y, p, P, acc, a0, bj)) return;
  const int lane = threadIdx.x & 63;
  if (p <= 16) {  // rows 16..31 of the tile (registers 8..15) are padding: half the epilogue
#pragma unroll
    for (int reg = 0; reg < 8; ++reg) {
      const int a = a0 + mf_row(reg, lane);
      if (a < p && bj < p) out(a, bj, acc[reg]);
    }
  } else {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int a = a0 + mf_row(reg, lane);
      if (a < p && bj < p) out(a, bj, acc[reg]);
    }
  }
}

// D[a][b] += (op(X) op(Y))[a][b] (D disjoint from X and Y, rows padded to P = p + 1): every old value is read before
// any sum is written back, so the 16 read-modify-writes of a lane are not one LDS round trip
// each; the sums are the per-entry ones (old + product)
template <bool TX, bool TY>
__device__ inline void lds_mm_acc(const float* X, const float* Y, int p, int P, float* D) {
  f32x16 acc;
  int a0, bj;
  if (!lds_mm_tile<TX, TY>(X, Y, p, P, acc, a0, bj)) return;
  // An entry outside p x p reads and writes its row's padding slot (column p, never read as an
  // operand) instead of branching around the access: no exec-mask branch per entry, so the
  // writes do not each wait for the previous one.
  const int lane = threadIdx.x & 63;
  const bool cin = bj < p;
  auto rmw = [&](auto nreg) {  // (p <= 16: rows 16..31, registers 8..15, are padding)
    constexpr int NR = decltype(nreg)::value;
    int ad[NR];
    float old[NR];
#pragma unroll
    for (int reg = 0; reg < NR; ++reg) {
      const int a = a0 + mf_row(reg, lane);
      ad[reg] = (cin && a < p) ? a * P + bj : min(a, p - 1) * P + p;
      old[reg] = D[ad[reg]];
    }
#pragma unroll
    for (int reg = 0; reg < NR; ++reg) D[ad[reg]] = old[reg] + acc[reg];
  };
  if (p <= 16)
    rmw(std::integral_constant<int, 8>{});
  else
    rmw(std::integral_constant<int, 16>{});
}

// Supports of normalize_A(A) (S_0 = I, S_1 = L, S_l = S_{l-1} L): A padded in LDS, L and its
// powers built in LDS slots 1..n-1 of Sl and written densely to S[n][p][p].  Used by the
// optimizer's adjacency workgroup and by k_supports, so both produce the same bits.
template <class Div>
__device__ __forceinline__ void supports_lds(const Div& dpv, const float* Al, float* Sl, float* S, float* dinv, int p, int n) {
  const int P = p + 1, PP = p * P, pp2 = p * p;
  lds_rowsum(p, [&](int i, int j) { return fmaxf(Al[i * P + j], 0.f); },
             [&](int i, float s) { dinv[i] = 1.f / sqrtf(s + 1e-10f); });
  __syncthreads();
  for (int e = threadIdx.x; e < pp2; e += RC_BLOCK) {
    const int i = dpv.div(e), j = e - i * p;
    S[e] = (i == j) ? 1.f : 0.f;
    if (n > 1) {
      const float lv = (dinv[i] * fmaxf(Al[i * P + j], 0.f)) * dinv[j];
      Sl[PP + i * P + j] = lv;
      S[pp2 + e] = lv;
    }
  }
  __syncthreads();
  for (int l = 2; l < n; ++l) {
    float* out = Sl + l * PP;
    float* og = S + (int64_t)l * pp2;
    lds_mm<false, false>(Sl + (l - 1) * PP, Sl + PP, p, P, [&](int a, int b, float v) { out[a * P + b] = v; });
    __syncthreads();
    // the dense copy out by every thread (one element each for p <= 16) instead of 16 scattered
    // stores with their address arithmetic on the product's one wave
    for (int e = threadIdx.x; e < pp2; e += RC_BLOCK) {
      const int i = dpv.div(e);
      og[e] = out[i * P + (e - i * p)];
    }
  }
}

// Supports for every replica from its current A (initialisation and host refreshes).
// grid (R), dynamic LDS (n + 1) p (p + 1) + 64 floats.
__global__ __launch_bounds__(RC_BLOCK) void k_supports(RedcliffDims d, const float* emb, int64_t es, float* ws,
                                                       int64_t wss, EmbOff eo, WsOff wo) {
  const int r = blockIdx.x, p = d.p, P = p + 1;
  extern __shared__ float sm[];
  const float* A = emb + r * es + eo.A;
  for (int e = threadIdx.x; e < p * p; e += RC_BLOCK) {
    const int i = e / p;
    sm[i * P + (e - i * p)] = A[e];
  }
  __syncthreads();
  supports_lds(RcDiv(p), sm, sm + p * P, ws + r * wss + wo.S, sm + (d.n + 1) * p * P, p, d.n);
}

// Data-parallel update after the all-reduce (DataParallelFit): Adam of both parameter groups from
// the summed gradients in one launch, and the Chebyshev supports of the updated adjacency in the
// workgroup that owns A's elements, so the next shard step starts without a refresh launch.
// grid (1 + nbE + nbF, R): workgroup 0 = A (p*p elements) + supports when the embedder group
// steps; then nbE workgroups over the embedder group (A's range skipped) and nbF over the factor
// group, DPU_EPT coalesced elements per thread (the fp64 bias corrections once per thread).  The
// per-element arithmetic is rc_adam's, as in k_emb_final / the factor kernels / k_adam_apply.
#define DPU_EPT 4  // (16: ~55 workgroups at TST, 9.6 us; the chip needs more of them)
__global__ __launch_bounds__(RC_BLOCK) void k_dp_update(StepCtx c, int64_t nE, int64_t nF, int nbE) {
  extern __shared__ float sm[];
  const int r = rc_rep(c, blockIdx.y), tid = threadIdx.x;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const int bx = blockIdx.x;
  const int p = c.d.p, pp = p * p;
  if (bx == 0) {
    if (!(c.flags & RC_STEP_A)) return;
    const RcAdamScalars s = rc_adam_scalars(hy.A, c.tA);
    float* P = c.emb + r * c.es;
    float* M = c.embM + r * c.es;
    float* V = c.embV + r * c.es;
    const float* G = c.gE + r * c.es;
    const int P1 = p + 1;
    for (int e = tid; e < pp; e += RC_BLOCK) {
      const int64_t i = c.eo.A + e;
      float pv = P[i], mv = M[i], vv = V[i];
      rc_adam(pv, mv, vv, G[i], s);
      P[i] = pv; M[i] = mv; V[i] = vv;
      const int a = e / p;
      sm[a * P1 + (e - a * p)] = pv;
    }
    __syncthreads();
    supports_lds(RcDiv32(p, c.mg[RC_MG_P]), sm, sm + p * P1, c.ws + r * c.wss + c.wo.S, sm + (c.d.n + 1) * p * P1, p, c.d.n);
    return;
  }
  const bool emb = bx <= nbE;
  const RcAdamScalars s = rc_adam_scalars(emb ? hy.A : hy.B, emb ? c.tA : c.tB);
  const int64_t st = emb ? c.es : c.fs, n = emb ? nE : nF;
  float* P = (emb ? c.emb : c.fac) + r * st;
  float* M = (emb ? c.embM : c.facM) + r * st;
  float* V = (emb ? c.embV : c.facV) + r * st;
  const float* G = (emb ? c.gE : c.gF) + r * st;
  const int64_t i0 = (int64_t)(emb ? bx - 1 : bx - 1 - nbE) * RC_BLOCK * DPU_EPT + tid;
  const int64_t a0 = emb ? c.eo.A : -1, a1 = emb ? c.eo.A + pp : -1;
  float pv[DPU_EPT], mv[DPU_EPT], vv[DPU_EPT], gv[DPU_EPT];
#pragma unroll
  for (int k = 0; k < DPU_EPT; ++k) {
    const int64_t i = i0 + (int64_t)k * RC_BLOCK;
    const bool on = i < n;
    pv[k] = on ? P[i] : 0.f;
    mv[k] = on ? M[i] : 0.f;
    vv[k] = on ? V[i] : 0.f;
    gv[k] = on ? G[i] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < DPU_EPT; ++k) {
    const int64_t i = i0 + (int64_t)k * RC_BLOCK;
    if (i >= n || (i >= a0 && i < a1)) continue;
    rc_adam(pv[k], mv[k], vv[k], gv[k], s);
    P[i] = pv[k]; M[i] = mv[k]; V[i] = vv[k];
  }
}

// Window-block partials of k_emb_bwd read in place by k_emb_final (c.defer == 2): element
// off of (node, chunk) group grp summed over the window blocks in block order -- the sum
// k_emb_combine forms, so the fused read and the separate launch give the same bits.
struct EmbWbSum {
  const float* base;
  int pst, nbw, nbwm;
  __device__ EmbWbSum(const StepCtx& c, const float* ws)
      : base(ws + c.wo.ebp), pst(rc_emb_pstride(c.d)), nbw(c.enbw), nbwm(c.enbwm) {}
  __device__ float operator()(int grp, int off) const { return nodes(grp, 1, 1, off); }
  // Sum over u < nn, in order, of the window-block sums of group grp0 + u * gs: the combined
  // records added one after another, as k_emb_final adds them.  Four groups x eight window
  // blocks of loads are in flight at once (one memory round per 4 groups for nbw <= 8).
  __device__ float nodes(int grp0, int gs, int nn, int off) const {
    float g = 0.f;
    for (int u0 = 0; u0 < nn; u0 += 4) {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int w0 = 0; w0 < nbw; w0 += 8) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* b = base + (int64_t)(grp0 + (u0 + u) * gs) * nbwm * pst + off;
#pragma unroll
          for (int q = 0; q < 8; ++q) v[u][q] = (u0 + u < nn && w0 + q < nbw) ? b[(int64_t)(w0 + q) * pst] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (w0 + q < nbw) t[u] += v[u][q];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u0 + u < nn) g += t[u];
    }
    return g;
  }
  // the four chains of consecutive groups grp0 .. grp0 + 3 (BatchNorm affine partials)
  __device__ void four(int grp0, int off, float* g4) const {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w0 = 0; w0 < nbw; w0 += 8) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* b = base + (int64_t)(grp0 + u) * nbwm * pst + off;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[u][q] = (w0 + q < nbw) ? b[(int64_t)(w0 + q) * pst] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (w0 + q < nbw) t[u] += v[u][q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) g4[u] += t[u];
  }
};

// ------------------------------------------------------------------------------------------
// K4: embedder optimizer finalisation.  Workgroups [1, nw] apply Adam to W_i, fc2, fc1 bias,
// BN affine (reducing per-node partials in fixed order); workgroup 0 handles the
// adjacency A (Chebyshev + normalize_A backward, adjacency-L1 gradient), the BN running
// statistics and recomputes the supports for the next step.
// NR = elements of a p x p matrix per thread (p * p <= NR * RC_BLOCK): staging width and the
// register prefetch; small adjacencies get the short code (one-shot code is fetched cold).
// One workgroup of K4 (wx = 0: the adjacency workgroup, wx >= 1: parameter workgroup wx - 1) of
// replica slot wy.  fused (c.defer == 2): the parameter workgroups sum the window-block partials
// in place; sc1: they read the combined records with coherent loads (k_emb_tail, where the
// combine runs in the same launch); adj_inplace: the adjacency workgroup sums its dS partials in
// place (k_emb_tail, where it does not wait for the combine).
#define EF_EPT_MAX 8  // runs per thread of the batched parameter path (k_emb_final's ept <= this)
#ifndef RC_EF_PMV_FIRST
#define RC_EF_PMV_FIRST 1  // batched path: parameters / moments requested with (1) or after (0) the gradients
#endif
template <int NR>
__device__ __forceinline__ void emb_final_wg(const StepCtx& c, int wx, int wy, int ept, bool sc1, bool adj_inplace) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, wy);
  const int p = d.p, n = d.n, F = d.F, H = d.H, K = d.K, M1 = d.M1;
  float* E = c.emb + r * c.es;
  float* Mm = c.embM + r * c.es;
  float* V = c.embV + r * c.es;
  float* ws = c.ws + r * c.wss;
  const bool stepA = c.flags & RC_STEP_A;
  const RcAdamScalars as = rc_adam_scalars(c.hyp[r].A, c.tA);
  const int nFH = n * F * H, nfc = K * M1 + K + M1, nf1 = M1 * p * H;
  const int total = nFH + nfc + 2 * F + nf1;
  // c.defer == 2: the node blocks' window-block partials are summed here (no combine launch);
  // record layout of emb_bwd_node: fc1 chunk | W_i chunk | dS rows i >= 1 | dgamma dbeta | head
  const bool fused = c.defer == 2;
  auto ldr = [&](const float* q) { return sc1 ? rc_load_sc1(q) : *q; };
  const int HC = EMB_HC, nch = rc_nchunk(d);
  const int ofs_w = M1 * HC, ofs_s = ofs_w + n * F * HC, ofs_g = ofs_s + (n - 1) * p, ofs_h = ofs_g + 2 * F;
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FINAL, 0);
  // workgroup 0 is the adjacency workgroup (the longest; dispatched first), 1..nw the parameters
  if (wx > 0) {
    if (!stepA) return;
    if (!fused && !sc1 && ept > 1 && ept <= EF_EPT_MAX && !(c.flags & RC_GRAD_ONLY)) {
      // packed replicas (combined records, several runs per thread): every run's gradient, then
      // the parameters and both moments of all runs requested together and the Adam steps -- one
      // memory round for the workgroup instead of one per run; the same values and operations
      // per run: the parameter index and where its gradient comes from (no loads yet): one
      // combined record (fc / fc1 weights -- all runs of every workgroup but the first), or the
      // dwN node slices of W_i / the dgN BatchNorm partials (the first parameter workgroup)
      float g[EF_EPT_MAX];
      int64_t ix[EF_EPT_MAX], go[EF_EPT_MAX];
      int kind[EF_EPT_MAX];  // 0: past the end, 1: one record at go, 2: W_i slices, 3: BN affine
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        ix[run] = -1;
        go[run] = 0;
        kind[run] = 0;
        const int e = ((wx - 1) * ept + run) * RC_BLOCK + threadIdx.x;
        if (run >= ept || e >= total) continue;
        if (e < nFH) {
          kind[run] = 2;
          ix[run] = c.eo.gcW + e;
        } else if (e < nFH + nfc) {
          const int q = e - nFH;
          kind[run] = 1;
          go[run] = c.wo.gfc + q;
          ix[run] = q < K * M1 ? c.eo.fc2W + q : (q < K * M1 + K ? c.eo.fc2b + (q - K * M1) : c.eo.fc1b + (q - K * M1 - K));
        } else if (e < nFH + nfc + 2 * F) {
          const int q = e - nFH - nfc;
          kind[run] = 3;
          ix[run] = (q < F ? c.eo.bnw : c.eo.bnb) + (q < F ? q : q - F);
        } else {
          const int q = e - nFH - nfc - 2 * F;
          kind[run] = 1;
          go[run] = c.wo.gfc1 + q;
          ix[run] = c.eo.fc1W + q;
        }
      }
      float pv[EF_EPT_MAX], mv[EF_EPT_MAX], vv[EF_EPT_MAX];
#if RC_EF_PMV_FIRST
      // the parameters and both moments requested with the gradients (one round, not two)
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        const int64_t i = ix[run] >= 0 ? ix[run] : 0;
        pv[run] = E[i];
        mv[run] = Mm[i];
        vv[run] = V[i];
      }
#endif
      // the one-record gradients of all runs requested together (the other runs read offset 0)
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        const float v = ws[go[run]];
        g[run] = kind[run] == 1 ? v : 0.f;
      }
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        const int e = ((wx - 1) * ept + run) * RC_BLOCK + threadIdx.x;
        if (kind[run] == 2) {  // sum of the dwN node slices in slice order, 8 loads per round
          float t = 0.f;
          for (int c0 = 0; c0 < c.dwN; c0 += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ws[c.wo.dWi + (int64_t)(c0 + u < c.dwN ? c0 + u : 0) * nFH + e];
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (c0 + u < c.dwN) t += v[u];
          }
          g[run] = t;
        } else if (kind[run] == 3) {
          const int q = e - nFH - nfc;
          const int which = q / F, f = q - which * F;
          float g4[4] = {0.f, 0.f, 0.f, 0.f};
          int pt = 0;
          for (; pt + 3 < c.dgN; pt += 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) g4[u] += ws[c.wo.dgb + ((int64_t)(pt + u) * 2 + which) * F + f];
          for (; pt < c.dgN; ++pt) g4[0] += ws[c.wo.dgb + ((int64_t)pt * 2 + which) * F + f];
          g[run] = (g4[0] + g4[1]) + (g4[2] + g4[3]);
        }
      }
#if !RC_EF_PMV_FIRST
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        const int64_t i = ix[run] >= 0 ? ix[run] : 0;
        pv[run] = E[i];
        mv[run] = Mm[i];
        vv[run] = V[i];
      }
#endif
#pragma unroll
      for (int run = 0; run < EF_EPT_MAX; ++run) {
        if (ix[run] < 0) continue;
        rc_adam(pv[run], mv[run], vv[run], g[run], as);
        E[ix[run]] = pv[run];
        Mm[ix[run]] = mv[run];
        V[ix[run]] = vv[run];
      }
      RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FINAL, 1);
      return;
    }
    // ept runs of RC_BLOCK consecutive elements per workgroup (1 for a single fit; 4 for packed
    // replicas, where one element per thread made ~10K short workgroups at R = 128)
    for (int run = 0; run < ept; ++run) {
    const int e = ((wx - 1) * ept + run) * RC_BLOCK + threadIdx.x;
    if (e >= total) break;
    float g = 0.f;
    int64_t idx;
    if (fused) {
      const EmbWbSum wbs(c, ws);
      if (e < nFH) {  // W_i[i][f][h]: node cc's record of chunk h / HC
        const int ih = e / H, h = e - ih * H, off = ofs_w + ih * HC + h % HC, ch = h / HC;
        g = wbs.nodes(ch, nch, p, off);
        idx = c.eo.gcW + e;
      } else if (e < nFH + nfc) {
        const int q = e - nFH;
        g = wbs(0, ofs_h + q);
        if (q < K * M1) idx = c.eo.fc2W + q;
        else if (q < K * M1 + K) idx = c.eo.fc2b + (q - K * M1);
        else idx = c.eo.fc1b + (q - K * M1 - K);
      } else if (e < nFH + nfc + 2 * F) {
        const int q = e - nFH - nfc;
        const int which = q / F, f = q - which * F;
        float g4[4] = {0.f, 0.f, 0.f, 0.f};
        int pt = 0;
        for (; pt + 3 < c.dgN; pt += 4) wbs.four(pt, ofs_g + which * F + f, g4);
        for (; pt < c.dgN; ++pt) g4[0] += wbs(pt, ofs_g + which * F + f);
        g = (g4[0] + g4[1]) + (g4[2] + g4[3]);
        idx = (which == 0 ? c.eo.bnw : c.eo.bnb) + f;
      } else {  // fc1 weight [m][node * H + h]
        const int q = e - nFH - nfc - 2 * F, pH = p * H;
        const int m = q / pH, rem = q - m * pH, node = rem / H, h = rem - node * H;
        g = wbs(node * nch + h / HC, m * HC + h % HC);
        idx = c.eo.fc1W + q;
      }
    } else if (e < nFH) {
#pragma unroll 8
      for (int cc = 0; cc < c.dwN; ++cc) g += ldr(ws + c.wo.dWi + (int64_t)cc * nFH + e);
      idx = c.eo.gcW + e;
    } else if (e < nFH + nfc) {
      const int q = e - nFH;
      g = ldr(ws + c.wo.gfc + q);
      if (q < K * M1) idx = c.eo.fc2W + q;
      else if (q < K * M1 + K) idx = c.eo.fc2b + (q - K * M1);
      else idx = c.eo.fc1b + (q - K * M1 - K);
    } else if (e < nFH + nfc + 2 * F) {
      const int q = e - nFH - nfc;
      const int which = q / F, f = q - which * F;  // 0: gamma, 1: beta
      // fixed-order sum of the c.dgN partial records (4 independent chains)
      float g4[4] = {0.f, 0.f, 0.f, 0.f};
      int pt = 0;
      for (; pt + 3 < c.dgN; pt += 4)
#pragma unroll
        for (int u = 0; u < 4; ++u) g4[u] += ldr(ws + c.wo.dgb + ((int64_t)(pt + u) * 2 + which) * F + f);
      for (; pt < c.dgN; ++pt) g4[0] += ldr(ws + c.wo.dgb + ((int64_t)pt * 2 + which) * F + f);
      g = (g4[0] + g4[1]) + (g4[2] + g4[3]);
      idx = (which == 0 ? c.eo.bnw : c.eo.bnb) + f;
    } else {
      const int q = e - nFH - nfc - 2 * F;  // fc1 weight (gradient combined by the node blocks)
      g = ldr(ws + c.wo.gfc1 + q);
      idx = c.eo.fc1W + q;
    }
    rc_update(c, E, Mm, V, c.gE + r * c.es, idx, g, as);
    }
    RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FINAL, 1);
    return;
  }
  // ---- adjacency workgroup: every p x p operand lives in LDS (dynamic, (2n + 2) p (p+1)
  // floats, rows padded to P = p + 1); the p x p products run on the matrix cores
  const int tid = threadIdx.x;
  extern __shared__ float sm[];
  const int pp2 = p * p, P = p + 1, PP = p * P;
  const RcDiv32 dpv(p, c.mg[RC_MG_P]);
  float* Al = sm;                  // A (pre-update, then the updated A)
  float* Ar = Al + PP;             // relu(A)
  float* dL = Ar + PP;             // dL/dL (the normalised Laplacian)
  float* dSw = dL + PP;            // dS_1 .. dS_{n-1}
  float* Sl = dSw + (n - 1) * PP;  // slot 0: adjacency-L1 gradient of A; slots 1..n-1: S_1 .. S_{n-1}
  float* dinv = Sl + n * PP;       // [64]
  float* dd = dinv + 64;           // [64]
  // dense index e of a stack of p x p matrices -> padded LDS index
  auto at = [&](int e) { const int i = dpv.div(e); return i * P + (e - i * p); };
  RC_PHASE(c.ws, c.wo.total, wx, 48);
  if (stepA) {
    float* A = E + c.eo.A;
    const float* S = ws + c.wo.S;
    const bool adjL1 = c.flags & RC_LOSS_ADJ;
    const bool adam = !(c.flags & RC_GRAD_ONLY);
    // A's Adam moments, prefetched into registers
    float mreg[NR], vreg[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int e = tid + u * RC_BLOCK;
      const bool in = adam && e < pp2;
      mreg[u] = in ? Mm[c.eo.A + e] : 0.f;
      vreg[u] = in ? V[c.eo.A + e] : 0.f;
    }
    RC_PHASE(c.ws, c.wo.total, wx, 49);
#ifdef RC_PROBE_DELAY
    // race probe (scripts/race_probe.py): waves >= 1 store their staged operands late, as they
    // do when their loads come back later than wave 0's (e.g. under a concurrent kernel chain)
    if ((tid >> 6) >= 1)
      for (int i = 0; i < 64; ++i) __builtin_amdgcn_s_sleep(127);
#endif
    rc_stage_all(
        rc_seg<NR>(pp2, [&](int e) { return A[e]; }, [&](int e, float v) {
          const int q = at(e);
          Al[q] = v;
          Ar[q] = fmaxf(v, 0.f);
        }),
        rc_seg<NR>((n - 1) * pp2, [&](int e) { return S[pp2 + e]; }, [&](int e, float v) { Sl[PP + at(e)] = v; }),
        // dS_i[c][c'] = fixed-order sum of the backward kernel's partial records
        rc_seg<NR>((n - 1) * pp2, [&](int e) {
          const int i = 1 + e / pp2, rem = e - (i - 1) * pp2, cc = rem / p, cp = rem - cc * p;
          float t = 0.f;
          if (fused || adj_inplace) {
            t = EmbWbSum(c, ws).nodes(cc * nch, 1, nch, ofs_s + (i - 1) * p + cp);
          } else {
            // DSB records' loads in flight per round and staged element (a runtime-count loop
            // waited for each load in turn: one memory latency per column chunk), added in record
            // order; 32 / NR keeps the NR elements' loads within 32 registers
            constexpr int DSB = NR <= 4 ? 8 : (32 / NR > 1 ? 32 / NR : 1);
            const float* q = ws + c.wo.dS + cc * c.dsCC + i * c.dsI + cp;
            for (int c0 = 0; c0 < c.dsN; c0 += DSB) {
              float v[DSB];
#pragma unroll
              for (int u = 0; u < DSB; ++u) v[u] = c0 + u < c.dsN ? q[(int64_t)(c0 + u) * c.dsS] : 0.f;
#pragma unroll
              for (int u = 0; u < DSB; ++u)
                if (c0 + u < c.dsN) t += v[u];
            }
          }
          return t;
        }, [&](int e, float v) { dSw[at(e)] = v; }),
        // adjacency-L1 gradient (summed over the factors by k_emb_bwd's reduce workgroups)
        rc_seg<NR>(adjL1 ? pp2 : 0, [&](int e) { return ws[c.wo.dAadj + e]; }, [&](int e, float v) { Sl[at(e)] = v; }));
#ifndef RC_PROBE_NO_BARRIER
    // Every LDS operand above was stored by the thread that loaded it; the row sums below read
    // whole rows, i.e. entries other waves stored.  Without this barrier a wave whose staging
    // loads returned early read relu(A) rows another wave had not stored yet (stale LDS), and
    // A's Adam step used a wrong D^-1/2 for those rows and columns: the intermittent A mismatch
    // of round 1 ("Root cause of the round-1 A mismatch").
    __syncthreads();
#endif
    RC_PHASE(c.ws, c.wo.total, wx, 50);
    for (int e = tid; e < pp2; e += RC_BLOCK) dL[at(e)] = 0.f;
    lds_rowsum(p, [&](int i, int j) { return Ar[i * P + j]; },
               [&](int i, float s) { dinv[i] = 1.f / sqrtf(s + 1e-10f); });
    __syncthreads();
    RC_PHASE(c.ws, c.wo.total, wx, 51);
#ifdef RC_ADJ_TWICE
    // timing experiment (trace builds, wrong results): the products below run twice, marks 55 / 56
    // after each pass -- a second pass much faster than the first means instruction fetch, not the
    // arithmetic, sets the phase's length
    for (int rep = 0; rep < 2; ++rep) {
#endif
    // back through S_l = S_{l-1} L, l = n-1 .. 2
    for (int l = n - 1; l >= 2; --l) {
      const float* dSl = dSw + (l - 1) * PP;
      float* dSprev = dSw + (l - 2) * PP;
      const float* Sprev = Sl + (l - 1) * PP;
      const float* Lm = Sl + PP;
      lds_mm_acc<false, true>(dSl, Lm, p, P, dSprev);  // dS_l L^T
      lds_mm_acc<true, false>(Sprev, dSl, p, P, dL);   // S_{l-1}^T dS_l
      __syncthreads();
    }
    if (n >= 2) {
      for (int e = tid; e < pp2; e += RC_BLOCK) {
        const int q = at(e);
        dL[q] += dSw[q];
      }
      __syncthreads();
    }
#ifdef RC_ADJ_TWICE
    RC_PHASE(c.ws, c.wo.total, wx, 55 + rep);
    }
#endif
    RC_PHASE(c.ws, c.wo.total, wx, 52);
    // normalize_A backward: L[i][j] = dinv_i relu(A)[i][j] dinv_j, dinv_i = (sum_j relu(A)[i][j] + 1e-10)^-1/2,
    // d(dinv)/d(sum) = -1/2 (sum + 1e-10)^-3/2
    lds_rowsum(p, [&](int i, int j) {
      return dL[i * P + j] * Ar[i * P + j] * dinv[j] + dL[j * P + i] * dinv[j] * Ar[j * P + i];
    }, [&](int i, float g) { dd[i] = g * (-0.5f) * dinv[i] * dinv[i] * dinv[i]; });
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int e = tid + u * RC_BLOCK;
      if (e < pp2) {
        const int i = dpv.div(e), j = e - i * p, q = i * P + j;
        float g = (Al[q] > 0.f) ? (dL[q] * dinv[i] * dinv[j] + dd[i]) : 0.f;
        if (adjL1) g += Sl[q];
        if (!adam) {
          c.gE[r * c.es + c.eo.A + e] = g;
        } else {
          float pv = Al[q], mv = mreg[u], vv = vreg[u];
          rc_adam(pv, mv, vv, g, as);
          A[e] = pv; Mm[c.eo.A + e] = mv; V[c.eo.A + e] = vv;
          Al[q] = pv;  // the new A for the supports below
        }
      }
    }
    __syncthreads();
    RC_PHASE(c.ws, c.wo.total, wx, 53);
    // supports of the updated A for the next step (after a gradient-only shard step A changes
    // later, in redcliff_adam_apply, and the host refreshes them)
    if (adam) supports_lds(dpv, Al, Sl, ws + c.wo.S, dinv, p, n);
#ifdef RC_ADJ_TWICE
    RC_PHASE(c.ws, c.wo.total, wx, 57);
    if (adam) supports_lds(dpv, Al, Sl, ws + c.wo.S, dinv, p, n);  // (same values again)
    RC_PHASE(c.ws, c.wo.total, wx, 58);
#endif
  }
  RC_PHASE(c.ws, c.wo.total, wx, 54);
  // BatchNorm running statistics (torch: double math, momentum*stat + (1-momentum)*running)
  if (c.nbn > 0 && tid < F) {
    const double* st = c.bns + r * c.bnsr;
    const double mom = c.hyp[r].bn_momentum;
    const double N = (double)c.Bg * p;  // unbiased correction over the global batch
    const double mean = st[tid], var_u = st[F + tid] * N / (N - 1.0);
    float rm = c.rm[r * F + tid], rv = c.rv[r * F + tid];
    for (int t = 0; t < c.nbn; ++t) {
      rm = (float)(mom * mean + (1.0 - mom) * (double)rm);
      rv = (float)(mom * var_u + (1.0 - mom) * (double)rv);
    }
    c.rm[r * F + tid] = rm;
    c.rv[r * F + tid] = rv;
  }
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FINAL, 1);
}

template <int NR>
__global__ __launch_bounds__(RC_BLOCK) void k_emb_final(StepCtx c, int nw, int ept) {
  rc_critical_priority();
  // the adjacency workgroups (the longest) are dispatched first for ALL replicas: linear
  // workgroup i < nrep is replica i's adjacency workgroup, the rest run the parameter updates
  // (R = 128 D4IC grid: the last replicas' adjacency workgroups no longer start behind ~10K
  // parameter workgroups)
  const int lin = blockIdx.x + blockIdx.y * gridDim.x;
  if (lin < c.nrep) {
    emb_final_wg<NR>(c, 0, lin, ept, false, false);
  } else {
    const int wy = (lin - c.nrep) / nw;
    emb_final_wg<NR>(c, 1 + (lin - c.nrep) - wy * nw, wy, ept, false, false);
  }
}

// k_emb_final as two launches for packed grids at small node counts: the one launch's register
// allocation is the adjacency workgroup's (k_emb_final<4>: 190 VGPRs + 16 AGPRs, 2 waves per SIMD), so
// its ~11 parameter workgroups per replica (R = 128 D4IC: 1,408) ran in three rounds; the parameter
// workgroups in a launch of their own take only the registers of the Adam pass.  The same device
// function per workgroup, so the same bits.  (At C5 the adjacency workgroup alone outlasts the
// combined launch -- measured, not used there.)
template <int NR>
__global__ __launch_bounds__(RC_BLOCK) void k_emb_final_adj(StepCtx c) {
  rc_critical_priority();
  emb_final_wg<NR>(c, 0, blockIdx.x, 1, false, false);
}
template <int NR>
__global__ __launch_bounds__(RC_BLOCK) void k_emb_final_params(StepCtx c, int ept) {
  rc_critical_priority();
  emb_final_wg<NR>(c, 1 + (int)(blockIdx.x & 0xffffff), blockIdx.y, ept, false, false);  // (wx > 0 provably: no adjacency code)
}

// k_emb_combine + k_emb_final as one launch (single fits with the fused embedder; round 3):
// workgroup 0 is the adjacency workgroup, which sums its dS partials in place (the sums
// k_emb_combine forms) and so starts at once; workgroups 1 .. ncomb are the combine's, which
// store their sums coherently and publish; the parameter workgroups after them wait for all
// ncomb and then read the combined records coherently.  Producers precede consumers in
// dispatch order and the whole grid is resident (rc_emb_tail_grid), as in k_bwd_merged; a wait
// that runs out of polls counts into the status word.  Same sums, same order: the same bits as
// the two launches (tests/test_gpu_forked.py).  grid (1 + ncomb + nw, R).
#ifndef TAIL_CE
#define TAIL_CE 1   // combine elements per thread in k_emb_tail (4: the grid fits C1(K=4) / TST but is slower)
#endif
#ifndef TAIL_EPT
#define TAIL_EPT 1  // parameter elements per thread in k_emb_tail (2: slower, r03_emb_tail_variants.jsonl)
#endif
template <int NR>
__global__ __launch_bounds__(RC_BLOCK) void k_emb_tail(StepCtx c, int ncx, int nw) {
  rc_critical_priority();
  const int ncomb = ncx * c.d.p * rc_nchunk(c.d);
  const int b = blockIdx.x, r = rc_rep(c, blockIdx.y);
  float* ws = c.ws + r * c.wss;
  unsigned* cnt = rc_tail_cnt(c, ws);
  if (b == 0) {
    emb_final_wg<NR>(c, 0, blockIdx.y, 1, false, true);
    return;
  }
  if (b <= ncomb) {
    const int q = b - 1, grp = q / ncx, x = q - grp * ncx;
    float t[TAIL_CE];
#pragma unroll
    for (int u = 0; u < TAIL_CE; ++u) t[u] = emb_combine_sum(c, r, grp, (x * TAIL_CE + u) * RC_BLOCK + threadIdx.x);
#pragma unroll
    for (int u = 0; u < TAIL_CE; ++u) emb_combine_store(c, r, grp, (x * TAIL_CE + u) * RC_BLOCK + threadIdx.x, t[u], true);
    rc_publish(cnt);
    return;
  }
  if (!(c.flags & RC_STEP_A)) return;
  rc_wait_count(cnt, (unsigned)ncomb, reinterpret_cast<unsigned*>(ws + c.wo.errw), RC_WAIT_POLLS);
  emb_final_wg<NR>(c, b - ncomb, blockIdx.y, TAIL_EPT, true, false);
}

// BatchNorm batch statistics for consecutive batches: one workgroup per (batch, feature),
// grid (nbatch, F, R).  Two double-precision passes over the batch's B*p values of that
// feature (the second pass re-reads them from L2), as torch's batch_norm statistics.
__global__ __launch_bounds__(RC_BLOCK) void k_bn_stats(RedcliffDims d, const float* X, int64_t xr, int64_t N,
                                                       int B, double* st, int64_t str) {
  const int r = blockIdx.z, bi = blockIdx.x, f = blockIdx.y;
  const int64_t b0 = (int64_t)bi * B;
  const int nb = (int)((N - b0) < B ? (N - b0) : B);
  const int p = d.p, F = d.F;
  const int Lmax = rc_lmax(d);
  const float* Xf = X + r * xr + (b0 * d.T + (Lmax - F + f)) * p;
  const int64_t rs = (int64_t)d.T * p;  // one window (row of the data set) to the next
  __shared__ double red[8];
  const int cnt = nb * p;
  double s = 0.0;
  for (int e = threadIdx.x; e < cnt; e += RC_BLOCK) {
    const int b = e / p, cc = e - b * p;
    s += Xf[b * rs + cc];
  }
  const double mean = rc_block_sum_d(s, red) / (double)cnt;
  double q = 0.0;
  for (int e = threadIdx.x; e < cnt; e += RC_BLOCK) {
    const int b = e / p, cc = e - b * p;
    const double v = Xf[b * rs + cc] - mean;
    q += v * v;
  }
  const double var = rc_block_sum_d(q, red) / (double)cnt;
  if (threadIdx.x == 0) {
    double* o = st + r * str + (int64_t)bi * 2 * F;
    o[f] = mean;
    o[F + f] = var;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// host launchers

size_t rc_emb_bwd_lds(const RedcliffDims& d, bool late) {
  const size_t head = 32 + (size_t)d.nsup * d.nsup;
  const int BC = rc_emb_bc(d);
  const size_t node = late ? rc_emb_node_alloc_floats(d, BC) : rc_emb_node_floats(d, BC);
  return (head > node ? head : node) * sizeof(float);
}

int rc_launch_emb_bwd(const StepCtx& c, hipStream_t s, bool node_wgs) {
  const RedcliffDims& d = c.d;
  const int BC = rc_emb_bc(d), WPB = rc_emb_wpb(d);
  const size_t lds = rc_emb_bwd_lds(d, WPB <= BC);  // the single-sub-block variant stages late
  if (lds > RC_LDS_MAX_FLOATS * sizeof(float)) { rc_set_error("embedder backward: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  const int nnode = node_wgs ? d.p * rc_nchunk(d) * ((c.B + WPB - 1) / WPB) : 0;
  const int head = (c.flags & (RC_VALUES | RC_CONFUSION)) ? 1 : 0;
  const bool dadj = (c.flags & RC_STEP_A) && (c.flags & RC_LOSS_ADJ);
  const int nred = dadj ? (d.p * d.p + RC_BLOCK - 1) / RC_BLOCK : 0;
  if (nnode + head + nred == 0) return 0;
  if (nnode == 0) {
    hipLaunchKernelGGL(k_emb_head_dadj, dim3(head + nred, c.nrep), dim3(RC_BLOCK), 0, s, c, head);
    return rc_check(hipGetLastError(), "k_emb_head_dadj");
  }
  if (WPB > BC) {
    int e = rc_lds_optin(k_emb_bwd<true>, lds, "k_emb_bwd LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_emb_bwd<true>, dim3(nnode + head + nred, c.nrep), dim3(RC_BLOCK), lds, s, c, nnode, head, BC, WPB);
  } else {
    int e = rc_lds_optin(k_emb_bwd<false>, lds, "k_emb_bwd LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_emb_bwd<false>, dim3(nnode + head + nred, c.nrep), dim3(RC_BLOCK), lds, s, c, nnode, head, BC, WPB);
  }
  return rc_check(hipGetLastError(), "k_emb_bwd");
}

// Workgroups of the merged launch, or 0 when it should not be used: the embedder side must be
// the single-sub-block variant (the multi-sub-block one needs 256 VGPRs), and the whole grid
// must be resident at once at the merged kernel's occupancy, as the runtime computes it from
// the kernel's VGPRs and this launch's LDS (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs;
// 174 VGPRs -> 2 workgroups of 256 lanes per CU at D4IC).  Residency is the performance
// condition (otherwise the factor body's register budget throttles the embedder workgroups and
// the two launches are faster: C1(K=4) 81 us merged vs 29 + 41 us) and the safety margin of
// the hand-off: with every workgroup resident no waiting consumer can hold a slot a producer
// needs, even if dispatch order were not monotone.  (Producers precede consumers in workgroup
// order and never wait, so in-order dispatch alone already guarantees progress; a poll that
// still runs out is reported through the status word, rc_wait_count.)
static int rc_bwd_merged_occupancy(size_t lds) {
  static thread_local size_t cached_lds = (size_t)-1;
  static thread_local int cached = 0;
  if (lds == cached_lds) return cached;
  int nb = 0;
  if (rc_lds_optin(k_bwd_merged<false>, lds, "k_bwd_merged LDS") != 0 ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_bwd_merged<false>, RC_BLOCK, lds) != hipSuccess)
    nb = 0;
  cached_lds = lds;
  cached = nb;
  return nb;
}

int rc_bwd_merged_grid(const StepCtx& c) {
  const RedcliffDims& d = c.d;
  if (rc_emb_wpb(d) > rc_emb_bc(d)) return 0;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  const int Q = d.p * d.L;
  const int nQ = (c.flags & RC_STEP_B) ? (Q + FB_QT - 1) / FB_QT : 1;
  const int nUl = (c.flags & RC_STEP_B) ? rc_nuchunk(d) : 1;
  const int WPB = rc_emb_wpb(d);
  const int nnode = d.p * rc_nchunk(d) * ((c.B + WPB - 1) / WPB);
  const int head = (c.flags & RC_CONFUSION) ? 1 : 0;
  const bool dadj = (c.flags & RC_STEP_A) && (c.flags & RC_LOSS_ADJ);
  const int nred = dadj ? (d.p * d.p + RC_BLOCK - 1) / RC_BLOCK : 0;
  const int grid = d.K * d.p * nUl * nQ + nnode + head + nred + (RC_MERGED_LEAD_SPLIT && (c.flags & RC_STEP_B) ? d.K * d.p : 0);
  const size_t le = rc_emb_bwd_lds(d, false), lf = sizeof(float) * (size_t)fac_bwd_lds_floats(d);
  const int occ = rc_bwd_merged_occupancy(le > lf ? le : lf);
  return (int64_t)grid * c.nrep <= (int64_t)occ * cus ? grid : 0;
}

// The merged backward (k_bwd_merged); requires the deferred combine (c.defer == 1) and no
// loss values (the head's loss sums read the factor leads' records).
int rc_launch_bwd_merged(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  if (c.defer != 1 || (c.flags & RC_VALUES)) { rc_set_error("merged backward: needs defer == 1 and no values"); return REDCLIFF_EINVAL; }
  const size_t le = rc_emb_bwd_lds(d, false), lf = sizeof(float) * (size_t)fac_bwd_lds_floats(d);
  const size_t lds = le > lf ? le : lf;
  if (lds > RC_LDS_MAX_FLOATS * sizeof(float)) { rc_set_error("merged backward: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  const int Q = d.p * d.L;
  const int nQ = (c.flags & RC_STEP_B) ? (Q + FB_QT - 1) / FB_QT : 1;
  const int nUl = (c.flags & RC_STEP_B) ? rc_nuchunk(d) : 1;
  const int BC = rc_emb_bc(d), WPB = rc_emb_wpb(d);
  const int nnode = d.p * rc_nchunk(d) * ((c.B + WPB - 1) / WPB);
  const int head = (c.flags & RC_CONFUSION) ? 1 : 0;
  const bool dadj = (c.flags & RC_STEP_A) && (c.flags & RC_LOSS_ADJ);
  const int nred = dadj ? (d.p * d.p + RC_BLOCK - 1) / RC_BLOCK : 0;
  const int KP = d.K * d.p;
  const int grid = KP * nUl * nQ + nnode + head + nred + (RC_MERGED_LEAD_SPLIT && (c.flags & RC_STEP_B) ? KP : 0);
  if (WPB > BC) {
    int e = rc_lds_optin(k_bwd_merged<true>, lds, "k_bwd_merged LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_bwd_merged<true>, dim3(grid, c.nrep), dim3(RC_BLOCK), lds, s, c, nUl, nQ, nnode, head, nred, BC, WPB);
  } else {
    int e = rc_lds_optin(k_bwd_merged<false>, lds, "k_bwd_merged LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_bwd_merged<false>, dim3(grid, c.nrep), dim3(RC_BLOCK), lds, s, c, nUl, nQ, nnode, head, nred, BC, WPB);
  }
  return rc_check(hipGetLastError(), "k_bwd_merged");
}

int rc_launch_cos_values(const StepCtx& c, hipStream_t s) {
  if (c.d.K < 2 || !(c.flags & RC_VALUES)) return 0;
  const int st = (c.d.K + 1) * c.d.p * c.d.p;
  const size_t lds = st <= COS_LDS ? sizeof(float) * st : 0;
  hipLaunchKernelGGL(k_cos_values, dim3((c.B + COS_WPW - 1) / COS_WPW, c.nrep), dim3(RC_BLOCK), lds, s, c);
  return rc_check(hipGetLastError(), "k_cos_values");
}

int rc_launch_emb_combine(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int pst = rc_emb_pstride(d);
  hipLaunchKernelGGL(k_emb_combine, dim3((pst + RC_BLOCK - 1) / RC_BLOCK, d.p * rc_nchunk(d), c.nrep), dim3(RC_BLOCK), 0,
                     s, c);
  return rc_check(hipGetLastError(), "k_emb_combine");
}

#ifndef RC_EMB_FINAL_SPLIT_NW
#define RC_EMB_FINAL_SPLIT_NW 32  // parameter workgroups per replica from which packed grids split k_emb_final
#endif
static size_t rc_emb_final_lds(const RedcliffDims& d) {
  return sizeof(float) * ((size_t)(2 * d.n + 2) * d.p * (d.p + 1) + 3 * 64);
}

// Workgroups of k_emb_tail per replica, or 0 when the two launches should be used: single fits
// (R = 1) whose whole grid is resident at the kernel's occupancy (runtime occupancy x CUs).
int rc_emb_tail_grid(const StepCtx& c) {
  const RedcliffDims& d = c.d;
  if (c.nrep != 1 || d.p * d.p > 4 * RC_BLOCK) return 0;
  const int total = d.n * d.F * d.H + d.K * d.M1 + d.K + d.M1 + 2 * d.F + d.M1 * d.p * d.H;
  const int nw = (total + TAIL_EPT * RC_BLOCK - 1) / (TAIL_EPT * RC_BLOCK);
  const int ncx = (rc_emb_pstride(d) + TAIL_CE * RC_BLOCK - 1) / (TAIL_CE * RC_BLOCK);
  const int grid = 1 + ncx * d.p * rc_nchunk(d) + nw;
  const size_t lds = rc_emb_final_lds(d);
  static thread_local size_t cached_lds = (size_t)-1;
  static thread_local int occ = 0;
  if (lds != cached_lds) {
    occ = 0;
    if (rc_lds_optin(k_emb_tail<4>, lds, "k_emb_tail LDS") != 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_emb_tail<4>, RC_BLOCK, lds) != hipSuccess)
      occ = 0;
    cached_lds = lds;
  }
  return grid <= occ * rc_cu_count() ? grid : 0;
}

int rc_launch_emb_tail(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int grid = rc_emb_tail_grid(c);
  if (grid == 0 || c.defer != 1) { rc_set_error("embedder tail launch: grid not resident or defer != 1"); return REDCLIFF_EINVAL; }
  const int total = d.n * d.F * d.H + d.K * d.M1 + d.K + d.M1 + 2 * d.F + d.M1 * d.p * d.H;
  const int nw = (total + TAIL_EPT * RC_BLOCK - 1) / (TAIL_EPT * RC_BLOCK);
  const int ncx = (rc_emb_pstride(d) + TAIL_CE * RC_BLOCK - 1) / (TAIL_CE * RC_BLOCK);
  const size_t lds = rc_emb_final_lds(d);
  int e = rc_lds_optin(k_emb_tail<4>, lds, "k_emb_tail LDS");
  if (e) return e;
  hipLaunchKernelGGL(k_emb_tail<4>, dim3(grid, c.nrep), dim3(RC_BLOCK), lds, s, c, ncx, nw);
  return rc_check(hipGetLastError(), "k_emb_tail");
}

int rc_launch_emb_final(const StepCtx& c, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int total = d.n * d.F * d.H + d.K * d.M1 + d.K + d.M1 + 2 * d.F + d.M1 * d.p * d.H;
  // parameter elements per thread: 4 from 8 replicas, 8 from 96 (R = 128 D4IC with the forked step:
  // 0.732 -> 0.728 ms, profiles/r04_grid_fork_sweep.log); REDCLIFF_EMB_FINAL_EPT overrides (tuning)
  const char* ev = getenv("REDCLIFF_EMB_FINAL_EPT");
  const int ept = (ev && atoi(ev) > 0) ? atoi(ev) : (c.nrep >= 96 ? 8 : (c.nrep >= 8 ? 4 : 1));
  const int nw = (total + ept * RC_BLOCK - 1) / (ept * RC_BLOCK);
  const size_t lds = rc_emb_final_lds(d);
  if (lds > RC_LDS_MAX_FLOATS * sizeof(float)) { rc_set_error("embedder final: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
  const char* sv = getenv("REDCLIFF_EMB_FINAL_SPLIT");  // read per launch (A/B): 0 one launch, 1 two
  // default: packed grids with many parameter workgroups per replica -- R = 128 TST (40 per replica)
  // 119.4 -> 112.1 us, step 1.027 -> 1.001 ms; R = 128 D4IC (11 per replica) 44.0-44.8 -> 48.3-49.1 us,
  // where the adjacency launch's own time is not won back (profiles/r06_emb_final_split_ab.jsonl)
  const bool split = sv ? sv[0] == '1' : (c.nrep >= 8 && nw >= RC_EMB_FINAL_SPLIT_NW);
  if (split && d.p * d.p <= 4 * RC_BLOCK) {
    int e = rc_lds_optin(k_emb_final_adj<4>, lds, "k_emb_final LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_emb_final_adj<4>, dim3(c.nrep), dim3(RC_BLOCK), lds, s, c);
    if ((e = rc_check(hipGetLastError(), "k_emb_final_adj"))) return e;
    hipLaunchKernelGGL(k_emb_final_params<4>, dim3(nw, c.nrep), dim3(RC_BLOCK), 0, s, c, ept);
    return rc_check(hipGetLastError(), "k_emb_final_params");
  }
  if (d.p * d.p <= 4 * RC_BLOCK) {
    int e = rc_lds_optin(k_emb_final<4>, lds, "k_emb_final LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_emb_final<4>, dim3(nw + 1, c.nrep), dim3(RC_BLOCK), lds, s, c, nw, ept);
  } else {
    int e = rc_lds_optin(k_emb_final<16>, lds, "k_emb_final LDS");
    if (e) return e;
    hipLaunchKernelGGL(k_emb_final<16>, dim3(nw + 1, c.nrep), dim3(RC_BLOCK), lds, s, c, nw, ept);
  }
  return rc_check(hipGetLastError(), "k_emb_final");
}

int rc_launch_supports(const RedcliffDims& d, const float* emb, int64_t es, float* ws, int64_t wss, EmbOff eo,
                       WsOff wo, hipStream_t s) {
  const size_t lds = sizeof(float) * ((size_t)(d.n + 1) * d.p * (d.p + 1) + 64);
  int e = rc_lds_optin(k_supports, lds, "k_supports LDS");
  if (e) return e;
  hipLaunchKernelGGL(k_supports, dim3(d.R), dim3(RC_BLOCK), lds, s, d, emb, es, ws, wss, eo, wo);
  return rc_check(hipGetLastError(), "k_supports");
}

int rc_launch_dp_update(const StepCtx& c, int64_t nE, int64_t nF, hipStream_t s) {
  const RedcliffDims& d = c.d;
  const int64_t per = (int64_t)RC_BLOCK * DPU_EPT;
  const bool sa = c.flags & RC_STEP_A, sb = c.flags & RC_STEP_B;
  const int64_t nbE = sa ? (nE + per - 1) / per : 0, nbF = sb ? (nF + per - 1) / per : 0;
  if (1 + nbE + nbF > 0x7fffffff) { rc_set_error("dp_update: parameter groups too large"); return REDCLIFF_ELIMIT; }
  const size_t lds = sizeof(float) * ((size_t)(d.n + 1) * d.p * (d.p + 1) + 64);
  int e = rc_lds_optin(k_dp_update, lds, "k_dp_update LDS");
  if (e) return e;
  hipLaunchKernelGGL(k_dp_update, dim3((unsigned)(1 + nbE + nbF), c.nrep), dim3(RC_BLOCK), lds, s, c, nE, nF, (int)nbE);
  return rc_check(hipGetLastError(), "k_dp_update");
}

int rc_launch_bn_stats(const RedcliffDims& d, const float* X, int64_t xr, int64_t N, int B, double* st, int64_t str,
                       hipStream_t s) {
  const int nbatch = (int)((N + B - 1) / B);
  hipLaunchKernelGGL(k_bn_stats, dim3(nbatch, d.F, d.R), dim3(RC_BLOCK), 0, s, d, X, xr, N, B, st, str);
  return rc_check(hipGetLastError(), "k_bn_stats");
}
