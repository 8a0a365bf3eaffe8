// rc_forward.hip -- forward half of the fused REDCLIFF-S step on gfx950: the DGCNN embedder
// and (vector path) the K x p factor networks, as ONE launch.
//
// The two forwards depend only on the window X and the parameters, so their workgroups share
// a grid: blocks [0, nemb) run the embedder on SB windows each, blocks [nemb, nemb + nfac) run
// one (factor, channel network, 16-unit hidden chunk) each.  One launch instead of two removes
// a kernel boundary and overlaps the two latency chains (at D4IC both are single waves of
// workgroups whose time is their own dependent global round trips).  Every workgroup issues
// all of its global loads in one multi-segment staging pass before computing.
//
// Reference: models/redcliff_factor_score_embedders.py:335-392 + models/dgcnn.py:15-64 +
// torcheeg 1.1.3 DGCNN (restated in oracle/torcheeg_dgcnn.py):
//   x_bn = BN1(x); L = D^-1/2 relu(A) D^-1/2; Z = sum_i (S_i x_bn) W_i; w = fc2(relu(fc1(vec(relu(Z)))))
// and models/cmlp.py:12-35 / :90-101 (MLP: Conv1d(p, h, L) -> ReLU -> Conv1d(h, 1, 1)),
// models/cmlp.py:147-167 (group norms of layer-0 weights, pre-update).
#include <cstdlib>
#include <type_traits>

#include "rc_common.h"

namespace {

#define FK_BT 128  // windows per factor-forward tile (16 row groups x 8)
#define FQ_MAX 96  // layer-0 contraction staged in one pass up to this length

__device__ inline int fq_tile(const RedcliffDims& d) { return d.p * d.L <= FQ_MAX ? d.p * d.L : 32; }

// ------------------------------------------------------------------------------------------
// Embedder forward of windows [bx*SB, bx*SB + SB).
//
// fc1 runs over channel slices of cs channels (columns [z*cs*H, min(p, (z+1)*cs)*H) of the p*H
// contraction, Zs = ceil(p / cs) slices): every slice's 64 lane chains are reduced on their own and
// f1 = ((part_0 + part_1) + ...) + fc1b, so the bits depend on cs only, never on how the slices are
// spread over workgroups.  zs < 0: this workgroup runs every slice of its windows.  zs >= 0 (one
// window per workgroup, the single fit): it runs slice zs only -- the Chebyshev rows, graph
// convolution and fc1 columns of its channels -- stores its fc1 partials write-through and counts
// itself in on the window's arrival counter; the workgroup that arrives last sums the partials in
// slice order and runs fc2.  No workgroup waits for another.
template <int NBT>
__device__ __attribute__((always_inline)) void emb_fwd_body(const StepCtx& c, int bx, int SB, int w_lds, int cs, int zs, float* sm) {
  const RedcliffDims& d = c.d;
  const int r = rc_rep(c, blockIdx.y);
  const int b0 = bx * SB;
  const int nb = min(SB, c.B - b0);
  if (nb <= 0) return;
  const int Zs = cs == (int)c.mg[RC_MG_CS] ? c.fzs : (d.p + cs - 1) / cs;
  const int zlo = zs < 0 ? 0 : zs, zhi = zs < 0 ? Zs : zs + 1;
  const int ch0 = zlo * cs, ch1 = min(d.p, zhi * cs);  // channels whose T / R rows this workgroup forms
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FWD, 0);
  RC_PHASE(c.ws, c.wo.total, bx, 0);
  const int p = d.p, F = d.F, H = d.H, n = d.n, M1 = d.M1, K = d.K;
  const int pF = p * F, pH = p * H, nFH = n * F * H;
  const RcDiv32 dF(F, c.mg[RC_MG_F]), dp(p, c.mg[RC_MG_P]), dpF(pF, c.mg[RC_MG_PF]), dH(H, c.mg[RC_MG_H]);
  const float* E = c.emb + r * c.es;
  float* ws = c.ws + r * c.wss;
  const float* X = c.X + r * c.xr;
  const int tid = threadIdx.x;

  float* xs = sm;                      // [SB][p][F]   raw window, then x_bn
  float* Sl = xs + SB * pF;            // [n][p][p]
  float* Wl = Sl + n * p * p;          // [n][F][H]    (w_lds)
  float* Tl = Wl + (w_lds ? nFH : 0);  // [SB][n][p][F]
  float* Rl = Tl + SB * n * pF;        // [SB][p*H]
  float* f1l = Rl + SB * pH;           // [SB][M1]
  float* fc2s = f1l + SB * M1;         // [K][M1]
  float* fb1 = fc2s + K * M1;          // [M1]
  float* fb2 = fb1 + M1;               // [K]
  float* alpha = fb2 + K;              // [F]
  float* beta = alpha + F;             // [F]

  if (blockIdx.x == 0) {  // arrival counters of the embedder backward (they also self-reset)
    unsigned* cnt = reinterpret_cast<unsigned*>(ws + c.wo.ecnt);
    for (int e = tid; e < p * rc_nchunk(d); e += RC_BLOCK) cnt[e] = 0u;
  }
  // BatchNorm statistics (torch forms the scale in double in train mode), issued first
  RC_PHASE(c.ws, c.wo.total, bx, 1);
  const bool train = c.flags & RC_BN_TRAIN;
  double st_mean = 0.0, st_var = 0.0;
  float bw = 0.f, bb = 0.f;
  if (tid < F) {
    if (train) {
      st_mean = c.bns[r * c.bnsr + tid];
      st_var = c.bns[r * c.bnsr + F + tid];
    } else {
      st_mean = c.rm[r * F + tid];
      st_var = c.rv[r * F + tid];
    }
    bw = E[c.eo.bnw + tid];
    bb = E[c.eo.bnb + tid];
  }
  const float* S = ws + c.wo.S;
  const float* gw = E + c.eo.gcW;
  // Loads per thread per segment sized so that the common shapes stage in ONE round (a second
  // round is another memory latency on every workgroup's path): n p^2 <= 512 (C1(K=4) 300, TST 432),
  // n F H <= 5,120 (4,800), K M1 <= 1,024 (TST 576)
  rc_stage_all(
      rc_seg<2>(n * p * p, [&](int e) { return S[e]; }, [&](int e, float v) { Sl[e] = v; }),
      rc_seg<20>(w_lds ? nFH : 0, [&](int e) { return gw[e]; }, [&](int e, float v) { Wl[e] = v; }),
      // window rows are contiguous in the channel index: read (s, f, ch), store [s][ch][f]
      rc_seg<4>(nb * pF, [&](int e) {
        const int s = dpF.div(e), rem = e - s * pF;
        return X[(c.row0 + b0 + s) * d.T * p + (int64_t)(c.Lmax - F) * p + rem];
      }, [&](int e, float v) {
        const int s = dpF.div(e), rem = e - s * pF, f = dp.div(rem), ch = rem - f * p;
        xs[s * pF + ch * F + f] = v;
      }),
      rc_seg<4>(K * M1, [&](int e) { return E[c.eo.fc2W + e]; }, [&](int e, float v) { fc2s[e] = v; }),
      rc_seg<1>(M1 + K, [&](int e) { return e < M1 ? E[c.eo.fc1b + e] : E[c.eo.fc2b + e - M1]; },
                [&](int e, float v) { fb1[e] = v; }));  // fb2 follows fb1
  RC_PHASE(c.ws, c.wo.total, bx, 2);
  if (tid < F) {
    // torch CPU batch_norm: y = x * alpha + beta, alpha = invstd * gamma, beta = bias - mean * alpha
    const float mean = (float)st_mean;
    const float inv = train ? (float)(1.0 / sqrt(st_var + c.hyp[r].bn_eps))
                            : 1.0f / sqrtf((float)st_var + (float)c.hyp[r].bn_eps);
    const float a = inv * bw;
    alpha[tid] = a;
    beta[tid] = bb - mean * a;
  }
  __syncthreads();
  for (int e = tid; e < nb * pF; e += RC_BLOCK) {
    const int f = dF.mod(e);
    xs[e] = xs[e] * alpha[f] + beta[f];
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, bx, 3);
  // Chebyshev filtering T_i = S_i x_bn (T_0 = x_bn exactly, as matmul(eye, x)), rows [ch0, ch1)
  const int cF = (ch1 - ch0) * F, cH = (ch1 - ch0) * H;
  // the slice width's multipliers (host-computed for the regular, the last and the whole width)
  const int cw = ch1 - ch0;
  const int mb = cw == (int)c.mg[RC_MG_CS] ? RC_MG_CSF : (cw == (int)c.mg[RC_MG_LS] ? RC_MG_LSF : -1);
  const RcDiv32 dcF = mb >= 0 ? RcDiv32(cF, c.mg[mb]) : (cw == p ? RcDiv32(cF, c.mg[RC_MG_PF]) : RcDiv32(cF));
  const RcDiv32 dncF = mb >= 0 ? RcDiv32(n * cF, c.mg[mb + 1]) : (cw == p ? RcDiv32(n * cF, c.mg[RC_MG_NPF]) : RcDiv32(n * cF));
  const RcDiv32 dcH = mb >= 0 ? RcDiv32(cH, c.mg[mb + 2]) : (cw == p ? RcDiv32(cH, c.mg[RC_MG_PH]) : RcDiv32(cH));
  for (int e = tid; e < nb * n * cF; e += RC_BLOCK) {
    const int s = dncF.div(e), rs = e - s * n * cF, i = dcF.div(rs), qs = rs - i * cF;
    const int q = ch0 * F + qs, rem = i * pF + q, ch = dF.div(q), f = q - ch * F;
    float v;
    if (i == 0) {
      v = xs[s * pF + q];
    } else {
      v = 0.f;
      const float* Srow = Sl + (i * p + ch) * p;
      const float* xc = xs + s * pF + f;
      for (int cc = 0; cc < p; ++cc) v += Srow[cc] * xc[cc * F];
    }
    Tl[s * n * pF + rem] = v;
    ws[c.wo.T + (int64_t)(b0 + s) * n * pF + rem] = v;
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, bx, 4);
  // fc1 weights of the first column step are issued before the graph convolution runs
  const float* W1 = E + c.eo.fc1W;
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int RW = (M1 + 3) / 4, m0 = wv * RW;
  // three buffers of column-step weights in rotation (p*H = 1,000 - 1,200 at C1 / TST is 16 - 19
  // column steps): each buffer is refilled right after it is multiplied and read two steps
  // later, with no register moves in between (a move of a loading register waits for the load).
  // Rows past M1 are wave-uniform zeros; a lane past p*H loads a clamped (valid) column that its
  // masked multiply never uses, so no load sits behind a lane-varying condition.
  auto qend = [&](int z) { return min(p, (z + 1) * cs) * H; };  // fc1 columns of slice z: [z*cs*H, qend(z))
  int qb = qend(zlo);
  auto ldw = [&](float (&w)[16], int qn) {
    const int qc = qn < qb ? qn : qb - 1;
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = (j < RW && m0 + j < M1) ? W1[(int64_t)(m0 + j) * pH + qc] : 0.f;
  };
  float wb0[16], wb1[16], wb2[16];
  ldw(wb0, zlo * cs * H + lane);
  ldw(wb1, zlo * cs * H + lane + 64);
  RC_PHASE(c.ws, c.wo.total, bx, 5);
  // Z = sum_i T_i W_i ; R = relu(Z)
  const float* Wsrc = w_lds ? Wl : gw;
  for (int e = tid; e < nb * cH; e += RC_BLOCK) {
    const int s = dcH.div(e), rem = ch0 * H + (e - s * cH), ch = dH.div(rem), hh = rem - ch * H;
    float a4[4] = {0.f, 0.f, 0.f, 0.f};  // four independent chains hide the LDS latency
    for (int i = 0; i < n; ++i) {
      const float* trow = Tl + (s * n + i) * pF + ch * F;
      const float* wc = Wsrc + i * F * H + hh;
      int f = 0;
      for (; f + 3 < F; f += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] += trow[f + u] * wc[(f + u) * H];
      }
      for (; f < F; ++f) a4[0] += trow[f] * wc[f * H];
    }
    const float v = fmaxf((a4[0] + a4[1]) + (a4[2] + a4[3]), 0.f);
    Rl[s * pH + rem] = v;
    ws[c.wo.R + (int64_t)(b0 + s) * pH + rem] = v;
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, bx, 6);
  // fc1: wave wv owns rows [wv*RW, wv*RW+RW) (RW <= 16); lanes split the slice's columns.
  // The next column step's weights are loaded while the current one is multiplied.
  // one window per workgroup (the single fit) multiplies only its own column: NB = 1 accumulators
  const int jrow = (lane >> 2) & 15, mrow = m0 + jrow;
  const bool wrow = (lane & 3) == 0 && jrow < RW && mrow < M1;  // the lane that holds row mrow's sum
  auto fc1 = [&](auto nbc) {
    constexpr int NB = decltype(nbc)::value;
    float tot[NB];  // row mrow of each window: the slice sums in slice order
    for (int z = zlo; z < zhi; ++z) {
      const int qa = z * cs * H;
      qb = qend(z);
      if (z > zlo) {  // the first slice's first two column steps were issued before the graph convolution
        ldw(wb0, qa + lane);
        ldw(wb1, qa + lane + 64);
      }
      float acc[16][NB];
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int s = 0; s < NB; ++s) acc[j][s] = 0.f;
      // column q of this lane (q ascending per lane: the same chains as one step per iteration)
      auto mul = [&](const float (&w)[16], int q) {
        if (q < qb) {
          float rv[NB];
#pragma unroll
          for (int s = 0; s < NB; ++s) rv[s] = s < nb ? Rl[s * pH + q] : 0.f;
#pragma unroll
          for (int j = 0; j < 16; ++j)
#pragma unroll
            for (int s = 0; s < NB; ++s) acc[j][s] += w[j] * rv[s];
        }
      };
      for (int q0 = qa; q0 < qb; q0 += 192) {  // wave-uniform steps of three column blocks
        const int q = q0 + lane;
        ldw(wb2, q + 128);
        mul(wb0, q);
        if (q0 + 64 >= qb) break;
        ldw(wb0, q + 192);
        mul(wb1, q + 64);
        if (q0 + 128 >= qb) break;
        ldw(wb1, q + 256);
        mul(wb2, q + 128);
      }
      // reduce-scatter of the 16 row partials over the 64 lanes: 17 shuffles per window instead of
      // 16 full reductions (96); afterwards lane l holds row (l >> 2) & 15 in every lane of its quad
#pragma unroll
      for (int s = 0; s < NB; ++s) {
        if (s >= nb) break;
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = acc[j][s];
#pragma unroll
        for (int half = 8; half >= 1; half >>= 1) {
          const int off = half * 4;  // lane bit that selects the kept half: 32, 16, 8, 4
          const bool hi = lane & off;
#pragma unroll
          for (int i = 0; i < half; ++i) {
            const float send = hi ? v[i] : v[i + half];
            const float keep = hi ? v[i + half] : v[i];
            v[i] = keep + __shfl_xor(send, off, 64);
          }
        }
        float t = v[0];
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 1, 64);
        tot[s] = z == zlo ? t : tot[s] + t;
      }
    }
    if (zs < 0) {  // every slice here: f1 = slice sums + bias
#pragma unroll
      for (int s = 0; s < NB; ++s) {
        if (s >= nb) break;
        if (wrow) {
          const float val = tot[s] + fb1[mrow];
          f1l[s * M1 + mrow] = val;
          ws[c.wo.f1 + (int64_t)(b0 + s) * M1 + mrow] = val;
        }
      }
    } else if (wrow) {  // this slice's partial, written through for the window's last workgroup
      rc_store_sc1(ws + c.wo.f1p + ((int64_t)zs * d.Bmax + b0) * M1 + mrow, tot[0]);
    }
  };
  fc1(std::integral_constant<int, NBT>{});  // NBT >= SB (k_forward's instantiation for this launch)
  if (zs >= 0) {  // arrival: the last of the window's Zs workgroups sums the partials and runs fc2
    __shared__ unsigned last;
    unsigned* cnt = reinterpret_cast<unsigned*>(ws + c.wo.ecnt) + p * rc_nchunk(d) + 2 + b0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its partials
    __syncthreads();
    if (tid == 0) last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(Zs - 1);
    __syncthreads();
    if (!last) return;
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler barrier only: the partial loads are sc1
    if (tid < M1) {
      // the slice partials' loads in flight together, eight per round (a runtime-count loop waited
      // for each load in turn), summed in slice order
      const float* part = ws + c.wo.f1p + (int64_t)b0 * M1 + tid;
      float sum = 0.f;
      for (int z0 = 0; z0 < Zs; z0 += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = z0 + u < Zs ? rc_load_sc1(part + (int64_t)(z0 + u) * d.Bmax * M1) : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (z0 + u < Zs) sum = z0 + u == 0 ? v[0] : sum + v[u];
      }
      const float val = sum + fb1[tid];
      f1l[tid] = val;
      ws[c.wo.f1 + (int64_t)b0 * M1 + tid] = val;
    }
  }
  __syncthreads();
  RC_PHASE(c.ws, c.wo.total, bx, 7);
  for (int e = tid; e < nb * K; e += RC_BLOCK) {
    const int s = e / K, k = e - s * K;
    const float* w2 = fc2s + k * M1;
    float a = 0.f;
    for (int m = 0; m < M1; ++m) a += w2[m] * fmaxf(f1l[s * M1 + m], 0.f);
    ws[c.wo.w + (int64_t)(b0 + s) * K + k] = a + fb2[k];
  }
  RC_PHASE(c.ws, c.wo.total, bx, 8);
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_EMB_FWD, 1);
}

size_t emb_fwd_floats(const RedcliffDims& d, int SB, int w_lds) {
  const size_t pF = (size_t)d.p * d.F, pH = (size_t)d.p * d.H;
  return SB * pF + (size_t)d.n * d.p * d.p + (w_lds ? (size_t)d.n * d.F * d.H : 0) + SB * d.n * pF + SB * pH +
         (size_t)SB * d.M1 + (size_t)d.K * d.M1 + d.M1 + d.K + 2 * d.F;
}

// ------------------------------------------------------------------------------------------
// Factor forward of one (factor, channel network, FAC_UC-unit hidden chunk): relu activations
// a[kj][b][u], partial outputs y[uc][kj][b] = sum_{u in chunk} W1[u] a[b][u] (+ b1 in chunk
// 0), the chunk's squared layer-0 group norms gq[uc][kj][q] and a snapshot of W1.
// The whole window block and weight chunk are staged in one pass when p*L <= FQ_MAX.
template <class Div>
__device__ inline float xwin(const StepCtx& c, const Div& dL, const float* X, int b, int q) {
  const int L = c.d.L;
  const int ch = dL.div(q), t = q - ch * L;
  return X[((c.row0 + b) * c.d.T + (c.Lmax - L + t)) * c.d.p + ch];
}

__device__ __attribute__((always_inline)) void fac_fwd_body(const StepCtx& c, int bx, float* sm) {
  const RedcliffDims& d = c.d;
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_FWD, 0);
  const int nU = rc_nuchunk(d);
  const int r = rc_rep(c, blockIdx.y), kj = bx / nU, uc = bx - kj * nU;
  const int p = d.p, h = d.h, K = d.K;
  const int k = kj / p, j = kj - k * p;
  const int Q = p * d.L, QT = fq_tile(d), QP = QT + 1;
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
  const RcDiv dL(d.L), dQT(QT);
  float* Xs = sm;                // [FK_BT][QT+1]
  float* Ws = Xs + FK_BT * QP;   // [FAC_UC][QT+1]
  const float bu = u < h ? b0[u] : 0.f, w1 = u < h ? W1[u] : 0.f;

  for (int bc = 0; bc < c.B; bc += FK_BT) {
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int q0 = 0; q0 < Q; q0 += QT) {
      if (q0 > 0 || bc > 0) __syncthreads();
      rc_stage_all(
          rc_seg<24>(FK_BT * QT, [&](int e) {
            const int bb = dQT.div(e), qq = e - bb * QT;
            const int b = bc + bb, q = q0 + qq;
            return (b < c.B && q < Q) ? xwin(c, dL, X, b, q) : 0.f;
          }, [&](int e, float v) { Xs[dQT.div(e) * QP + dQT.mod(e)] = v; }),
          rc_seg<4>(FAC_UC * QT, [&](int e) {
            const int uu = dQT.div(e), qq = e - uu * QT;
            const int q = q0 + qq;
            return (u0 + uu < h && q < Q) ? W0[(int64_t)(u0 + uu) * Q + q] : 0.f;
          }, [&](int e, float v) { Ws[dQT.div(e) * QP + dQT.mod(e)] = v; }));
      __syncthreads();
      if (bc == 0)
        for (int qq = tid; qq < QT && q0 + qq < Q; qq += RC_BLOCK) {
          // squared group norms of the chunk's 16 units (GC, models/cmlp.py:162-166), pre-update
          float sq = 0.f;
          for (int uu = 0; uu < FAC_UC; ++uu) {
            const float w = Ws[uu * QP + qq];
            sq += w * w;
          }
          ws[c.wo.gq + ((int64_t)uc * K * p + kj) * Q + q0 + qq] = sq;
        }
      const int qn = min(QT, Q - q0);
#pragma unroll 8
      for (int qq = 0; qq < qn; ++qq) {
        const float wv = Ws[tu * QP + qq];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(Xs[(tb + 16 * i) * QP + qq], wv, acc[i]);  // rc_fac_bwd.h recomputes this chain
      }
    }
    if (bc == 0 && tb == 0 && u < h) ws[c.wo.w1 + (int64_t)kj * h + u] = w1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int b = bc + tb + 16 * i;
      float ys = 0.f;
      if (u < h) {
        const float a = fmaxf(acc[i] + bu, 0.f);
        if (b < c.B && !rc_fac_recompute(d)) ws[c.wo.a + ((int64_t)kj * d.Bmax + b) * h + u] = a;
        ys = w1 * a;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) ys += __shfl_xor(ys, o, 64);
      if (tu == 0 && b < c.B) ws[c.wo.y + rc_y_idx(d, uc, kj, b)] = ys + b1;
    }
  }
  RC_WG_MARK(c.ws, c.wo.total, RC_KID_FAC_FWD, 1);
}

size_t fac_fwd_floats(const RedcliffDims& d) {
  const int QT = d.p * d.L <= FQ_MAX ? d.p * d.L : 32;
  return (size_t)(FK_BT + FAC_UC) * (QT + 1);
}

// grid (nemb + nfac, R): embedder blocks first, then factor blocks.
// split: one (window, channel slice) per embedder workgroup (SB = 1), window-major.  NBT: the fc1
// accumulator columns (windows per workgroup, SB <= NBT): one instantiation per SB keeps the
// single fit's kernel (NBT = 1) at its own register count, not the 4-window one's.
template <int NBT>
__global__ __launch_bounds__(RC_BLOCK) void k_forward(StepCtx c, int SB, int w_lds, int nemb, int cs, int split) {
  extern __shared__ float sm[];
  // every step with an embedder forward re-arms the merged backward's factor-lead counter (the
  // kernel boundary orders this store before k_bwd_merged's polls)
  if (blockIdx.x == 0 && nemb > 0 && threadIdx.x == 0) {  // the counters of this step's later launches
    unsigned* lc = rc_fac_lead_cnt(c, c.ws + rc_rep(c, blockIdx.y) * c.wss);
    lc[0] = 0u;  // merged backward: published factor leads
    lc[1] = 0u;  // k_emb_tail: published combine workgroups
  }
  if ((int)blockIdx.x < nemb) {
    if (split) {
      const RcDiv32 dZs = cs == (int)c.mg[RC_MG_CS] ? RcDiv32(c.fzs, c.mg[RC_MG_ZS]) : RcDiv32((c.d.p + cs - 1) / cs);
      const int Zs = dZs.d, b = dZs.div(blockIdx.x);
      emb_fwd_body<NBT>(c, b, 1, w_lds, cs, blockIdx.x - b * Zs, sm);
    } else {
      emb_fwd_body<NBT>(c, blockIdx.x, SB, w_lds, cs, -1, sm);
    }
  } else
    fac_fwd_body(c, blockIdx.x - nemb, sm);
}

}  // namespace

// Dynamic LDS above 64 KiB (up to the CU's 160 KiB) must be opted into per kernel.
template <class Kern>
static int lds_optin(Kern k, size_t bytes, const char* what) {
  if (bytes <= RC_LDS_LIMIT_FLOATS * sizeof(float)) return 0;
  return rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bytes), what);
}

// Channels per fc1 slice of the embedder forward (emb_fwd_body): slices of about RC_EMB_FWD_COLS
// columns of the p*H contraction (REDCLIFF_EMB_FWD_COLS overrides; 0 = one slice).  A function of
// the model's dimensions only -- never of R or the windows per workgroup -- so a packed fit and an
// independent one sum fc1 in the same slices (bit for bit).
#ifndef RC_EMB_FWD_COLS
#define RC_EMB_FWD_COLS 200
#endif
int rc_emb_fwd_slice_channels(const RedcliffDims& d) {
  static const int cols = [] {
    const char* v = getenv("REDCLIFF_EMB_FWD_COLS");
    return v ? atoi(v) : RC_EMB_FWD_COLS;
  }();
  if (cols <= 0) return d.p;
  int cs = cols / d.H > 1 ? cols / d.H : 1;
  const int cmin = (d.p + 63) / 64;  // at most 64 slices (the partial region's slots)
  if (cs < cmin) cs = cmin;
  return cs < d.p ? cs : d.p;
}

void rc_ctx_magics(StepCtx& c) {
  const RedcliffDims& d = c.d;
  const int cs = rc_emb_fwd_slice_channels(d), Zs = (d.p + cs - 1) / cs, ls = d.p - (Zs - 1) * cs;
  const long long v[RC_MG_NCH] = {d.F, d.p, (long long)d.p * d.F, (long long)d.n * d.F, d.K, d.M1, d.H, d.L, c.B,
                                (long long)d.n * d.p * d.F, (long long)d.p * d.H,
                                0, (long long)cs * d.F, (long long)d.n * cs * d.F, (long long)cs * d.H,
                                0, (long long)ls * d.F, (long long)d.n * ls * d.F, (long long)ls * d.H};
  c.ewpb = rc_emb_wpb(d);
  c.enbwm = rc_emb_nbw(d);
  c.enbw = (c.B + c.ewpb - 1) / c.ewpb;
  for (int i = 0; i < RC_MG_NCH; ++i) c.mg[i] = rc_magic32(v[i]);
  c.mg[RC_MG_NCH] = rc_magic32(rc_nchunk(d));
  c.mg[RC_MG_ENBW] = rc_magic32(c.enbw);
  c.fzs = Zs;
  c.mg[RC_MG_ZS] = rc_magic32(Zs);
  c.mg[RC_MG_CS] = (unsigned)cs;  // the widths themselves (the slice's width picks its slots)
  c.mg[RC_MG_LS] = (unsigned)ls;
}

// One launch of the embedder forward (with_emb) and / or the vector-path factor forward (with_fac).
int rc_launch_forward(const StepCtx& c, hipStream_t s, bool with_emb, bool with_fac, hipEvent_t stop) {
  const RedcliffDims& d = c.d;
  int SB = 1, w_lds = 1, nemb = 0, split = 0;
  const int cs = rc_emb_fwd_slice_channels(d);
  size_t lds = 0;
  if (with_emb) {
    static const int sb_env = [] {
      const char* v = getenv("REDCLIFF_EMB_SB");  // tuning knob: windows per forward workgroup
      const int x = v ? atoi(v) : 0;
      return (x >= 1 && x <= 4) ? x : 0;  // the fc1 stage holds at most 4 windows per workgroup
    }();
    // one window per workgroup keeps a single fit's forward short (latency); packed replicas
    // fill the chip anyway, and 4 windows per workgroup share one staging of the embedder
    // weights (R = 32 D4IC grid: forward 158 -> 64 us).  Per-window arithmetic does not
    // depend on SB, so packed fits stay bitwise equal to independent ones.
    SB = sb_env ? sb_env : (d.R >= 8 ? 4 : 1);
    size_t limit = RC_LDS_LIMIT_FLOATS;
    while (SB > 1 && emb_fwd_floats(d, SB, w_lds) > limit) --SB;
    if (emb_fwd_floats(d, SB, w_lds) > limit) w_lds = 0;
    if (emb_fwd_floats(d, SB, w_lds) > limit) limit = RC_LDS_MAX_FLOATS;  // large p*F: one workgroup per CU
    if (emb_fwd_floats(d, SB, w_lds) > limit) { rc_set_error("embedder forward: LDS budget exceeded"); return REDCLIFF_ELIMIT; }
    lds = emb_fwd_floats(d, SB, w_lds);
    nemb = (c.B + SB - 1) / SB;
    if (SB == 1 && cs < d.p) {  // one window per workgroup: its slices on workgroups of their own
      split = 1;
      nemb = c.B * ((d.p + cs - 1) / cs);
    }
  }
  int nfac = 0;
  if (with_fac) {
    if (d.h > 128 || d.p * d.L > 4096) { rc_set_error("factor forward: h <= 128 and p*L <= 4096 required"); return REDCLIFF_ELIMIT; }
    nfac = d.K * d.p * rc_nuchunk(d);
    const size_t f = fac_fwd_floats(d);
    lds = f > lds ? f : lds;
  }
  if (nemb + nfac == 0) return 0;
  lds *= sizeof(float);
  auto launch = [&](auto kern) {
    int e = lds_optin(kern, lds, "k_forward LDS");
    if (e) return e;
    if (stop)
      hipExtLaunchKernelGGL(kern, dim3(nemb + nfac, c.nrep), dim3(RC_BLOCK), lds, s, nullptr, stop, 0, c, SB, w_lds, nemb,
                            cs, split);
    else
      hipLaunchKernelGGL(kern, dim3(nemb + nfac, c.nrep), dim3(RC_BLOCK), lds, s, c, SB, w_lds, nemb, cs, split);
    return rc_check(hipGetLastError(), "k_forward");
  };
  if (SB == 1) return launch(k_forward<1>);
  if (SB == 2) return launch(k_forward<2>);
  return launch(k_forward<4>);
}

int rc_launch_fac_fwd(const StepCtx& c, hipStream_t s) { return rc_launch_forward(c, s, false, true); }
