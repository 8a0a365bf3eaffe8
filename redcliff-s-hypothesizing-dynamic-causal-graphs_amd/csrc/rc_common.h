// rc_common.h -- shared layout / context definitions for the REDCLIFF-S gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include "redcliff_hip.h"

#define RC_BLOCK 256
#define RC_TRACE_FLOATS 32768  // trace builds: u64 timing slots at the end of the workspace (8 kernels x 2048)
#define RC_LDS_LIMIT_FLOATS 16384  // 64 KiB of dynamic LDS per workgroup (several workgroups per CU)
#define RC_LDS_MAX_FLOATS 40960    // 160 KiB: the whole CU's LDS, used only when a tile needs it (large p)
#define RC_MAX_ACTIVE 256          // longest active-replica list of one launch (RedcliffStepArgs.replicas)

// Offsets (in floats) inside one replica's packed embedder parameters.
struct EmbOff {
  int64_t A, gcW, bnw, bnb, fc1W, fc1b, fc2W, fc2b, total;
};
// Offsets inside one replica's packed factor parameters.
struct FacOff {
  int64_t W0, b0, W1, b1, total;
};
// Offsets (in floats) inside one replica's workspace slice.
struct WsOff {
  int64_t T;      // [Bmax][n][p][F]   Chebyshev-filtered embedder inputs S_i x
  int64_t R;      // [Bmax][p][H]      relu(graph-conv) activations
  int64_t f1;     // [Bmax][M1]        fc1 pre-activation
  int64_t w;      // [Bmax][K]         raw embedder output (pre-sigmoid)
  int64_t a;      // [K][p][Bmax][h]   factor hidden activations (reused for dz)
  int64_t y;      // [nU][Bmax][K][p]  per-factor predictions, partial over 16-unit hidden chunks
  int64_t G;      // [K][p][p][L]      lagged group norms of W0
  int64_t G0;     // [K][p][p]         lag-free group norms of W0
  int64_t w1;     // [K][p][h]         pre-update snapshot of the factor output weights
  int64_t gq;     // [nU][K][p][p*L]   squared layer-0 group norms, partial over hidden chunks
  int64_t ebp;    // [p*nch][nbw][pst] embedder-backward partials per (node, chunk, window block)
  int64_t ecnt;   // [p*nch + 2 + Bmax] arrival counters of those blocks (u32, self-resetting); the
                  //                   next two slots count published factor-lead workgroups (k_bwd_merged)
                  //                   and combine workgroups (k_emb_tail), the last Bmax the channel-slice
                  //                   workgroups of each window (k_forward, self-resetting)
  int64_t gfc1;   // [M1][p*H]         fc1 weight gradient (combined by the node blocks)
  int64_t dwp;    // [p][Bmax][K]      per-channel partial dL/dw
  int64_t dAadj;  // [K][p][p]         adjacency-L1 gradient wrt A, per factor
  int64_t dWi;    // [max(p, Bmax/16)][n][F][H] graph-conv weight gradient partials (per node / tile)
  int64_t dS;     // [p][nch][n][p]    gradient wrt Chebyshev supports (row c, partial per column chunk)
  int64_t dgb;    // [p][nch][2][F]    BatchNorm affine gradient partials (per node and chunk)
  int64_t S;      // [n][p][p]         supports (S_0 = I)
  int64_t dZ;     // [p][Bmax][H]      graph-conv output gradient per node
  int64_t amat;   // [8][p][p]         scratch for the adjacency backward
  int64_t lossp;  // [p + K*p + 8]     per-batch loss partials
  int64_t xsim;   // [Bmax][p]         mixed forecast
  int64_t gfc;    // [K*M1 + K + M1]   fc2W / fc2b / fc1b gradients (applied in the final kernel)
  int64_t xw;     // [Bmax][Qp]        factor input windows, q = c*L + t (MFMA path; Qp = Q rounded to 32)
  int64_t dyl;    // [K*p][Bmax]       dL/d(prediction of network kj) per window (MFMA path)
  int64_t dgs;    // [K*p][p*L]        adjacency-L1 gradient wrt the lagged group norms (MFMA path)
  int64_t f1p;    // [64][Bmax][M1]    fc1 split-K partials (GEMM embedder) / channel-slice partials (k_forward)
  int64_t edf1;   // [Bmax][M1]        dL/d fc1 pre-activation (GEMM embedder)
  int64_t edT;    // [Bmax][p][n][F]   dL/dT_i (GEMM embedder; T itself is [Bmax][p][n][F] there)
  int64_t edX;    // [Bmax][p][F]      dL/d x_bn (GEMM embedder)
  int64_t eAf;    // [p][p*n]          [S_0^T | ... | S_{n-1}^T] interleaved (GEMM embedder)
  int64_t edr;    // [Bmax][K]         dL/d(raw embedder output) (GEMM embedder)
  int64_t cosb;   // [Bmax] doubles    per-window cosine-similarity penalty values
  int64_t errw;   // [16] u32          device status words, never reset by a kernel: [0] counts the
                  //                   merged backward's hand-off waits that timed out (rc_wait_count);
                  //                   read and cleared by redcliff_device_status
  int64_t total;
};

__host__ __device__ inline int rc_lmax(const RedcliffDims& d) { return d.L > d.F ? d.L : d.F; }
__host__ __device__ inline int rc_ls(const RedcliffDims& d) { return d.L < d.F ? d.L : d.F; }

inline EmbOff rc_emb_off(const RedcliffDims& d) {
  EmbOff o;
  int64_t x = 0;
  o.A = x; x += (int64_t)d.p * d.p;
  o.gcW = x; x += (int64_t)d.n * d.F * d.H;
  o.bnw = x; x += d.F;
  o.bnb = x; x += d.F;
  o.fc1W = x; x += (int64_t)d.M1 * d.p * d.H;
  o.fc1b = x; x += d.M1;
  o.fc2W = x; x += (int64_t)d.K * d.M1;
  o.fc2b = x; x += d.K;
  o.total = x;
  return o;
}

inline FacOff rc_fac_off(const RedcliffDims& d) {
  FacOff o;
  int64_t x = 0;
  int64_t kp = (int64_t)d.K * d.p;
  o.W0 = x; x += kp * d.h * d.p * d.L;
  o.b0 = x; x += kp * d.h;
  o.W1 = x; x += kp * d.h;
  o.b1 = x; x += kp;
  o.total = x;
  return o;
}

// graph-conv hidden columns per embedder-backward workgroup
#define EMB_HC 16
__host__ __device__ inline int rc_nchunk(const RedcliffDims& d) { return (d.H + EMB_HC - 1) / EMB_HC; }
// factor hidden units per factor-kernel workgroup
#define FAC_UC 16
// vector factor path: with p*L <= 64 (one dW0 column tile) the backward recomputes the hidden
// activations from the window and W0 instead of the forward storing them (rc_fac_bwd.h)
__host__ __device__ inline bool rc_fac_recompute(const RedcliffDims& d) { return d.p * d.L <= 64; }
__host__ __device__ inline int rc_nuchunk(const RedcliffDims& d) { return (d.h + FAC_UC - 1) / FAC_UC; }

// Embedder backward node blocks: BC windows each (16, fewer if the LDS tiles do not fit).
__host__ __device__ inline int rc_emb_node_floats(const RedcliffDims& d, int BC) {
  const int nF = d.n * d.F;
  return 4 * BC * d.K + d.K * d.M1 + d.M1 * EMB_HC + nF * (EMB_HC + 1) + d.n * d.p + 8 + 4 * d.F + RC_BLOCK +
         BC * (2 * d.M1 + 2 * EMB_HC + 2 * nF + d.p * d.F);
}
// RC_EMB_LATE_X (experiment): the raw window tile of an embedder-backward sub-block is staged
// after the dW_i phase into the LDS of the tiles that are dead by then (f1, df1, R, dZ, T), when
// it fits there; the allocation shrinks by BC*p*F floats.  BC is still chosen on the full size,
// so the arithmetic (and the bits) do not change.
#ifndef RC_EMB_LATE_X
#define RC_EMB_LATE_X 0
#endif
__host__ __device__ inline bool rc_emb_late_x(const RedcliffDims& d) {
  return RC_EMB_LATE_X && d.p * d.F <= 2 * d.M1 + 2 * EMB_HC + d.n * d.F;
}
__host__ __device__ inline int rc_emb_node_alloc_floats(const RedcliffDims& d, int BC) {
  return rc_emb_node_floats(d, BC) - (rc_emb_late_x(d) ? BC * d.p * d.F : 0);
}
// Windows per LDS sub-block: as many as fit the 64 KiB budget; with fewer than 4 (large p*F)
// the budget grows to the CU's 160 KiB.
__host__ __device__ inline int rc_emb_bc(const RedcliffDims& d) {
  int BC = 16;
  while (BC > 1 && rc_emb_node_floats(d, BC) > RC_LDS_LIMIT_FLOATS) BC >>= 1;
  if (BC >= 4) return BC;
  BC = 16;
  while (BC > 1 && rc_emb_node_floats(d, BC) > RC_LDS_MAX_FLOATS) BC >>= 1;
  return BC;
}
// Windows per (node, chunk) workgroup: a multiple of BC, processed as sequential sub-blocks.
// Enough window blocks to give the launch ~1024 workgroups, never more than ceil(Bmax/BC).
__host__ __device__ inline int rc_emb_wpb(const RedcliffDims& d) {
  const int BC = rc_emb_bc(d);
  const int groups = d.p * rc_nchunk(d);
  const int target = (1024 + groups - 1) / groups;
  const int nblk = (d.Bmax + BC - 1) / BC;
  const int nbw = nblk < target ? nblk : target;
  return BC * ((nblk + nbw - 1) / nbw);
}
__host__ __device__ inline int rc_emb_nbw(const RedcliffDims& d) { return (d.Bmax + rc_emb_wpb(d) - 1) / rc_emb_wpb(d); }
// floats per partial record: fc1 chunk | W_i chunk | dS rows i >= 1 | dgamma | dbeta | fc2W fc2b fc1b (group 0)
__host__ __device__ inline int rc_emb_pstride(const RedcliffDims& d) {
  return d.M1 * EMB_HC + d.n * d.F * EMB_HC + (d.n - 1) * d.p + 2 * d.F + d.K * d.M1 + d.K + d.M1;
}

inline int64_t rc_align64(int64_t x) { return (x + 63) & ~(int64_t)63; }
// layer-0 contraction length p*L rounded up to the MFMA staging chunk
__host__ __device__ inline int rc_qpad(const RedcliffDims& d) { return (d.p * d.L + 31) & ~31; }

// Verification mode (redcliff_debug_guard_bands): every workspace region is followed by a
// guard band of this many floats, the last one doubling as the band after replica R-1, so a
// test can fill the bands with a NaN pattern and find any write past a region's end (the band
// changes) or read past it (NaN reaches the results).  0 in production.
extern int rc_ws_guard_floats;
#define RC_WS_MAX_REGIONS 40

// Region layout of one replica's workspace slice.  ext (optional) receives (start, size) of
// every region in layout order; *next its count.
inline WsOff rc_ws_off(const RedcliffDims& d, int64_t* ext = nullptr, int* next = nullptr) {
  WsOff o;
  int64_t x = 0;
  int nr = 0;
  const int64_t G = rc_ws_guard_floats;
  auto put = [&](int64_t& field, int64_t n) {
    field = x;
    if (ext && nr < RC_WS_MAX_REGIONS) { ext[2 * nr] = x; ext[2 * nr + 1] = n; }
    ++nr;
    x = rc_align64(x + n + G);
  };
  const int64_t B = d.Bmax, p = d.p, K = d.K;
  put(o.T, B * d.n * p * d.F);
  put(o.R, B * p * d.H);
  put(o.f1, B * d.M1);
  put(o.w, B * K);
  put(o.a, K * p * B * d.h);
  put(o.y, (int64_t)rc_nuchunk(d) * B * K * p);
  put(o.G, K * p * p * d.L);
  put(o.G0, K * p * p);
  put(o.w1, K * p * d.h);
  put(o.gq, (int64_t)rc_nuchunk(d) * K * p * p * d.L);
  put(o.ebp, (int64_t)p * rc_nchunk(d) * rc_emb_nbw(d) * rc_emb_pstride(d));
  // + the merged backward's factor-lead counter + k_emb_tail's + one per window (split embedder forward)
  put(o.ecnt, p * rc_nchunk(d) + 2 + B);
  put(o.gfc1, (int64_t)d.M1 * p * d.H);
  put(o.dwp, p * B * K);
  put(o.dAadj, K * p * p);
  // per-node slices (node-chunk / GEMM paths); the bound by 16-window tiles is kept from the removed
  // replica-batched embedder (round 5) and only over-allocates when ceil(B / 16) > p
  put(o.dWi, (p > (B + 15) / 16 ? p : (B + 15) / 16) * d.n * d.F * d.H);
  put(o.dS, (rc_nchunk(d) > 64 ? rc_nchunk(d) : 64) * d.n * p * p);
  put(o.dgb, (p * rc_nchunk(d) > 64 ? p * rc_nchunk(d) : 64) * 2 * d.F);
  put(o.S, d.n * p * p);
  put(o.dZ, p * B * d.H);
  put(o.amat, 8 * p * p);
  put(o.lossp, p + K * p + 8);
  put(o.xsim, B * p);
  put(o.gfc, K * d.M1 + K + d.M1);
  put(o.xw, B * rc_qpad(d));
  put(o.dyl, K * p * B);
  put(o.dgs, K * p * p * d.L);
  put(o.f1p, 64 * B * d.M1);
  put(o.edf1, B * d.M1);
  put(o.edT, B * p * d.n * d.F);
  put(o.edX, B * p * d.F);
  put(o.eAf, p * p * d.n);
  put(o.edr, B * K);
  put(o.cosb, 2 * B);
  put(o.errw, 16);
#ifdef RC_TRACE
  x += RC_TRACE_FLOATS;  // phase-timing slots at the end of the workspace (trace builds only)
#endif
  o.total = x;
  if (next) *next = nr < RC_WS_MAX_REGIONS ? nr : RC_WS_MAX_REGIONS;
  return o;
}

// Slots of the per-batch loss partials (after the p + K*p per-network entries).
#define LP_FACTOR 0
#define LP_FWL1 1
#define LP_COS 2
#define LP_SMOOTH 3
// Validation accumulator slots (coefficient-normalised, validate_training :1704-1729).
#define ACC_FORECAST 0
#define ACC_FACTOR 1
#define ACC_COS 2
#define ACC_FWL1 3
#define ACC_SMOOTH 4
#define ACC_ADJ 5
#define ACC_COMBO 6
#define ACC_BATCHES 7

// Everything a step kernel needs, passed by value.
// StepCtx::mg slots: F, p, p F, n F, K, M1, H, L, B, n p F, p H, and per fc1 slice width of the
// embedder forward (cw channels: the regular width cs and the last slice's): cw F, n cw F, cw H
enum {
  RC_MG_F, RC_MG_P, RC_MG_PF, RC_MG_NF, RC_MG_K, RC_MG_M1, RC_MG_H, RC_MG_L, RC_MG_B, RC_MG_NPF, RC_MG_PH,
  RC_MG_CS, RC_MG_CSF, RC_MG_NCSF, RC_MG_CSH, RC_MG_LS, RC_MG_LSF, RC_MG_NLSF, RC_MG_LSH, RC_MG_NCH, RC_MG_ENBW,
  RC_MG_ZS, RC_MG_N
};

struct StepCtx {
  RedcliffDims d;
  int B, Lmax, Ls, flags, nbn;
  int Bg;      // windows of the global batch (data-parallel normalisation; == B on one device)
  int tA, tB;  // Adam step numbers (1-based)
  const float* X; int64_t xr; int64_t row0;
  const float* lab; int64_t labr;
  const double* bns; int64_t bnsr;
  float *emb, *embM, *embV; int64_t es;
  float *fac, *facM, *facV; int64_t fs;
  float *rm, *rv;
  const RedcliffReplicaHyper* hyp;
  float* ws; int64_t wss;
  double* acc;
  int* conf;
  float *gE, *gF;  // RC_GRAD_ONLY gradient outputs (emb / fac layouts)
  // layout of the embedder-backward partials the final kernel reduces (node-chunk kernel vs GEMM path):
  // dS_i[cc][c'] = sum_s ws.dS[cc*dsCC + s*dsS + i*dsI + c'], s < dsN;  BN affine: ws.dgb[s][2][F], s < dgN;
  // graph-conv weights: dW_i = sum_s ws.dWi[s][n][F][H], s < dwN (p node slices)
  int dsN, dgN, dwN;
  int64_t dsCC, dsS, dsI;
  // matrix-core factor path: y / group-norm partial slots the forward writes (rc_fac_slots)
  int fslots;
  // 1: k_emb_bwd's node blocks leave their per-window-block partial records unreduced and
  // k_emb_combine sums them (no cross-workgroup ticket / fences inside the backward kernel)
  int defer;
  EmbOff eo;
  FacOff fo;
  WsOff wo;
  // replicas this launch processes: grid index i (blockIdx.y / .z) -> replica rc_rep(c, i).
  // rident: all R in order; else the active list of a packed fit whose stopped replicas
  // (early stopping, ...withStateSmoothing.py:1483-1559) drop out of every grid.
  int nrep, rident;
  // debug (REDCLIFF_DEBUG_WAIT_TIMEOUT=1): the merged backward's consumers wait for one more
  // producer than exists, with a short poll bound -- forces the timeout path (tests)
  int wait_dbg;
  uint8_t rmap[RC_MAX_ACTIVE];
  // RcDiv32 multipliers of the dimensions the hot kernels divide by (rc_ctx_magics; RC_MG_*)
  unsigned mg[RC_MG_N];
  // the embedder backward's window blocking, host-computed (each is several integer divisions on
  // the device): rc_emb_wpb(d), rc_emb_nbw(d) and the blocks of this step's B windows
  int ewpb, enbwm, enbw;
  int fzs;  // the embedder forward's fc1 slices per window (slice width mg[RC_MG_CS])
};

__host__ __device__ inline int rc_rep(const StepCtx& c, int i) { return c.rident ? i : (int)c.rmap[i]; }
inline int rc_rep_host(const StepCtx& c, int i) { return rc_rep(c, i); }

// ---------------------------------------------------------------------------------------------
// Workgroup timing (trace builds, -DRC_TRACE): thread 0 of workgroup x < 1024 of replica 0
// stores wall_clock64() (100 MHz) at its start / end into u64 slot kid*2048 + 2x (+1) of the
// trace area at the end of the workspace (scripts/phase_trace.py reads them back).
#define RC_KID_EMB_FWD 0
#define RC_KID_FAC_FWD 1
#define RC_KID_FAC_BWD 2
#define RC_KID_EMB_BWD 3
#define RC_KID_EMB_FINAL 4
#define RC_KID_FAC_MIX 5
#define RC_KID_EMB_WAIT 7  // merged backward: a node workgroup's hand-off wait returned (start slot only)
#ifdef RC_TRACE
#define RC_WG_MARK(wsbase, total, kid, end)                                                        \
  do {                                                                                            \
    if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && blockIdx.x < 1024)               \
      reinterpret_cast<unsigned long long*>((wsbase) + (total) - RC_TRACE_FLOATS)[(kid) * 2048 + 2 * blockIdx.x + (end)] = \
          wall_clock64();                                                                         \
  } while (0)
// phase mark i of workgroup `bx` == 0 of replica 0 (slot 6*2048 + i)
#define RC_PHASE(wsbase, total, bx, i)                                                            \
  do {                                                                                            \
    if (threadIdx.x == 0 && (bx) == 0 && blockIdx.y == 0 && blockIdx.z == 0)                       \
      reinterpret_cast<unsigned long long*>((wsbase) + (total) - RC_TRACE_FLOATS)[6 * 2048 + (i)] = wall_clock64(); \
  } while (0)
#else
#define RC_WG_MARK(wsbase, total, kid, end) \
  do {                                      \
  } while (0)
#define RC_PHASE(wsbase, total, bx, i) \
  do {                                 \
  } while (0)
#endif

// ---------------------------------------------------------------------------------------------
// device helpers

// Producer / consumer hand-off between workgroups of ONE launch (k_bwd_merged), the write-through
// form of cdna_hip_programming.md Guideline 16 (R1): every payload word is stored sc1 (agent-scope
// relaxed atomic store: write-through to the device coherence point, so no release fence and no
// L2 writeback), every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier, and
// one lane counts the workgroup in with an agent-scope atomic.  A consumer's lane 0 polls the
// count relaxed (s_sleep between polls, bounded), and EVERY load of the payload in the consumer is
// an sc1 load (agent-scope relaxed atomic load), so no acquire fence / L1 invalidate is needed --
// only a compiler barrier keeps the loads below the poll.  Producers have lower workgroup ids than
// their consumers and never wait, so they are dispatched first and finish (no co-residency
// assumption); the bounded poll means a missing producer cannot hang the GPU.  A poll that runs
// out is NOT silent: it counts itself into the replica's status word (WsOff.errw, a vector
// atomic), the host reads the words back (redcliff_device_status) and the Python side raises
// instead of using the step's results.
__device__ inline void rc_store_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline float rc_load_sc1(const float* p) {
  return __uint_as_float(
      __hip_atomic_load(reinterpret_cast<unsigned*>(const_cast<float*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// a payload store: sc1 inside the merged launch, plain otherwise (read by a later launch)
__device__ inline void rc_store_payload(float* p, float v, bool sc1) {
  if (sc1)
    rc_store_sc1(p, v);
  else
    *p = v;
}

__device__ inline void rc_publish(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define RC_WAIT_POLLS (1u << 24)      // ~1 s of s_sleep(2) polls
#define RC_WAIT_POLLS_DBG (1u << 12)  // the forced-timeout debug mode

__device__ inline void rc_wait_count(const unsigned* cnt, unsigned target, unsigned* status, unsigned polls) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(const_cast<unsigned*>(cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++spins >= polls) {
        __hip_atomic_fetch_add(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler barrier only: payload loads are sc1
  __syncthreads();
}

// the merged backward's factor-lead counter of replica slice `ws`
__device__ inline unsigned* rc_fac_lead_cnt(const StepCtx& c, float* ws) {
  return reinterpret_cast<unsigned*>(ws + c.wo.ecnt) + c.d.p * ((c.d.H + EMB_HC - 1) / EMB_HC);
}
// k_emb_tail's combine counter of replica slice `ws`
__device__ inline unsigned* rc_tail_cnt(const StepCtx& c, float* ws) { return rc_fac_lead_cnt(c, ws) + 1; }
// a consumer of the merged backward waits for `target` published factor leads of replica slice ws
__device__ inline void rc_wait_leads(const StepCtx& c, float* ws, const unsigned* cnt, unsigned target) {
  rc_wait_count(cnt, target + (c.wait_dbg ? 1u : 0u), reinterpret_cast<unsigned*>(ws + c.wo.errw),
                c.wait_dbg ? RC_WAIT_POLLS_DBG : RC_WAIT_POLLS);
}

__device__ inline float rc_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Division by a block-uniform runtime divisor without the ~40-instruction integer divide:
// q = (n * ceil(2^40 / d)) >> 40, exact for 0 <= n < 2^24 (error term n / 2^40 < 1 / d).
// Workspace y (the factor forward's per-slot prediction partials): [slot][network kj][Bmax],
// network-major so that a network's windows are contiguous for the kernels that write them (one
// network per block) and for the ones that read them (a network's windows per workgroup)
__host__ __device__ inline int64_t rc_y_idx(const RedcliffDims& d, int slot, int kj, int b) {
  return ((int64_t)slot * d.K * d.p + kj) * d.Bmax + b;
}

// XCD-aware order of a grid of nx workgroups x nz slices (replicas): workgroups are dealt
// round-robin over the 8 XCDs in dispatch order (observed, used for speed only), so the dispatch
// index L = x + nx z is remapped such that every workgroup of one slice runs on one XCD (L % 8)
// and that XCD's L2 serves the operands the slice's workgroups share.  A bijection of the grid
// when nz is a multiple of 8 (otherwise the identity): the same workgroups, the same bits.
__device__ inline void rc_xcd_order(int nx, int nz, int& x, int& z) {
  if ((nz & 7) != 0) return;
  const int L = x + nx * z, slot = L >> 3, q = slot / nx;
  x = slot - q * nx;
  z = (L & 7) + 8 * q;
}

// ceil(2^40 / d) for d > 1 (0 for d <= 1): RcDiv's multiplier
__host__ __device__ inline unsigned long long rc_magic40(long long d) {
  return d > 1 ? ((1ull << 40) + (unsigned long long)d - 1) / (unsigned long long)d : 0ull;
}

struct RcDiv {
  unsigned long long m;
  int d;
  // On the device the 64-bit integer division expands to ~150 dependent scalar instructions:
  // with six divisors that is ~2 us of a kernel prologue (k_emb_bwd's node workgroups, phase trace).
  // The hot kernels take the multipliers the host computed (StepCtx::mg, RcDiv(d, m)).
  __device__ inline explicit RcDiv(int dd) : m(rc_magic40(dd)), d(dd) {}
  __device__ inline int div(int n) const {
    return d == 1 ? n : (int)(((unsigned long long)(unsigned)n * m) >> 40);
  }
  __device__ inline int mod(int n) const { return n - div(n) * d; }
};

// ceil(2^32 / d) for d > 1 (0 for d <= 1): RcDiv32's multiplier
__host__ __device__ inline unsigned rc_magic32(long long d) {
  return d > 1 ? (unsigned)(((1ull << 32) + (unsigned long long)d - 1) / (unsigned long long)d) : 0u;
}
// n / d as one v_mul_hi_u32 with the multiplier the host computed (StepCtx::mg): exact for
// 0 <= n, n * d < 2^32 (every use: indices < 2^20, divisors < 2^14).  One 32-bit register for the
// multiplier where RcDiv's 64-bit one took two: the hot kernels run short of scalar registers
// (k_emb_bwd spilled ~1,600 of them to vector lanes), and the 64-bit product was ~5 instructions.
struct RcDiv32 {
  unsigned m;
  int d;
  __device__ inline RcDiv32(int dd, unsigned mm) : m(mm), d(dd) {}
  __device__ inline explicit RcDiv32(int dd) : m(rc_magic32(dd)), d(dd) {}  // (fallback: a device division)
  __device__ inline int div(int n) const { return d == 1 ? n : (int)__umulhi((unsigned)n, m); }
  __device__ inline int mod(int n) const { return n - div(n) * d; }
};

// Global -> LDS staging with U independent loads in flight per thread: the loads of U
// elements are issued before any of them is consumed, so a staging loop costs ~N/(U*256)
// memory latencies instead of N/256.  ld(e) returns element e, st(e, v) consumes it.
// NT: the workgroup's threads (RC_BLOCK unless the kernel launches narrower workgroups).
template <int U, int NT = RC_BLOCK, class Ld, class St>
__device__ inline void rc_stage(int N, Ld ld, St st) {
  for (int base = threadIdx.x; base < N; base += U * NT) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * NT;
      v[u] = e < N ? ld(e) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * NT;
      if (e < N) st(e, v[u]);
    }
  }
}

// Several staging segments with all their loads in flight together: round r issues the
// loads of elements [r*U*256, (r+1)*U*256) of EVERY segment, then stores them.  A segment
// is rc_seg<U>(N, ld, st); U is its loads per thread per round.
template <int U, class Ld, class St>
struct RcSeg {
  int N;
  Ld ld;
  St st;
  float v[U];
  __device__ inline bool active(int r) const { return r * U * RC_BLOCK < N; }
  __device__ inline void load(int r) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = r * U * RC_BLOCK + u * RC_BLOCK + (int)threadIdx.x;
      v[u] = e < N ? ld(e) : 0.f;
    }
  }
  __device__ inline void store(int r) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = r * U * RC_BLOCK + u * RC_BLOCK + (int)threadIdx.x;
      if (e < N) st(e, v[u]);
    }
  }
};
template <int U, class Ld, class St>
__device__ inline RcSeg<U, Ld, St> rc_seg(int N, Ld ld, St st) {
  return RcSeg<U, Ld, St>{N, ld, st, {}};
}
template <class... S>
__device__ inline void rc_stage_all(S&&... s) {
  for (int r = 0; (s.active(r) || ...); ++r) {
    (s.load(r), ...);
    (s.store(r), ...);
  }
}

// Kernels of the embedder chain (the critical path when the factor chain runs concurrently on
// a second stream) raise their waves' issue priority over the co-resident factor waves.
__device__ inline void rc_critical_priority() { __builtin_amdgcn_s_setprio(2); }

// fp32 matrix cores: v_mfma_f32_32x32x2f32 accumulator, and the row of accumulator register
// `reg` of lane `lane` in its 32x32 tile (columns = lane & 31).
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ inline int mf_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

// Block-wide sum; every thread gets the result.  `red` must hold >= RC_BLOCK/64 floats.
__device__ inline float rc_block_sum(float v, float* red) {
  v = rc_wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  __syncthreads();
  return s;
}

__device__ inline double rc_block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  __syncthreads();
  return s;
}

__device__ inline float rc_sign(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }
__device__ inline float rc_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// Bias-correction scalars of step t, computed the way torch's Python side does (doubles),
// then rounded to the fp32 values the element-wise kernels apply.
struct RcAdamScalars {
  float neg_step, bc2s, eps, wd, b2, omb1, omb2;
};
__device__ inline RcAdamScalars rc_adam_scalars(const RedcliffAdamHyper& h, int t) {
  RcAdamScalars s;
  t += h.t_offset;  // per-replica step number of a packed launch (0 unless the pack's schedules differ)
  const double bc1 = 1.0 - pow(h.beta1, (double)t);
  const double bc2 = 1.0 - pow(h.beta2, (double)t);
  s.neg_step = (float)(-(h.lr / bc1));
  s.bc2s = (float)sqrt(bc2);
  s.eps = h.eps;
  s.wd = h.weight_decay;
  s.b2 = h.beta2_f;
  s.omb1 = h.one_minus_beta1_f;
  s.omb2 = h.one_minus_beta2_f;
  return s;
}

// torch.optim.Adam (_single_tensor_adam, coupled L2 weight decay) for one element:
//   g += wd*p; m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, -lr/bc1)
// Every multiply-add is an explicit fmaf: left to -ffp-contract=fast, the compiler fuses (or,
// when it packs two updates into v_pk_mul / v_pk_add, does not fuse) per call site, and the same
// parameter stepped by two different kernels would then differ in the last ulp.
__device__ inline void rc_adam(float& p, float& m, float& v, float g, const RcAdamScalars& s) {
  if (s.wd != 0.f) g = __builtin_fmaf(p, s.wd, g);
  m = __builtin_fmaf(s.omb1, g - m, m);
  v = __builtin_fmaf(s.omb2 * g, g, v * s.b2);
  const float denom = sqrtf(v) / s.bc2s + s.eps;
  p = __builtin_fmaf(s.neg_step, m / denom, p);
}

// Apply Adam to element idx of a group, or (data-parallel shard, RC_GRAD_ONLY) store its
// gradient for the all-reduce; weight decay is added by Adam, once, after the reduction.
__device__ inline void rc_update(const StepCtx& c, float* P, float* M, float* V, float* G, int64_t idx, float g,
                                 const RcAdamScalars& s) {
  if (c.flags & RC_GRAD_ONLY) {
    G[idx] = g;
    return;
  }
  float pp = P[idx], mm = M[idx], vv = V[idx];
  rc_adam(pp, mm, vv, g, s);
  P[idx] = pp; M[idx] = mm; V[idx] = vv;
}

// dL/d(raw embedder output w[b][k]) from the factor side's dL/dw (gw, channel partials summed by
// the caller) and the batch_update loss terms on the embedder output (...withStateSmoothing.py:
// 633-666): the factor-score MSE against label y on the first nsup columns (mean over B_global *
// nsup), the fw-L1 sign, both through the optional sigmoid restriction (:383-386).
__device__ inline float rc_emb_draw(const StepCtx& c, int r, int k, float raw, float gw, float y) {
  const RedcliffDims& d = c.d;
  const int K = d.K, nsup = d.nsup;
  const RedcliffReplicaHyper& hy = c.hyp[r];
  const bool sig = d.use_sigmoid;
  const float ecc = d.sigmoid_ecc;
  const int ncol = nsup > 0 ? nsup : K;
  const float weff = sig ? rc_sigmoid(ecc * raw) : raw;
  float graw = sig ? gw * ecc * weff * (1.f - weff) : gw;
  if (k < ncol) {
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

// Shared host-side helpers (defined in rc_capi.hip).
void rc_set_error(const char* fmt, ...);
int rc_check(hipError_t e, const char* what);

// Dynamic LDS above 64 KiB (up to the CU's 160 KiB) must be opted into per kernel.
template <class Kern>
inline int rc_lds_optin(Kern k, size_t bytes, const char* what) {
  if (bytes <= RC_LDS_LIMIT_FLOATS * sizeof(float)) return 0;
  return rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bytes), what);
}

// Launchers implemented in the kernel translation units.
// embedder forward and / or vector-path factor forward in one launch (rc_forward.hip)
// stop (optional): an event the launch itself completes (hipExtLaunchKernel), so a second stream can
// wait for this kernel without an event-record packet between it and the next kernel of `s`
int rc_launch_forward(const StepCtx& c, hipStream_t s, bool with_emb, bool with_fac, hipEvent_t stop = nullptr);
// fills StepCtx::mg from c.d and c.B (every StepCtx builder calls it last)
void rc_ctx_magics(StepCtx& c);
int rc_launch_fac_fwd(const StepCtx& c, hipStream_t s);
// factor backward roles (rc_fac_bwd.h fac_bwd_wg): one launch, or the split-lead pair
enum { RC_FB_ALL = 0, RC_FB_RECORDS = 1, RC_FB_UPDATE = 2 };
int rc_launch_fac_bwd(const StepCtx& c, hipStream_t s, int role, hipEvent_t stop = nullptr);
int rc_fac_bwd_grid(const StepCtx& c);  // workgroups per replica of the update launch

// compute units of the current device (cached per host thread)
inline int rc_cu_count() {
  static thread_local int dev_c = -1, n_c = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (dev != dev_c) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    dev_c = dev;
    n_c = n;
  }
  return n_c;
}
// MFMA path of the factor networks (large p*L): window transpose, GEMM forward, per-network
// mixing / penalties / small-parameter updates, GEMM dW0 + Adam.
bool rc_fac_use_mfma(const RedcliffDims& d);
int rc_launch_fac_fwd_mfma(const StepCtx& c, hipStream_t s);
int rc_launch_fac_mix(const StepCtx& c, hipStream_t s);
int rc_launch_cos_values(const StepCtx& c, hipStream_t s);  // per-window cos-sim penalty values (rc_embed.hip)   // mixing, loss terms, output layer (MFMA path)
int rc_launch_fac_dw0(const StepCtx& c, hipStream_t s);   // dW0 on the matrix cores + Adam (MFMA path)
// GEMM-shaped embedder for large p*F (rc_embed_gemm.hip)
bool rc_emb_use_gemm(const RedcliffDims& d);
int rc_fac_slots(const RedcliffDims& d);  // rc_factor_mfma.hip
void rc_emb_partial_layout(StepCtx& c, bool gemm);
int rc_launch_emb_fwd_gemm(const StepCtx& c, hipStream_t s);
int rc_launch_emb_bwd_gemm(const StepCtx& c, hipStream_t s);
int rc_launch_emb_bwd(const StepCtx& c, hipStream_t s, bool node_wgs);
int rc_launch_emb_final(const StepCtx& c, hipStream_t s);
int rc_emb_tail_grid(const StepCtx& c);
int rc_launch_emb_tail(const StepCtx& c, hipStream_t s);
int rc_launch_emb_combine(const StepCtx& c, hipStream_t s);
int rc_launch_bwd_merged(const StepCtx& c, hipStream_t s);  // factor + embedder backward, one launch
int rc_bwd_merged_grid(const StepCtx& c);                    // its grid, 0 when not worth it  // window-block partials (c.defer)
int rc_launch_dp_update(const StepCtx& c, int64_t nE, int64_t nF, hipStream_t s);
int rc_launch_supports(const RedcliffDims& d, const float* emb, int64_t es, float* ws, int64_t wss, EmbOff eo,
                       WsOff wo, hipStream_t s);
int rc_launch_bn_stats(const RedcliffDims& d, const float* X, int64_t xr, int64_t N, int B, double* st, int64_t str,
                       hipStream_t s);
