// rc_gemm.h -- fp32 GEMM core shared by the generic path (rc_generic.hip) and the GEMM-shaped
// embedder for large p*F (rc_embed_gemm.hip).
//
//   C[z] = alpha * sum_{kb} op(A[z] + kb*rA) op(B[z] + kb*rB) + beta * C[z]   (then an epilogue)
//
// row-major, op(X) = X or X^T; z = blockIdx.z (batch / split-K slice); the contraction index
// k in [0, K) is split as k = kb * Kblk + kr, which lets one launch sum products over many
// small matrices (e.g. over the windows of a batch) without materialising per-window partials.
// K staged through LDS in steps of 16.  Two cores: k_rc_gemm_mfma (fp32 matrix cores, the
// default) and k_rc_gemm (vector-ALU fmaf chains, REDCLIFF_GEMM_CORE=valu); each is
// deterministic and independent of the tile size it is launched with.
#pragma once
#include <cstdlib>

#include "rc_common.h"

#define RC_GEMM_T 64
#ifndef RC_GEMM_K
#define RC_GEMM_K 16  // K step staged through LDS (a power of two)
#endif
static_assert((RC_GEMM_K & (RC_GEMM_K - 1)) == 0 && RC_GEMM_K >= 16, "RC_GEMM_K: power of two >= 16");

enum { RC_EPI_NONE = 0, RC_EPI_RELU = 1, RC_EPI_MASK = 2 };  // MASK: times (aux > 0)

struct RcGemm {
  int ta, tb, M, N, K;
  const float* A; int64_t lda, sA;
  const float* B; int64_t ldb, sB;
  float* C; int64_t ldc, sC;
  float alpha, beta;
  int Kblk; int64_t rA, rB;
  int epi;
  const float* aux; int64_t ldaux, sAux;
  // replica axis (packed grid-search fits): grid z = nrep x batch, z = i * batch + zb; operand
  // bases advance by replica r = rmap[i] (or i when rident) times the r-strides.  nrep = 1,
  // strides 0: a plain batched product.
  int batch, nrep, rident;
  int xcd;  // 1: XCD-aware tile order (rc_gemm_tile)
  int64_t qA, qB, qC, qAux;
  int extA, extB;  // wave core: elements of A / B one slice spans (set by rc_gemm_launch)
  uint8_t rmap[RC_MAX_ACTIVE];
};

inline RcGemm rc_gemm_args(int ta, int tb, int M, int N, int K, const float* A, int64_t lda, int64_t sA,
                           const float* B, int64_t ldb, int64_t sB, float* C, int64_t ldc, int64_t sC) {
  RcGemm g;
  g.ta = ta; g.tb = tb; g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = lda; g.sA = sA;
  g.B = B; g.ldb = ldb; g.sB = sB;
  g.C = C; g.ldc = ldc; g.sC = sC;
  g.alpha = 1.f; g.beta = 0.f;
  g.Kblk = K > 0 ? K : 1; g.rA = 0; g.rB = 0;
  g.epi = RC_EPI_NONE; g.aux = nullptr; g.ldaux = 0; g.sAux = 0;
  g.batch = 1; g.nrep = 1; g.rident = 1; g.xcd = 0; g.qA = g.qB = g.qC = g.qAux = 0;
  return g;
}

// Replica axis of a step's products: c.nrep replicas (c's active list), operand r-strides.
inline void rc_gemm_reps(RcGemm& g, const StepCtx& c, int64_t qA, int64_t qB, int64_t qC, int64_t qAux = 0) {
  g.nrep = c.nrep;
  g.rident = c.rident;
  for (int i = 0; i < c.nrep && i < RC_MAX_ACTIVE; ++i) g.rmap[i] = c.rmap[i];
  g.qA = qA; g.qB = qB; g.qC = qC; g.qAux = qAux;
}

// The output tile (x, y) and grid slice z of this workgroup.  XCD-aware order (g.xcd, slice count
// a multiple of 8): workgroups are dealt round-robin over the 8 XCDs in dispatch order (observed,
// used for speed only), so the dispatch index L = x + nx (y + ny z) is remapped such that every
// tile of one slice -- which share their A rows and B columns -- runs on one XCD (L % 8) and
// its L2 fetches those operands once, not once per XCD.  A bijection of the grid: the same
// tiles are computed, with the same bits.
struct RcTile {
  int x, y, z;
};
// rc_gemm_tile_in: the same for the workgroup at linear index L of an nx x ny x nz grid (x fastest,
// as the hardware linearises dispatch), when several products share one launch (rc_gemm_launch_set).
__device__ inline RcTile rc_gemm_tile_in(const RcGemm& g, int L, int nx, int ny, int nz) {
  const int T = nx * ny;
  if (!g.xcd || (nz & 7) != 0) {
    const int z = L / T, t = L - z * T, y = t / nx;
    return RcTile{t - y * nx, y, z};
  }
  const int slot = L >> 3, zq = slot / T, t = slot - zq * T, ty = t / nx;
  return RcTile{t - ty * nx, ty, (L & 7) + 8 * zq};
}
__device__ inline RcTile rc_gemm_tile(const RcGemm& g) {
  const int nx = gridDim.x, ny = gridDim.y, nz = gridDim.z;
  if (!g.xcd || (nz & 7) != 0) return RcTile{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  return rc_gemm_tile_in(g, (int)blockIdx.x + nx * ((int)blockIdx.y + ny * (int)blockIdx.z), nx, ny, nz);
}

// The replica of grid slice z and the slice inside it: (replica, zb).
struct RcGemmZ {
  int64_t r;
  int zb;
};
__device__ inline RcGemmZ rc_gemm_z(const RcGemm& g, int z) {
  // one replica in the launch: replica 0, or the active list's only entry (a packed fit whose other
  // replicas have stopped)
  if (g.nrep == 1) return RcGemmZ{g.rident ? 0 : (int)g.rmap[0], z};
  const int i = z / g.batch, zb = z - i * g.batch;
  return RcGemmZ{g.rident ? i : (int)g.rmap[i], zb};
}

// TT x TT output tile per 256-thread workgroup (TT = 64: 4x4 outputs per thread; TT = 32:
// 2x2, four times the workgroups for short / skinny products).  Each output is the same
// in-order fmaf chain over k whatever the tile, so both variants give identical bits.
template <int TT>
__global__ __launch_bounds__(RC_BLOCK) static void k_rc_gemm(RcGemm g) {
  constexpr int TP = TT / 16;           // outputs per thread along each tile dimension
  constexpr int NL = RC_GEMM_K * TT / RC_BLOCK;  // operand elements per thread per K step
  rc_critical_priority();
  const RcTile tl = rc_gemm_tile(g);
  const RcGemmZ zz = rc_gemm_z(g, tl.z);
  const int bz = zz.zb;
  const float* A = g.A + bz * g.sA + zz.r * g.qA;
  const float* B = g.B + bz * g.sB + zz.r * g.qB;
  float* C = g.C + bz * g.sC + zz.r * g.qC;
  const float* aux = g.aux ? g.aux + zz.r * g.qAux : nullptr;
  const int n0 = tl.x * TT, m0 = tl.y * TT;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const RcDiv dkb(g.Kblk);
  __shared__ float As[RC_GEMM_K][TT + 4];  // As[k][m]
  __shared__ float Bs[RC_GEMM_K][TT + 4];  // Bs[k][n]
  float acc[TP][TP];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = 0.f;
  // the next K step's operands are loaded into registers while the current step multiplies
  float av[NL], bv[NL];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int e = tid + r * RC_BLOCK;  // RC_GEMM_K x TT elements of each tile
      int kk, mm;
      if (g.ta) { kk = e / TT; mm = e % TT; } else { mm = e / RC_GEMM_K; kk = e % RC_GEMM_K; }
      const int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < g.M && gk < g.K) {
        const int kb = dkb.div(gk), kr = gk - kb * g.Kblk;
        const float* Ab = A + kb * g.rA;
        v = g.ta ? Ab[(int64_t)kr * g.lda + gm] : Ab[(int64_t)gm * g.lda + kr];
      }
      av[r] = v;
      int kb2, nb;
      if (g.tb) { nb = e / RC_GEMM_K; kb2 = e % RC_GEMM_K; } else { kb2 = e / TT; nb = e % TT; }
      const int gn = n0 + nb, gk2 = k0 + kb2;
      float w = 0.f;
      if (gn < g.N && gk2 < g.K) {
        const int kb = dkb.div(gk2), kr = gk2 - kb * g.Kblk;
        const float* Bb = B + kb * g.rB;
        w = g.tb ? Bb[(int64_t)gn * g.ldb + kr] : Bb[(int64_t)kr * g.ldb + gn];
      }
      bv[r] = w;
    }
  };
  if (g.K > 0) load(0);
  for (int k0 = 0; k0 < g.K; k0 += RC_GEMM_K) {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int e = tid + r * RC_BLOCK;
      if (g.ta) As[e / TT][e % TT] = av[r]; else As[e % RC_GEMM_K][e / RC_GEMM_K] = av[r];
      if (g.tb) Bs[e % RC_GEMM_K][e / RC_GEMM_K] = bv[r]; else Bs[e / TT][e % TT] = bv[r];
    }
    __syncthreads();
    if (k0 + RC_GEMM_K < g.K) load(k0 + RC_GEMM_K);
#pragma unroll
    for (int kk = 0; kk < RC_GEMM_K; ++kk) {
      float a[TP], b[TP];
#pragma unroll
      for (int i = 0; i < TP; ++i) a[i] = As[kk][ty * TP + i];
#pragma unroll
      for (int j = 0; j < TP; ++j) b[j] = Bs[kk][tx * TP + j];
#pragma unroll
      for (int i = 0; i < TP; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    const int gm = m0 + ty * TP + i;
    if (gm >= g.M) continue;
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int gn = n0 + tx * TP + j;
      if (gn >= g.N) continue;
      float* cp = C + (int64_t)gm * g.ldc + gn;
      float v = g.beta == 0.f ? g.alpha * acc[i][j] : g.alpha * acc[i][j] + g.beta * *cp;
      if (g.epi == RC_EPI_RELU) v = fmaxf(v, 0.f);
      else if (g.epi == RC_EPI_MASK) v = aux[bz * g.sAux + (int64_t)gm * g.ldaux + gn] > 0.f ? v : 0.f;
      *cp = v;
    }
  }
}

// Epilogue of the matrix-core kernels: this lane's NR outputs of column gn (rows row(reg)),
// C = alpha acc + beta C, then ReLU or the (aux > 0) mask.  The C / aux operands of all NR rows are
// requested together (rows past M clamped, not stored) -- one branch per row around each load made
// the compiler wait for every load in turn (16 round trips per wave for dZ's mask).
template <int NR, typename RowF>
__device__ inline void rc_gemm_store(const RcGemm& g, float* C, const float* aux, int bz, int gn, const float (&av)[NR],
                                     RowF row) {
  // one operand array: the mask's aux rows, else C's rows when beta != 0 (both at once -- no caller
  // does that -- reads C per row)
  const bool mask = g.epi == RC_EPI_MASK, bc = g.beta != 0.f;
  float xv[NR];
#pragma unroll
  for (int reg = 0; reg < NR; ++reg) xv[reg] = 0.f;
  if (mask || bc) {
    const float* src = mask ? aux + bz * g.sAux : C;
    const int64_t ld = mask ? g.ldaux : g.ldc;
#pragma unroll
    for (int reg = 0; reg < NR; ++reg) xv[reg] = src[(int64_t)min(row(reg), g.M - 1) * ld + gn];
  }
#pragma unroll
  for (int reg = 0; reg < NR; ++reg) {
    const int gm = row(reg);
    if (gm >= g.M) continue;
    const float cv = !bc ? 0.f : mask ? C[(int64_t)gm * g.ldc + gn] : xv[reg];
    float v = !bc ? g.alpha * av[reg] : g.alpha * av[reg] + g.beta * cv;
    if (g.epi == RC_EPI_RELU) v = fmaxf(v, 0.f);
    else if (mask) v = xv[reg] > 0.f ? v : 0.f;
    C[(int64_t)gm * g.ldc + gn] = v;
  }
}

// Matrix-core variant: the same tiles, staging and workgroup shape as k_rc_gemm, the
// products on the fp32 matrix cores.  TT = 64: each of the 4 waves owns a 32x32 quarter
// (v_mfma_f32_32x32x2f32); TT = 32: a 16x16 quarter (v_mfma_f32_16x16x4f32).  The fp32 MFMA
// forms are exact fmaf chains over k in order (MI355X_MICROARCH.md, "F32 (f32 in)"), so an
// output has the same bits as k_rc_gemm's in-order fmaf chain, whatever the tile or core
// (tests/test_gpu_generic.py::test_gemm_cores_bitwise).
template <int TT>
__device__ __forceinline__ void rc_gemm_mfma_body(const RcGemm& g, const RcTile tl) {
  constexpr int NL = RC_GEMM_K * TT / RC_BLOCK;  // operand elements per thread per K step
  constexpr int QT = TT / 2;                      // quarter tile per wave
  const RcGemmZ zz = rc_gemm_z(g, tl.z);
  const int bz = zz.zb;
  const float* A = g.A + bz * g.sA + zz.r * g.qA;
  const float* B = g.B + bz * g.sB + zz.r * g.qB;
  float* C = g.C + bz * g.sC + zz.r * g.qC;
  const float* aux = g.aux ? g.aux + zz.r * g.qAux : nullptr;
  const int n0 = tl.x * TT, m0 = tl.y * TT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = QT * (wv >> 1), wn = QT * (wv & 1);
  const RcDiv dkb(g.Kblk);
  __shared__ float As[RC_GEMM_K][TT + 4];  // As[k][m]
  __shared__ float Bs[RC_GEMM_K][TT + 4];  // Bs[k][n]
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x16 acc32;
  f32x4 acc16;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc32[i] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc16[i] = 0.f;
  float av[NL], bv[NL];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int e = tid + r * RC_BLOCK;  // RC_GEMM_K x TT elements of each tile
      int kk, mm;
      if (g.ta) { kk = e / TT; mm = e % TT; } else { mm = e / RC_GEMM_K; kk = e % RC_GEMM_K; }
      const int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < g.M && gk < g.K) {
        const int kb = dkb.div(gk), kr = gk - kb * g.Kblk;
        const float* Ab = A + kb * g.rA;
        v = g.ta ? Ab[(int64_t)kr * g.lda + gm] : Ab[(int64_t)gm * g.lda + kr];
      }
      av[r] = v;
      int kb2, nb;
      if (g.tb) { nb = e / RC_GEMM_K; kb2 = e % RC_GEMM_K; } else { kb2 = e / TT; nb = e % TT; }
      const int gn = n0 + nb, gk2 = k0 + kb2;
      float w = 0.f;
      if (gn < g.N && gk2 < g.K) {
        const int kb = dkb.div(gk2), kr = gk2 - kb * g.Kblk;
        const float* Bb = B + kb * g.rB;
        w = g.tb ? Bb[(int64_t)gn * g.ldb + kr] : Bb[(int64_t)kr * g.ldb + gn];
      }
      bv[r] = w;
    }
  };
  if (g.K > 0) load(0);
  for (int k0 = 0; k0 < g.K; k0 += RC_GEMM_K) {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int e = tid + r * RC_BLOCK;
      if (g.ta) As[e / TT][e % TT] = av[r]; else As[e % RC_GEMM_K][e / RC_GEMM_K] = av[r];
      if (g.tb) Bs[e % RC_GEMM_K][e / RC_GEMM_K] = bv[r]; else Bs[e / TT][e % TT] = bv[r];
    }
    __syncthreads();
    if (k0 + RC_GEMM_K < g.K) load(k0 + RC_GEMM_K);
    if constexpr (TT == 64) {
      const int l31 = lane & 31, kh = lane >> 5;
#pragma unroll
      for (int kk = 0; kk < RC_GEMM_K; kk += 2)
        acc32 = __builtin_amdgcn_mfma_f32_32x32x2f32(As[kk + kh][wm + l31], Bs[kk + kh][wn + l31], acc32, 0, 0, 0);
    } else {
      const int l15 = lane & 15, kq = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < RC_GEMM_K; kk += 4)
        acc16 = __builtin_amdgcn_mfma_f32_16x16x4f32(As[kk + kq][wm + l15], Bs[kk + kq][wn + l15], acc16, 0, 0, 0);
    }
    __syncthreads();
  }
  constexpr int NR = TT == 64 ? 16 : 4;
  const int gn = n0 + wn + (TT == 64 ? (lane & 31) : (lane & 15));
  if (gn >= g.N) return;
  float accv[NR];
#pragma unroll
  for (int reg = 0; reg < NR; ++reg) accv[reg] = TT == 64 ? acc32[reg] : acc16[reg];
  rc_gemm_store<NR>(g, C, aux, bz, gn, accv, [&](int reg) { return m0 + wm + (TT == 64 ? mf_row(reg, lane) : 4 * (lane >> 4) + reg); });
}

template <int TT>
__global__ __launch_bounds__(RC_BLOCK) static void k_rc_gemm_mfma(RcGemm g) {
  rc_critical_priority();
  rc_gemm_mfma_body<TT>(g, rc_gemm_tile(g));
}

// Up to three INDEPENDENT products in one launch (the same LDS-tiled matrix-core body, TT x TT tiles):
// product i owns the linear workgroups [start[i], start[i + 1]), its grid nx x ny x nz laid out from
// start[i] (a multiple of 8, so a workgroup's XCD is its product-local index mod 8 and the XCD-aware
// tile order holds per product; the padding workgroups exit).  Every output is computed by the same
// body with the same k order as in its own launch: the same bits.  A chain of short single-replica
// products (the GEMM-shaped embedder's backward at C5: dfc1W with dZ, dW with dT) is bound by one
// workgroup's chain of operand round trips per launch, not by the chip; products that do not depend
// on each other then share that latency instead of paying it one after the other.
#define RC_GEMM_SET_MAX 3
struct RcGemmSet {
  RcGemm g[RC_GEMM_SET_MAX];
  int nx[RC_GEMM_SET_MAX], ny[RC_GEMM_SET_MAX], nz[RC_GEMM_SET_MAX];
  int start[RC_GEMM_SET_MAX + 1];
  int n;
};
template <int TT>
__global__ __launch_bounds__(RC_BLOCK) static void k_rc_gemm_mfma_set(RcGemmSet s) {
  rc_critical_priority();
  const int bx = blockIdx.x;
  // (no dynamic index into the kernel-argument struct: each product's branch reads its own fields)
#define RC_SET_CASE(i)                                                                                 \
  if (i < s.n && bx >= s.start[i] && bx < s.start[i + 1]) {                                            \
    const int L = bx - s.start[i];                                                                     \
    if (L >= s.nx[i] * s.ny[i] * s.nz[i]) return;                                                      \
    rc_gemm_mfma_body<TT>(s.g[i], rc_gemm_tile_in(s.g[i], L, s.nx[i], s.ny[i], s.nz[i]));              \
    return;                                                                                            \
  }
  RC_SET_CASE(0)
  RC_SET_CASE(1)
  RC_SET_CASE(2)
#undef RC_SET_CASE
}

// Wave core: one 64-lane workgroup per 32x32 output tile, no workgroup-wide barriers, so every
// wave runs on its own and a SIMD holds several to cover the loads' latency (the packed grid's
// embedder products are 0.4 - 0.6 GFLOP over 128 replicas with K = 30 - 300: short chains of
// dependent loads, not arithmetic).  v_mfma_f32_32x32x2f32 wants 32 rows of A / columns of B across
// the lanes: an operand contiguous along m (A^T) or n (B) is loaded straight into the operand
// registers (coalesced); one contiguous along k (LA: A, LB: B^T) is loaded 16 k x 4 rows per
// instruction (coalesced) and transposed through the wave's own LDS tile.  16 k per chunk, the next
// chunk's loads in flight while the current one multiplies.  The k order and the zero padding past K
// are k_rc_gemm_mfma<64>'s, so an output has the same bits.
template <bool LA, bool LB>
__device__ __forceinline__ void rc_gemm_wave_body(const RcGemm& g, const RcTile tl) {
  const RcGemmZ zz = rc_gemm_z(g, tl.z);
  const int bz = zz.zb;
  const float* A = g.A + bz * g.sA + zz.r * g.qA;
  const float* B = g.B + bz * g.sB + zz.r * g.qB;
  float* C = g.C + bz * g.sC + zz.r * g.qC;
  const float* aux = g.aux ? g.aux + zz.r * g.qAux : nullptr;
  const int lane = threadIdx.x, l31 = lane & 31, kh = lane >> 5, k16 = lane & 15, r4 = lane >> 4;
  const int n0 = tl.x * 32, m0 = tl.y * 32;
  // buffer loads with 32-bit offsets (the launcher checks every operand's extent fits); k >= K reads
  // past the resource's end, which returns 0 -- the zero padding, without a branch.  Rows / columns
  // past M / N are clamped into the matrix: they only feed outputs that are not stored.
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), (short)0, g.extA * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), (short)0, g.extB * 4, 0x00020000);
  const int lda = (int)g.lda, ldb = (int)g.ldb;
  const bool split = g.Kblk < g.K;
  const RcDiv dkb(split ? g.Kblk : 1);
  constexpr int OOB = 0x7ffffff0;
  __shared__ float As[LA ? 16 : 1][33], Bs[LB ? 16 : 1][33];
  auto load = [&](int k0, float* a_, float* b_) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ka = LA ? k0 + k16 : k0 + 2 * j + kh, kb_ = LB ? k0 + k16 : k0 + 2 * j + kh;
      const int am = min(m0 + (LA ? r4 + 4 * j : l31), g.M - 1), bn = min(n0 + (LB ? r4 + 4 * j : l31), g.N - 1);
      int qa = 0, ra_ = ka, qb = 0, rb_ = kb_;
      if (split) {
        qa = dkb.div(ka); ra_ = ka - qa * g.Kblk;
        qb = dkb.div(kb_); rb_ = kb_ - qb * g.Kblk;
      }
      const int oa = ka < g.K ? 4 * (qa * (int)g.rA + (g.ta ? ra_ * lda + am : am * lda + ra_)) : OOB;
      const int ob = kb_ < g.K ? 4 * (qb * (int)g.rB + (g.tb ? bn * ldb + rb_ : rb_ * ldb + bn)) : OOB;
      a_[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, oa, 0, 0));
      b_[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, ob, 0, 0));
    }
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  auto mult = [&](const float* a_, const float* b_) {
    if constexpr (LA || LB) {
      __syncthreads();  // one wave: orders the previous chunk's operand reads before these writes
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (LA) As[k16][r4 + 4 * j] = a_[j];
        if constexpr (LB) Bs[k16][r4 + 4 * j] = b_[j];
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float av = LA ? As[LA ? 2 * j + kh : 0][l31] : a_[j];
      const float bv = LB ? Bs[LB ? 2 * j + kh : 0][l31] : b_[j];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
  };
  float a0[8], b0[8], a1[8], b1[8];
  if (g.K > 0) load(0, a0, b0);
  for (int k0 = 0; k0 < g.K; k0 += 32) {
    if (k0 + 16 < g.K) load(k0 + 16, a1, b1);
    mult(a0, b0);
    if (k0 + 16 >= g.K) break;
    if (k0 + 32 < g.K) load(k0 + 32, a0, b0);
    mult(a1, b1);
  }
  const int gn = n0 + l31;
  if (gn >= g.N) return;
  float accv[16];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) accv[reg] = acc[reg];
  rc_gemm_store<16>(g, C, aux, bz, gn, accv, [&](int reg) { return m0 + mf_row(reg, lane); });
}

template <bool LA, bool LB>
__global__ __launch_bounds__(64, 5) static void k_rc_gemm_wave(RcGemm g) {
  rc_critical_priority();
  rc_gemm_wave_body<LA, LB>(g, rc_gemm_tile(g));
}

// Two independent products on the wave core in one launch (packed grids: dfc1W with dZ, dW with dT):
// the layout of k_rc_gemm_mfma_set (product i's 32 x 32 tiles from start[i], a multiple of 8), each
// product with its own operand-staging form (LA / LB), the same body and bits as its own launch.
template <bool LA0, bool LB0, bool LA1, bool LB1>
__global__ __launch_bounds__(64, 5) static void k_rc_gemm_wave_pair(RcGemmSet s) {
  rc_critical_priority();
  const int bx = blockIdx.x;
  if (bx < s.start[1]) {
    if (bx >= s.nx[0] * s.ny[0] * s.nz[0]) return;
    rc_gemm_wave_body<LA0, LB0>(s.g[0], rc_gemm_tile_in(s.g[0], bx, s.nx[0], s.ny[0], s.nz[0]));
  } else {
    const int L = bx - s.start[1];
    if (L >= s.nx[1] * s.ny[1] * s.nz[1]) return;
    rc_gemm_wave_body<LA1, LB1>(s.g[1], rc_gemm_tile_in(s.g[1], L, s.nx[1], s.ny[1], s.nz[1]));
  }
}
typedef void (*RcWavePairKern)(RcGemmSet);
template <int I>
struct RcWavePairTab {
  static void fill(RcWavePairKern* t) {
    t[I] = k_rc_gemm_wave_pair<(I & 1) != 0, (I & 2) != 0, (I & 4) != 0, (I & 8) != 0>;
    RcWavePairTab<I - 1>::fill(t);
  }
};
template <>
struct RcWavePairTab<-1> {
  static void fill(RcWavePairKern*) {}
};

// Whether rc_gemm_launch runs a product on the LDS-tiled matrix-core workgroups (k_rc_gemm_mfma) --
// the products rc_gemm_launch_set can group -- rather than the wave or vector-ALU cores.
inline bool rc_gemm_lds_core(const RcGemm& g0) {
  const char* core = getenv("REDCLIFF_GEMM_CORE");
  if (core != nullptr) return core[0] == 'm';
  return g0.nrep <= 1;
}

inline int rc_gemm_launch(const RcGemm& g0, int batch, hipStream_t s, const char* what);

// Independent products gs[0 .. n) (each with its batch count) in ONE launch of k_rc_gemm_mfma_set
// when all of them run on the LDS-tiled matrix-core workgroups (single-replica steps); otherwise, or
// with REDCLIFF_GEMM_SET=0, one rc_gemm_launch each, in order.  The same bits either way.
inline int rc_gemm_launch_set(const RcGemm* gs, const int* batches, int n, hipStream_t s, const char* what) {
  const char* sv = getenv("REDCLIFF_GEMM_SET");  // read per call: the tests switch it in-process
  const bool on = !(sv && sv[0] == '0');
  bool ok = on && n > 1 && n <= RC_GEMM_SET_MAX;
  for (int i = 0; ok && i < n; ++i)
    ok = gs[i].M > 0 && gs[i].N > 0 && batches[i] > 0 && (int64_t)batches[i] * gs[i].nrep <= 65535;
  const char* core = getenv("REDCLIFF_GEMM_CORE");
  if (ok && core != nullptr && core[0] == 'v') ok = false;
  // every product on the LDS-tiled core (single replica), or a PAIR on the wave core (packed grids)
  bool lds = ok, wave = ok && n == 2;
  for (int i = 0; ok && i < n; ++i) {
    lds = lds && rc_gemm_lds_core(gs[i]);
    wave = wave && !rc_gemm_lds_core(gs[i]);
  }
  if (wave) {
    const bool wd = core != nullptr && core[0] == 'w' && core[1] == 'd';
    RcGemmSet set;
    set.n = 2;
    set.start[0] = 0;
    int idx = 0;
    for (int i = 0; i < 2 && wave; ++i) {
      RcGemm g = gs[i];
      g.batch = batches[i];
      const char* xe = getenv("REDCLIFF_GEMM_XCD");
      g.xcd = !(xe && xe[0] == '0');
      const int64_t nkb = (g.K + g.Kblk - 1) / g.Kblk;
      const int64_t extA = g.K <= 0 ? 1 : (nkb - 1) * g.rA + (g.ta ? (int64_t)(g.Kblk - 1) * g.lda + g.M : (int64_t)(g.M - 1) * g.lda + g.Kblk);
      const int64_t extB = g.K <= 0 ? 1 : (nkb - 1) * g.rB + (g.tb ? (int64_t)(g.N - 1) * g.ldb + g.Kblk : (int64_t)(g.Kblk - 1) * g.ldb + g.N);
      wave = extA < (1 << 28) && extB < (1 << 28) && g.rA >= 0 && g.rB >= 0;
      g.extA = (int)extA;
      g.extB = (int)extB;
      set.g[i] = g;
      set.nx[i] = (g.N + 31) / 32;
      set.ny[i] = (g.M + 31) / 32;
      set.nz[i] = batches[i] * g.nrep;
      const int64_t nb = (int64_t)set.nx[i] * set.ny[i] * set.nz[i];
      set.start[i + 1] = set.start[i] + (int)((nb + 7) / 8 * 8);
      const bool la = !wd && !g.ta, lb = !wd && g.tb;
      idx |= (la ? 1 : 0) << (2 * i) | (lb ? 2 : 0) << (2 * i);
    }
    if (wave) {
      static RcWavePairKern tab[16];
      static const bool init = (RcWavePairTab<15>::fill(tab), true);
      (void)init;
      set.start[3] = set.start[2];
      hipLaunchKernelGGL(tab[idx], dim3(set.start[2]), dim3(64), 0, s, set);
      return rc_check(hipGetLastError(), what);
    }
  }
  ok = lds;
  if (!ok) {
    for (int i = 0; i < n; ++i) {
      const int e = rc_gemm_launch(gs[i], batches[i], s, what);
      if (e) return e;
    }
    return 0;
  }
  static const int tile_env = [] {
    const char* v = getenv("REDCLIFF_GEMM_TILE");
    return v ? atoi(v) : 0;
  }();
  const char* xe = getenv("REDCLIFF_GEMM_XCD");
  // one tile size for the launch (the bits do not depend on it): 32 x 32 unless the products hold at
  // least two 64 x 64 tiles per CU between them
  RcGemmSet set;
  set.n = n;
  int64_t t64 = 0;
  for (int i = 0; i < n; ++i) {
    const int z = batches[i] * gs[i].nrep;
    t64 += (int64_t)((gs[i].N + 63) / 64) * ((gs[i].M + 63) / 64) * z;
  }
  const bool small = tile_env == 32 || (tile_env != 64 && t64 < 512);
  const int TT = small ? 32 : 64;
  set.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    set.g[i] = gs[i];
    set.g[i].batch = batches[i];
    set.g[i].xcd = !(xe && xe[0] == '0');
    set.nx[i] = (gs[i].N + TT - 1) / TT;
    set.ny[i] = (gs[i].M + TT - 1) / TT;
    set.nz[i] = batches[i] * gs[i].nrep;
    const int64_t nb = (int64_t)set.nx[i] * set.ny[i] * set.nz[i];
    set.start[i + 1] = set.start[i] + (int)((nb + 7) / 8 * 8);
  }
  for (int i = n; i < RC_GEMM_SET_MAX; ++i) set.start[i + 1] = set.start[n];
  if (small) hipLaunchKernelGGL(k_rc_gemm_mfma_set<32>, dim3(set.start[n]), dim3(RC_BLOCK), 0, s, set);
  else hipLaunchKernelGGL(k_rc_gemm_mfma_set<RC_GEMM_T>, dim3(set.start[n]), dim3(RC_BLOCK), 0, s, set);
  return rc_check(hipGetLastError(), what);
}

inline int rc_gemm_launch(const RcGemm& g0, int batch, hipStream_t s, const char* what) {
  if (g0.M <= 0 || g0.N <= 0 || batch <= 0 || g0.nrep <= 0) return 0;
  if (batch > 65535) { rc_set_error("%s: batch %d > 65535", what, batch); return REDCLIFF_ELIMIT; }
  RcGemm g = g0;
  g.batch = batch;
  if ((int64_t)batch * g.nrep > 65535) {  // grid z limit: the replicas in groups
    const int per = 65535 / batch;
    for (int i0 = 0; i0 < g0.nrep; i0 += per) {
      RcGemm h = g;
      h.nrep = g0.nrep - i0 < per ? g0.nrep - i0 : per;
      h.rident = 0;
      for (int i = 0; i < h.nrep; ++i) h.rmap[i] = (uint8_t)(g0.rident ? i0 + i : g0.rmap[i0 + i]);
      const int e = rc_gemm_launch(h, batch, s, what);
      if (e) return e;
    }
    return 0;
  }
  batch *= g.nrep;  // grid z: replicas x slices
  // fewer than two 64x64 tiles per CU: 32x32 tiles (more workgroups in flight to hide the
  // operand latency of these short products).  REDCLIFF_GEMM_TILE=64|32 overrides (tuning);
  // REDCLIFF_GEMM_CORE=valu selects the vector-ALU fmaf kernel (measurements).
  static const int tile_env = [] {
    const char* v = getenv("REDCLIFF_GEMM_TILE");
    return v ? atoi(v) : 0;
  }();
  const char* core = getenv("REDCLIFF_GEMM_CORE");  // read per launch: the tests switch it
  const bool valu = core != nullptr && core[0] == 'v';
  // Core choice (same bits): REDCLIFF_GEMM_CORE=wave (wave core, k-contiguous operands through LDS),
  // wd (wave core, every operand loaded straight into the lanes), mfma (LDS-tiled workgroups), valu.
  // Default: the wave core for every product.  Measured by product on the R = 128 D4IC grid, one stream
  // (profiles/r05_gemm_wave_ab.txt, r5aw): dW 33 -> 19.4 us, dfc1W 25 -> 20.2, graph conv ~26 -> 18.1,
  // dZ 25.0 -> 22.9, fc1 22.8 -> 21.6, dT 25.5 -> 25.7 against the LDS-tiled workgroups.  A single
  // fit's products (one replica: C5, p = 64, B = 128) keep the LDS-tiled workgroups, whose k-contiguous
  // tiles are shared by the workgroup's four column quarters: C5 with the wave core 0.4351 -> 0.4558 ms
  // per step (profiles/r05_c5_gemm_core_ab_ax.jsonl).
  const bool wd = core != nullptr && core[0] == 'w' && core[1] == 'd';
  const bool wave = core == nullptr ? g0.nrep > 1 : core[0] == 'w';
  const char* xe = getenv("REDCLIFF_GEMM_XCD");  // XCD-aware tile order: default on; 0 = dispatch order
  g.xcd = !(xe && xe[0] == '0');
  const int64_t t64 = (int64_t)((g.N + 63) / 64) * ((g.M + 63) / 64) * batch;
  // the wave core addresses its operands with 32-bit offsets: only slices whose extent fits
  const int64_t nkb = (g.K + g.Kblk - 1) / g.Kblk;
  const int64_t extA = g.K <= 0 ? 1 : (nkb - 1) * g.rA + (g.ta ? (int64_t)(g.Kblk - 1) * g.lda + g.M : (int64_t)(g.M - 1) * g.lda + g.Kblk);
  const int64_t extB = g.K <= 0 ? 1 : (nkb - 1) * g.rB + (g.tb ? (int64_t)(g.N - 1) * g.ldb + g.Kblk : (int64_t)(g.Kblk - 1) * g.ldb + g.N);
  if (wave && extA < (1 << 28) && extB < (1 << 28) && g.rA >= 0 && g.rB >= 0) {
    g.extA = (int)extA;
    g.extB = (int)extB;
    dim3 grid((g.N + 31) / 32, (g.M + 31) / 32, batch);
    const bool la = !wd && !g.ta, lb = !wd && g.tb;
    if (la && lb) hipLaunchKernelGGL((k_rc_gemm_wave<true, true>), grid, dim3(64), 0, s, g);
    else if (la) hipLaunchKernelGGL((k_rc_gemm_wave<true, false>), grid, dim3(64), 0, s, g);
    else if (lb) hipLaunchKernelGGL((k_rc_gemm_wave<false, true>), grid, dim3(64), 0, s, g);
    else hipLaunchKernelGGL((k_rc_gemm_wave<false, false>), grid, dim3(64), 0, s, g);
    return rc_check(hipGetLastError(), what);
  }
  const bool small = tile_env == 32 || (tile_env != 64 && t64 < 512);
  if (small) {
    dim3 grid((g.N + 31) / 32, (g.M + 31) / 32, batch);
    if (valu) hipLaunchKernelGGL(k_rc_gemm<32>, grid, dim3(RC_BLOCK), 0, s, g);
    else hipLaunchKernelGGL(k_rc_gemm_mfma<32>, grid, dim3(RC_BLOCK), 0, s, g);
  } else {
    dim3 grid((g.N + RC_GEMM_T - 1) / RC_GEMM_T, (g.M + RC_GEMM_T - 1) / RC_GEMM_T, batch);
    if (valu) hipLaunchKernelGGL(k_rc_gemm<RC_GEMM_T>, grid, dim3(RC_BLOCK), 0, s, g);
    else hipLaunchKernelGGL(k_rc_gemm_mfma<RC_GEMM_T>, grid, dim3(RC_BLOCK), 0, s, g);
  }
  return rc_check(hipGetLastError(), what);
}
