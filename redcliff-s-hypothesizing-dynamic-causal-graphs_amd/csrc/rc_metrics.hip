// rc_metrics.hip -- the per-epoch GC-progress metrics of REDCLIFF-S fit() on the GPU.
//
// Reference: general_utils/model_utils.py:18-160 (track_receiver_operating_characteristic_stats_
// for_redcliff_models, track_deltacon0_related_stats_for_redcliff_models) over
// general_utils/metrics.py:111-252 (get_k_length_path_adjacencies, matsusita_distance,
// compute_node_affinity_matrix, deltacon0, deltacon0_with_directed_degrees, deltaffinity,
// path_length_mse) and :396-430 (get_f1_score), sklearn.metrics.roc_auc_score.  The reference
// runs them in numpy / sklearn on the host once per epoch; at microsecond training steps that
// host work is most of a fit's wall clock.
//
// One workgroup per (sample s, graph g), p <= 64.  The dtype flow of the reference is kept:
// the estimate side is float32 (np.sum over lags with numpy's pairwise order, the max
// normalisation, the python-float scalings, the matrix powers), the truth side float64, the
// affinity matrices and distances float64 (inverses by Gauss-Jordan with partial pivoting where
// numpy calls LAPACK).  F1 is the float32 arithmetic of get_f1_score on exact counts; ROC-AUC
// is the Mann-Whitney form of sklearn's trapezoidal area (ties count 1/2), from exact counts.
#include <cstdlib>
#include <cstring>

#include "rc_common.h"

namespace {

// Threads per workgroup NT: 1024 for p > 32 (16 waves keep the LDS / FP64 latencies of one
// (sample, graph) hidden; one workgroup per CU at 36 p^2 bytes of LDS, p = 64), 256 for
// 16 < p <= 32, 64 for p <= 16: one wave per (sample, graph), whose ~300 barriers (four
// Gauss-Jordan inverses, the path-length powers) are then single-wave barriers -- a D4IC-sized
// packed grid's 2,048 (sample, graph) workgroups ran 178 us with four waves each.  The NT = 64
// form sums its float64 terms in the 256-thread form's association (gp_sum_terms), so every
// metric is the same bits (REDCLIFF_GCP_WAVE=0 keeps the 256-thread form).
#define GP_NR 4     // matrix elements per thread: p * p <= GP_NR * NT

// numpy's float32 pairwise sum of a contiguous run (loops_utils.h.src, n <= 128)
__device__ inline float np_pairwise_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}
__device__ inline double np_pairwise_f64(const double* a, int stride, int n) {
  if (n < 8) {
    double r = 0.;
    for (int i = 0; i < n; ++i) r += a[i * stride];
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * stride];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i * stride];
  return res;
}
__device__ inline float np_pairwise_f32s(const float* a, int stride, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i * stride];
    return r;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * stride];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i * stride];
  return res;
}

template <int NT>
__device__ inline float gp_block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float m = red[0];
  for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[i]);
  __syncthreads();
  return m;
}

// Sum of per-element float64 terms tu[u] (element e = tid + u * NT, 0 where e >= p * p) in the
// arithmetic of the 256-thread workgroup: thread partials, each wave's butterfly sum (lane 0's),
// the waves in order.  NT = 64 (one wave per (sample, graph), p * p <= 256): the 256-thread
// workgroup's thread t held exactly element t, so its wave u is this wave's term u -- the same
// association without a block barrier.
template <int NT>
__device__ inline double gp_sum_terms(const double* tu, double* redd) {
  if (NT == 64) {
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      double v = tu[u];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      s += __shfl(v, 0, 64);
    }
    return s;
  }
  double acc = 0.;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) acc += tu[u];
  return rc_block_sum_d(acc, redd);
}

// inverse of the p x p float64 matrix in the left half of Aug[p][2p] (right half := I):
// Gauss-Jordan with partial pivoting (first maximal |pivot|, as LAPACK's idamax), result in
// the right half.  Singular columns leave inf / nan, as numpy's inv would raise.
template <int NT>
__device__ void gp_inverse(double* Aug, int p, double* redd, int* redi) {
  const int tid = threadIdx.x, P2 = 2 * p;
  for (int e = tid; e < p * p; e += NT) {
    const int i = e / p, j = e - i * p;
    Aug[i * P2 + p + j] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int c = 0; c < p; ++c) {
    // pivot row: max |Aug[r][c]|, r >= c, first index on ties (one wave, p <= 64)
    if (tid < 64) {
      double v = (tid >= c && tid < p) ? fabs(Aug[tid * P2 + c]) : -1.0;
      int idx = tid;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(idx, o, 64);
        if (v2 > v || (v2 == v && i2 < idx)) { v = v2; idx = i2; }
      }
      if (tid == 0) redi[0] = idx;
    }
    __syncthreads();
    const int piv = redi[0];
    if (piv != c)
      for (int j = tid; j < P2; j += NT) {
        const double t = Aug[c * P2 + j];
        Aug[c * P2 + j] = Aug[piv * P2 + j];
        Aug[piv * P2 + j] = t;
      }
    __syncthreads();
    const double inv = 1.0 / Aug[c * P2 + c];
    __syncthreads();
    for (int j = tid; j < P2; j += NT) Aug[c * P2 + j] *= inv;
    __syncthreads();
    // eliminate column c from every other row; the multipliers are read before any write
    if (tid < p) redd[tid] = Aug[tid * P2 + c];
    __syncthreads();
    for (int e = tid; e < p * P2; e += NT) {
      const int i = e / P2, j = e - i * P2;
      if (i != c) Aug[e] -= redd[i] * Aug[c * P2 + j];
    }
    __syncthreads();
  }
}

struct GpRoc {
  double f1, auc;
};
// ROC-AUC / F1 of one estimate variant: x (float32, prepared) against truth t (float64).
// ROC-AUC = Mann-Whitney count over (positive, negative) pairs; the positives' and negatives'
// scores are first compacted into LDS (xp, xn: any order -- the counts are integers, exact in
// double in any summation order), then every thread walks all negatives for its positives with
// one broadcast LDS read per pair.
template <int NT>
__device__ GpRoc gp_roc_f1(const float* xs, const double* t, int pp, double* redd, float* xp, float* xn, int* cnt) {
  const int tid = threadIdx.x;
  // F1 counts (get_f1_score): masks of x > 0, x == 0, t > 0, t == 0
  double tp = 0., ppos = 0., pz = 0., tn = 0., nan = 0.;
  if (tid < 2) cnt[tid] = 0;
  __syncthreads();
  for (int e = tid; e < pp; e += NT) {
    const float x = xs[e];
    const double tv = t[e];
    const bool pp_ = x > 0.f, pn_ = x == 0.f, lp = tv > 0.0, ln = tv == 0.0;
    tp += (pp_ && lp) ? 1.0 : 0.0;
    ppos += pp_ ? 1.0 : 0.0;
    pz += pn_ ? 1.0 : 0.0;
    tn += (pn_ && ln) ? 1.0 : 0.0;
    nan += (x != x) ? 1.0 : 0.0;
    // ROC-AUC labels int(t) (1 only where the normalised truth is 1)
    const int lab = (int)tv;
    if (lab == 1) xp[atomicAdd(&cnt[0], 1)] = x;
    else if (lab == 0) xn[atomicAdd(&cnt[1], 1)] = x;
  }
  tp = rc_block_sum_d(tp, redd);
  ppos = rc_block_sum_d(ppos, redd);
  pz = rc_block_sum_d(pz, redd);
  tn = rc_block_sum_d(tn, redd);
  nan = rc_block_sum_d(nan, redd);  // its barriers also publish xp / xn / cnt
  const float ftp = (float)tp, ffp = (float)(ppos - tp), ffn = (float)(pz - tn);
  const float prec = ftp / (ftp + ffp), rec = ftp / (ftp + ffn);
  GpRoc o;
  o.f1 = (prec + rec == 0.f) ? 0.0 : (double)((2.f * (prec * rec)) / (prec + rec));
  const int npos = cnt[0], nneg = cnt[1];
  double cnt2 = 0.;
  for (int a = tid; a < npos; a += NT) {
    const float xi = xp[a];
    int c2 = 0;
    for (int b = 0; b < nneg; ++b) {
      const float xj = xn[b];
      c2 += xi > xj ? 2 : (xi == xj ? 1 : 0);
    }
    cnt2 += (double)c2;
  }
  cnt2 = rc_block_sum_d(cnt2, redd);
  if (npos == 0) o.auc = 0.5;  // the reference's guard (sum(labels) == 0)
  else if (nneg == 0 || nan > 0.) o.auc = __builtin_nan("");  // sklearn raises
  else o.auc = cnt2 / (2.0 * (double)npos * (double)nneg);
  return o;
}

// grid (S * G); dynamic LDS 36 p^2 bytes (+ small statics).  Sample s is scored against truth
// block s / spt ([2][G][p][p] each): one block for a fit, one per replica for a packed grid whose
// replicas fit different data sets (each with its own true graphs).
template <int NT>
__global__ __launch_bounds__(NT) void k_gc_progress(int S, int spt, int nE, int G, int p, int Lt, const float* est,
                                                          const double* truth, const double* eps_pow, double cin,
                                                          double cout, double* out) {
  const int s = blockIdx.x / G, g = blockIdx.x - s * G;
  const int pp = p * p, NM = 6 + p, tid = threadIdx.x;
  truth += (int64_t)(s / spt) * 2 * G * pp;
  extern __shared__ double smd[];
  double* T = smd;                                   // [pp] truth (with self-connections)
  double* Aug = T + pp;                              // [p][2p] inverse workspace; later Tk | Tn
  float* Ex = reinterpret_cast<float*>(Aug + 2 * pp);  // [pp] prepared estimate (ROC / deltacon)
  float* Ek = Ex + pp;                               // [pp] E^k
  float* En = Ek + pp;                               // [pp] E^(k+1)
  __shared__ double redd[64];
  __shared__ float redf[NT / 64];
  __shared__ int cnt[2];
  __shared__ int redi[4];
  __shared__ double degT[64], degE[64];
  __shared__ double seb[NT == 64 ? GP_NR * 64 : 1];  // NT = 64: per-element terms, element order

  // estimate summed over lags: numpy float32 pairwise order
  const float* ep = est + ((int64_t)s * nE + g) * pp * Lt;
  float es[GP_NR];
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * NT;
    es[u] = e < pp ? np_pairwise_f32(ep + (int64_t)e * Lt, Lt) : 0.f;
  }
  double* o = out + ((int64_t)s * G + g) * NM;

  // ---- F1 / ROC-AUC, with and without self-connections (model_utils.py:18-86)
  for (int v = 0; v < 2; ++v) {
    const double* t = truth + ((int64_t)v * G + g) * pp;
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      const int e = tid + u * NT;
      if (e < pp) {
        const int i = e / p;
        const float x = (v == 1 && e == i * p + i) ? 0.f : es[u];
        mx = fmaxf(mx, x);
      }
    }
    mx = gp_block_max<NT>(mx, redf);
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      const int e = tid + u * NT;
      if (e < pp) {
        const int i = e / p;
        float x = (v == 1 && e == i * p + i) ? 0.f : es[u];
        if (mx != 0.f) x = x / mx;
        Ex[e] = x * ((x > 0.f) ? 1.f : 0.f);  // curr_est * (curr_est > 0.)
      }
    }
    __syncthreads();
    const GpRoc rr = gp_roc_f1<NT>(Ex, t, pp, redd, Ek, En, cnt);
    if (tid == 0) {
      o[2 * v] = rr.f1;
      o[2 * v + 1] = rr.auc;
    }
    __syncthreads();
  }

  // ---- deltacon0 / with directed degrees (model_utils.py:90-160, metrics.py:136-216)
  const double* t0 = truth + (int64_t)g * pp;
  double tm_all = -INFINITY;
  for (int e = tid; e < pp; e += NT) {
    T[e] = t0[e];
    tm_all = fmax(tm_all, t0[e]);
  }
  float emx = -INFINITY;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u)
    if (tid + u * NT < pp) emx = fmaxf(emx, es[u]);
  emx = gp_block_max<NT>(emx, redf);
  {
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) tm_all = fmax(tm_all, __shfl_xor(tm_all, o2, 64));
    const int lane = tid & 63, wv = tid >> 6;
    if (lane == 0) redd[8 + wv] = tm_all;
    __syncthreads();
    double m = redd[8];
    for (int i = 1; i < NT / 64; ++i) m = fmax(m, redd[8 + i]);
    tm_all = m;
    __syncthreads();
  }
  // the reference divides the estimate by its own max when the TRUTH's max is nonzero
  const bool tnorm = tm_all != 0.0;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * NT;
    if (e < pp) Ex[e] = tnorm ? es[u] / emx : es[u];
  }
  __syncthreads();
  const double eps = eps_pow[1], eps2 = eps_pow[2];
  const float eps_f = (float)eps, eps2_f = (float)eps2;
  double d_in = 0., d_out = 0.;
  double sreg[GP_NR];  // the truth-side affinity matrix of the current direction
  for (int dir = 0; dir < 2; ++dir) {
    // degrees: in = column sums (np.sum axis 0: sequential over rows), out = row sums (pairwise)
    if (tid < p) {
      if (dir == 0) {
        double a = 0.;
        float b = 0.f;
        for (int i = 0; i < p; ++i) {
          a += T[i * p + tid];
          b += Ex[i * p + tid];
        }
        degT[tid] = a;
        degE[tid] = (double)b;
      } else {
        degT[tid] = np_pairwise_f64(T + tid * p, 1, p);
        degE[tid] = (double)np_pairwise_f32s(Ex + tid * p, 1, p);
      }
    }
    __syncthreads();
    for (int side = 0; side < 2; ++side) {
      // I + (eps^2) D - eps A
      for (int e = tid; e < pp; e += NT) {
        const int i = e / p, j = e - i * p;
        double mval;
        if (side == 0) {
          const double a = (i == j ? 1.0 : 0.0) + (i == j ? eps2 * degT[i] : 0.0);
          mval = a - eps * T[e];
        } else {
          const float dd = (i == j) ? eps2_f * (float)degE[i] : 0.f;
          mval = ((i == j ? 1.0 : 0.0) + (double)dd) - (double)(eps_f * Ex[e]);
        }
        Aug[i * 2 * p + j] = mval;
      }
      __syncthreads();
      gp_inverse<NT>(Aug, p, redd, redi);
      if (side == 0) {
#pragma unroll
        for (int u = 0; u < GP_NR; ++u) {
          const int e = tid + u * NT;
          if (e < pp) {
            const int i = e / p, j = e - i * p;
            sreg[u] = Aug[i * 2 * p + p + j];
          }
        }
        __syncthreads();
      } else {
        double tu[GP_NR];
#pragma unroll
        for (int u = 0; u < GP_NR; ++u) {
          const int e = tid + u * NT;
          tu[u] = 0.;
          if (e < pp) {
            const int i = e / p, j = e - i * p;
            const double df = sqrt(sreg[u]) - sqrt(Aug[i * 2 * p + p + j]);
            tu[u] = df * df;
          }
        }
        const double d = sqrt(gp_sum_terms<NT>(tu, redd));
        if (dir == 0) d_in = d; else d_out = d;
      }
    }
  }
  if (tid == 0) {
    o[4] = 1.0 / (1.0 + d_in);
    o[5] = 1.0 / (1.0 + ((cin * d_in) + (cout * d_out)) / 2.0);
  }
  __syncthreads();

  // ---- deltaffinity and path-length MSE over k = 1..p-1 (metrics.py:142-252)
  // Thread layout of this section: column j = tid % p, rows r0, r0 + rpp, ... (rpp = NT / p
  // rows per pass, at most GP_NR passes), so a thread's outputs of A^k = A^(k-1) A share the
  // column operand A[m][j] and run GP_NR independent fma chains (each output still sums over m
  // in ascending order, as before).  Tk/Tn and Ek/En alternate instead of being copied back.
  const int rpp = NT / p, jc = tid % p, r0 = tid / p;
  const bool act = r0 < rpp;
  double* Tk = Aug;
  double* Tn = Aug + pp;
  double sa1[GP_NR], sa2[GP_NR];
  for (int e = tid; e < pp; e += NT) {
    Tk[e] = T[e];
    Ek[e] = Ex[e];
  }
#pragma unroll
  for (int v = 0; v < GP_NR; ++v) {
    const int i = r0 + v * rpp;
    sa1[v] = (act && i < p && i == jc) ? 1.0 : 0.0;
    sa2[v] = sa1[v];
  }
  __syncthreads();
  for (int k = 1; k < p; ++k) {
    if (k > 1) {  // A^k = A^(k-1) A
      if (act) {
        double a[GP_NR];
        float b[GP_NR];
#pragma unroll
        for (int v = 0; v < GP_NR; ++v) {
          a[v] = 0.;
          b[v] = 0.f;
        }
        for (int m = 0; m < p; ++m) {
          const double tm = T[m * p + jc];
          const float xm = Ex[m * p + jc];
#pragma unroll
          for (int v = 0; v < GP_NR; ++v) {
            const int i = r0 + v * rpp;
            if (i < p) {
              a[v] += Tk[i * p + m] * tm;
              b[v] += Ek[i * p + m] * xm;
            }
          }
        }
#pragma unroll
        for (int v = 0; v < GP_NR; ++v) {
          const int i = r0 + v * rpp;
          if (i < p) {
            Tn[i * p + jc] = a[v];
            En[i * p + jc] = b[v];
          }
        }
      }
      __syncthreads();
      double* tt = Tk;
      Tk = Tn;
      Tn = tt;
      float* ff = Ek;
      Ek = En;
      En = ff;
    }
    const double ck = eps_pow[k];
    const float ckf = (float)ck;
    double se = 0.;
    if (act) {
#pragma unroll
      for (int v = 0; v < GP_NR; ++v) {
        const int i = r0 + v * rpp;
        if (i < p) {
          const double tk = Tk[i * p + jc];
          const float ek = Ek[i * p + jc];
          sa1[v] = sa1[v] + ck * tk;
          sa2[v] = sa2[v] + (double)(ckf * ek);
          const double df = tk - (double)ek;
          if (NT == 64) seb[i * p + jc] = df * df;
          else se += df * df;
        }
      }
    }
    if (NT == 64) {  // the terms in element order (the 256-thread workgroup held element t in thread t)
      __syncthreads();
      double tu[GP_NR];
#pragma unroll
      for (int u = 0; u < GP_NR; ++u) tu[u] = (tid + u * NT < pp) ? seb[tid + u * NT] : 0.;
      se = gp_sum_terms<NT>(tu, redd);
      __syncthreads();  // this pass's reads before the next writes
    } else {
      se = rc_block_sum_d(se, redd);  // its barriers also order this pass's reads before the next writes
    }
    if (tid == 0) o[6 + k] = se / (double)pp;
  }
  double acc = 0.;
  if (act) {
#pragma unroll
    for (int v = 0; v < GP_NR; ++v) {
      const int i = r0 + v * rpp;
      if (i < p) {
        const double df = sqrt(sa1[v]) - sqrt(sa2[v]);
        if (NT == 64) seb[i * p + jc] = df * df;
        else acc += df * df;
      }
    }
  }
  double dsum;
  if (NT == 64) {
    __syncthreads();
    double tu[GP_NR];
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) tu[u] = (tid + u * NT < pp) ? seb[tid + u * NT] : 0.;
    dsum = gp_sum_terms<NT>(tu, redd);
  } else {
    dsum = rc_block_sum_d(acc, redd);
  }
  const double dd = sqrt(dsum);
  if (tid == 0) o[6] = 1.0 / (1.0 + dd);
}


// ---- per-epoch tracker statistics (model_utils.py:163-209: track_l1_stats, track_cosine_stats)
// The reference converts every estimate to float64 on the host and reduces it there; a packed
// grid search would copy R x S x K full lagged estimates per epoch (tens of MB at p = 64).
// Here one workgroup reduces one row (a fixed order: per-thread strided partial sums, wave tree,
// waves in order -- independent of how many rows a launch holds), so a replica's values do not
// depend on the pack it runs in.

__device__ inline float gp_block_maxf(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float m = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
  __syncthreads();
  return m;
}

// grid (nrows): out[row] = sum_i |x_i / max(x)| in float64 over the n floats of the row
__global__ __launch_bounds__(RC_BLOCK) void k_gc_l1(const float* x, int64_t n, double* out) {
  const float* r = x + (int64_t)blockIdx.x * n;
  __shared__ float redf[RC_BLOCK / 64];
  __shared__ double redd[RC_BLOCK / 64];
  float mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += RC_BLOCK) mx = fmaxf(mx, r[i]);
  const double m = (double)gp_block_maxf(mx, redf);
  double acc = 0.;
  for (int64_t i = threadIdx.x; i < n; i += RC_BLOCK) acc += fabs((double)r[i] / m);
  acc = rc_block_sum_d(acc, redd);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// grid (ceil(nsamp / 8)), one WAVE per GD_SPW samples: the K rows of sample s (n floats each), each
// divided by its own max in float64: out[s][i1][i2] = sum_e f1_e f2_e for i1 <= i2 (the diagonal
// is the squared norm).  The sums are those of a 256-thread workgroup per (sample, pair):
// virtual thread (vw, lane) sums e = 64 vw + lane + 256 i, each virtual wave's sum is lane 0's
// butterfly sum, the four are added in order -- the same bits without a block barrier (one
// workgroup per pair made ~50K tiny workgroups at a packed grid's 5,120 samples).
#define GD_VW (RC_BLOCK / 64)
#define GD_SPW 1  // samples per wave (2: slower at R = 128 D4IC, 26 -> 34 us)
__global__ __launch_bounds__(RC_BLOCK) void k_gc_dots(const float* x, int K, int64_t n, int nsamp, double* out) {
  const int lane = threadIdx.x & 63;
  const int s0 = (blockIdx.x * (RC_BLOCK / 64) + (threadIdx.x >> 6)) * GD_SPW;
  for (int s = s0; s < s0 + GD_SPW && s < nsamp; ++s) {
    const float* xs = x + (int64_t)s * K * n;
    double mine = 0.0;  // lane i < K: row i's max
    for (int i = 0; i < K; ++i) {
      const float* a = xs + (int64_t)i * n;
      float m = -INFINITY;
      for (int64_t e = lane; e < n; e += 64) m = fmaxf(m, a[e]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (lane == i) mine = (double)m;
    }
    // virtual waves holding elements; the others add exact +0 sums (one +0.0 stands for them)
    const int nvw = (int)((n + 63) / 64 < GD_VW ? (n + 63) / 64 : GD_VW);
    for (int i1 = 0; i1 < K; ++i1) {
      const float* a = xs + (int64_t)i1 * n;
      const double da = __shfl(mine, i1, 64);
      for (int i2 = i1; i2 < K; ++i2) {
        const float* b = xs + (int64_t)i2 * n;
        const double db = __shfl(mine, i2, 64);
        double acc = 0.0;
#pragma unroll
        for (int vw = 0; vw < GD_VW; ++vw) {
          if (vw >= nvw) break;
          double v = 0.;
          for (int64_t e = vw * 64 + lane; e < n; e += RC_BLOCK) v += ((double)a[e] / da) * ((double)b[e] / db);
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
          acc += __shfl(v, 0, 64);
        }
        if (nvw < GD_VW) acc += 0.0;  // the empty virtual waves' +0 sums (x + 0 + 0 == x + 0)
        if (lane == 0) out[((int64_t)s * K + i1) * K + i2] = acc;
      }
    }
  }
}

}  // namespace

extern "C" int redcliff_gc_progress_grouped(int32_t S, int32_t spt, int32_t nE, int32_t G, int32_t p, int32_t Lt,
                                            const float* est, const double* truth, const double* eps_pow,
                                            double in_degree_coeff, double out_degree_coeff, double* out,
                                            void* stream) {
  if (S > 0 && spt < 1) { rc_set_error("gc_progress: samples per truth block must be >= 1"); return REDCLIFF_EINVAL; }
  if (S < 0 || G < 0 || nE < G || p < 2 || p > 64 || Lt < 1 || Lt > 128 || (S * G > 0 && (!est || !truth || !eps_pow || !out))) {
    rc_set_error("gc_progress: bad arguments (S=%d nE=%d G=%d p=%d Lt=%d; need 2 <= p <= 64, Lt <= 128, G <= nE)", S, nE,
                 G, p, Lt);
    return REDCLIFF_EINVAL;
  }
  if (S * G == 0) return 0;
  const size_t lds = (size_t)36 * p * p;
  static const bool wave_form = [] {
    const char* v = getenv("REDCLIFF_GCP_WAVE");
    return !(v && strcmp(v, "0") == 0);
  }();
  if (p <= 16 && wave_form) {  // one wave per (sample, graph): the same bits as the 256-thread form
    hipLaunchKernelGGL(k_gc_progress<64>, dim3(S * G), dim3(64), lds, (hipStream_t)stream, S, spt, nE, G, p, Lt, est,
                       truth, eps_pow, in_degree_coeff, out_degree_coeff, out);
  } else if (p <= 32) {
    hipLaunchKernelGGL(k_gc_progress<256>, dim3(S * G), dim3(256), lds, (hipStream_t)stream, S, spt, nE, G, p, Lt, est,
                       truth, eps_pow, in_degree_coeff, out_degree_coeff, out);
  } else {
    if (lds > 64 * 1024) {
      const int e = rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k_gc_progress<1024>),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                             "k_gc_progress LDS");
      if (e) return e;
    }
    hipLaunchKernelGGL(k_gc_progress<1024>, dim3(S * G), dim3(1024), lds, (hipStream_t)stream, S, spt, nE, G, p, Lt, est,
                       truth, eps_pow, in_degree_coeff, out_degree_coeff, out);
  }
  return rc_check(hipGetLastError(), "k_gc_progress");
}

extern "C" int redcliff_gc_progress(int32_t S, int32_t nE, int32_t G, int32_t p, int32_t Lt, const float* est,
                                    const double* truth, const double* eps_pow, double in_degree_coeff,
                                    double out_degree_coeff, double* out, void* stream) {
  return redcliff_gc_progress_grouped(S, S > 0 ? S : 1, nE, G, p, Lt, est, truth, eps_pow, in_degree_coeff,
                                      out_degree_coeff, out, stream);
}

extern "C" int redcliff_gc_track_stats(int32_t n_l1_rows, int64_t l1_len, const float* est, double* l1_out,
                                       int32_t n_samples, int32_t K, int64_t row_len, const float* nolag,
                                       double* dots_out, void* stream) {
  if (n_l1_rows < 0 || n_samples < 0 || K < 1 || K > 64 || (n_l1_rows > 0 && (l1_len < 1 || !est || !l1_out)) ||
      (n_samples > 0 && (row_len < 1 || !nolag || !dots_out))) {
    rc_set_error("gc_track_stats: bad arguments (rows=%d len=%lld samples=%d K=%d row_len=%lld)", n_l1_rows,
                 (long long)l1_len, n_samples, K, (long long)row_len);
    return REDCLIFF_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (n_l1_rows > 0) {
    hipLaunchKernelGGL(k_gc_l1, dim3(n_l1_rows), dim3(RC_BLOCK), 0, s, est, l1_len, l1_out);
    const int e = rc_check(hipGetLastError(), "k_gc_l1");
    if (e) return e;
  }
  if (n_samples > 0) {
    const int per = GD_VW * GD_SPW;  // samples per workgroup
    hipLaunchKernelGGL(k_gc_dots, dim3((n_samples + per - 1) / per), dim3(RC_BLOCK), 0, s, nolag, K, row_len,
                       n_samples, dots_out);
    return rc_check(hipGetLastError(), "k_gc_dots");
  }
  return 0;
}
