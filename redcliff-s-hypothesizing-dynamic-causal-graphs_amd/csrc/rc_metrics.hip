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
#include "rc_common.h"

namespace {

#define GP_NR 16  // matrix elements per thread: p * p <= GP_NR * RC_BLOCK

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

__device__ inline float gp_block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float m = red[0];
  for (int i = 1; i < RC_BLOCK / 64; ++i) m = fmaxf(m, red[i]);
  __syncthreads();
  return m;
}

// inverse of the p x p float64 matrix in the left half of Aug[p][2p] (right half := I):
// Gauss-Jordan with partial pivoting (first maximal |pivot|, as LAPACK's idamax), result in
// the right half.  Singular columns leave inf / nan, as numpy's inv would raise.
__device__ void gp_inverse(double* Aug, int p, double* redd, int* redi) {
  const int tid = threadIdx.x, P2 = 2 * p;
  for (int e = tid; e < p * p; e += RC_BLOCK) {
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
      for (int j = tid; j < P2; j += RC_BLOCK) {
        const double t = Aug[c * P2 + j];
        Aug[c * P2 + j] = Aug[piv * P2 + j];
        Aug[piv * P2 + j] = t;
      }
    __syncthreads();
    const double inv = 1.0 / Aug[c * P2 + c];
    __syncthreads();
    for (int j = tid; j < P2; j += RC_BLOCK) Aug[c * P2 + j] *= inv;
    __syncthreads();
    // eliminate column c from every other row; the multipliers are read before any write
    if (tid < p) redd[tid] = Aug[tid * P2 + c];
    __syncthreads();
    for (int e = tid; e < p * P2; e += RC_BLOCK) {
      const int i = e / P2, j = e - i * P2;
      if (i != c) Aug[e] -= redd[i] * Aug[c * P2 + j];
    }
    __syncthreads();
  }
}

// ROC-AUC / F1 of one estimate variant: x (float32, prepared) against truth t (float64)
struct GpRoc {
  double f1, auc;
};
__device__ GpRoc gp_roc_f1(const float* xs, const double* t, int pp, double* redd) {
  const int tid = threadIdx.x;
  // F1 counts (get_f1_score): masks of x > 0, x == 0, t > 0, t == 0
  double tp = 0., ppos = 0., pz = 0., tn = 0.;
  for (int e = tid; e < pp; e += RC_BLOCK) {
    const float x = xs[e];
    const double tv = t[e];
    const bool pp_ = x > 0.f, pn_ = x == 0.f, lp = tv > 0.0, ln = tv == 0.0;
    tp += (pp_ && lp) ? 1.0 : 0.0;
    ppos += pp_ ? 1.0 : 0.0;
    pz += pn_ ? 1.0 : 0.0;
    tn += (pn_ && ln) ? 1.0 : 0.0;
  }
  tp = rc_block_sum_d(tp, redd);
  ppos = rc_block_sum_d(ppos, redd);
  pz = rc_block_sum_d(pz, redd);
  tn = rc_block_sum_d(tn, redd);
  const float ftp = (float)tp, ffp = (float)(ppos - tp), ffn = (float)(pz - tn);
  const float prec = ftp / (ftp + ffp), rec = ftp / (ftp + ffn);
  GpRoc o;
  o.f1 = (prec + rec == 0.f) ? 0.0 : (double)((2.f * (prec * rec)) / (prec + rec));
  // ROC-AUC: labels int(t) (1 only where the normalised truth is 1); ties count 1/2
  double npos = 0., nneg = 0., cnt2 = 0., nan = 0.;
  for (int e = tid; e < pp; e += RC_BLOCK) {
    const int lab = (int)t[e];
    npos += lab == 1 ? 1.0 : 0.0;
    nneg += lab == 0 ? 1.0 : 0.0;
    nan += (xs[e] != xs[e]) ? 1.0 : 0.0;
    if (lab == 1) {
      const float xi = xs[e];
      double c2 = 0.;
      for (int j = 0; j < pp; ++j)
        if ((int)t[j] == 0) {
          const float xj = xs[j];
          c2 += xi > xj ? 2.0 : (xi == xj ? 1.0 : 0.0);
        }
      cnt2 += c2;
    }
  }
  npos = rc_block_sum_d(npos, redd);
  nneg = rc_block_sum_d(nneg, redd);
  cnt2 = rc_block_sum_d(cnt2, redd);
  nan = rc_block_sum_d(nan, redd);
  if (npos == 0.) o.auc = 0.5;  // the reference's guard (sum(labels) == 0)
  else if (nneg == 0. || nan > 0.) o.auc = __builtin_nan("");  // sklearn raises
  else o.auc = cnt2 / (2.0 * npos * nneg);
  return o;
}

// grid (S * G); dynamic LDS 36 p^2 bytes (+ small statics)
__global__ __launch_bounds__(RC_BLOCK) void k_gc_progress(int S, int nE, int G, int p, int Lt, const float* est,
                                                          const double* truth, const double* eps_pow, double cin,
                                                          double cout, double* out) {
  const int s = blockIdx.x / G, g = blockIdx.x - s * G;
  const int pp = p * p, NM = 6 + p, tid = threadIdx.x;
  extern __shared__ double smd[];
  double* T = smd;                                   // [pp] truth (with self-connections)
  double* Aug = T + pp;                              // [p][2p] inverse workspace; later Tk | Tn
  float* Ex = reinterpret_cast<float*>(Aug + 2 * pp);  // [pp] prepared estimate (ROC / deltacon)
  float* Ek = Ex + pp;                               // [pp] E^k
  float* En = Ek + pp;                               // [pp] E^(k+1)
  __shared__ double redd[64];
  __shared__ float redf[8];
  __shared__ int redi[4];
  __shared__ double degT[64], degE[64];

  // estimate summed over lags: numpy float32 pairwise order
  const float* ep = est + ((int64_t)s * nE + g) * pp * Lt;
  float es[GP_NR];
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * RC_BLOCK;
    es[u] = e < pp ? np_pairwise_f32(ep + (int64_t)e * Lt, Lt) : 0.f;
  }
  double* o = out + ((int64_t)s * G + g) * NM;

  // ---- F1 / ROC-AUC, with and without self-connections (model_utils.py:18-86)
  for (int v = 0; v < 2; ++v) {
    const double* t = truth + ((int64_t)v * G + g) * pp;
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      const int e = tid + u * RC_BLOCK;
      if (e < pp) {
        const int i = e / p;
        const float x = (v == 1 && e == i * p + i) ? 0.f : es[u];
        mx = fmaxf(mx, x);
      }
    }
    mx = gp_block_max(mx, redf);
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      const int e = tid + u * RC_BLOCK;
      if (e < pp) {
        const int i = e / p;
        float x = (v == 1 && e == i * p + i) ? 0.f : es[u];
        if (mx != 0.f) x = x / mx;
        Ex[e] = x * ((x > 0.f) ? 1.f : 0.f);  // curr_est * (curr_est > 0.)
      }
    }
    __syncthreads();
    const GpRoc rr = gp_roc_f1(Ex, t, pp, redd);
    if (tid == 0) {
      o[2 * v] = rr.f1;
      o[2 * v + 1] = rr.auc;
    }
    __syncthreads();
  }

  // ---- deltacon0 / with directed degrees (model_utils.py:90-160, metrics.py:136-216)
  const double* t0 = truth + (int64_t)g * pp;
  double tm_all = -INFINITY;
  for (int e = tid; e < pp; e += RC_BLOCK) {
    T[e] = t0[e];
    tm_all = fmax(tm_all, t0[e]);
  }
  float emx = -INFINITY;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u)
    if (tid + u * RC_BLOCK < pp) emx = fmaxf(emx, es[u]);
  emx = gp_block_max(emx, redf);
  {
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) tm_all = fmax(tm_all, __shfl_xor(tm_all, o2, 64));
    const int lane = tid & 63, wv = tid >> 6;
    if (lane == 0) redd[8 + wv] = tm_all;
    __syncthreads();
    double m = redd[8];
    for (int i = 1; i < RC_BLOCK / 64; ++i) m = fmax(m, redd[8 + i]);
    tm_all = m;
    __syncthreads();
  }
  // the reference divides the estimate by its own max when the TRUTH's max is nonzero
  const bool tnorm = tm_all != 0.0;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * RC_BLOCK;
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
      for (int e = tid; e < pp; e += RC_BLOCK) {
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
      gp_inverse(Aug, p, redd, redi);
      if (side == 0) {
#pragma unroll
        for (int u = 0; u < GP_NR; ++u) {
          const int e = tid + u * RC_BLOCK;
          if (e < pp) {
            const int i = e / p, j = e - i * p;
            sreg[u] = Aug[i * 2 * p + p + j];
          }
        }
        __syncthreads();
      } else {
        double acc = 0.;
#pragma unroll
        for (int u = 0; u < GP_NR; ++u) {
          const int e = tid + u * RC_BLOCK;
          if (e < pp) {
            const int i = e / p, j = e - i * p;
            const double df = sqrt(sreg[u]) - sqrt(Aug[i * 2 * p + p + j]);
            acc += df * df;
          }
        }
        const double d = sqrt(rc_block_sum_d(acc, redd));
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
  double* Tk = Aug;
  double* Tn = Aug + pp;
  double sa1[GP_NR], sa2[GP_NR];
  for (int e = tid; e < pp; e += RC_BLOCK) {
    Tk[e] = T[e];
    Ek[e] = Ex[e];
  }
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * RC_BLOCK;
    const int i = e / p, j = e - i * p;
    sa1[u] = (e < pp && i == j) ? 1.0 : 0.0;
    sa2[u] = sa1[u];
  }
  __syncthreads();
  for (int k = 1; k < p; ++k) {
    if (k > 1) {  // A^k = A^(k-1) A
      for (int e = tid; e < pp; e += RC_BLOCK) {
        const int i = e / p, j = e - i * p;
        double a = 0.;
        float b = 0.f;
        for (int m = 0; m < p; ++m) {
          a += Tk[i * p + m] * T[m * p + j];
          b += Ek[i * p + m] * Ex[m * p + j];
        }
        Tn[e] = a;
        En[e] = b;
      }
      __syncthreads();
      for (int e = tid; e < pp; e += RC_BLOCK) {
        Tk[e] = Tn[e];
        Ek[e] = En[e];
      }
      __syncthreads();
    }
    const double ck = eps_pow[k];
    const float ckf = (float)ck;
    double se = 0.;
#pragma unroll
    for (int u = 0; u < GP_NR; ++u) {
      const int e = tid + u * RC_BLOCK;
      if (e < pp) {
        const double tk = Tk[e];
        const float ek = Ek[e];
        sa1[u] = sa1[u] + ck * tk;
        sa2[u] = sa2[u] + (double)(ckf * ek);
        const double df = tk - (double)ek;
        se += df * df;
      }
    }
    se = rc_block_sum_d(se, redd);
    if (tid == 0) o[6 + k] = se / (double)pp;
  }
  double acc = 0.;
#pragma unroll
  for (int u = 0; u < GP_NR; ++u) {
    const int e = tid + u * RC_BLOCK;
    if (e < pp) {
      const double df = sqrt(sa1[u]) - sqrt(sa2[u]);
      acc += df * df;
    }
  }
  const double dd = sqrt(rc_block_sum_d(acc, redd));
  if (tid == 0) o[6] = 1.0 / (1.0 + dd);
}

}  // namespace

extern "C" int redcliff_gc_progress(int32_t S, int32_t nE, int32_t G, int32_t p, int32_t Lt, const float* est,
                                    const double* truth, const double* eps_pow, double in_degree_coeff,
                                    double out_degree_coeff, double* out, void* stream) {
  if (S < 0 || G < 0 || nE < G || p < 2 || p > 64 || Lt < 1 || Lt > 128 || (S * G > 0 && (!est || !truth || !eps_pow || !out))) {
    rc_set_error("gc_progress: bad arguments (S=%d nE=%d G=%d p=%d Lt=%d; need 2 <= p <= 64, Lt <= 128, G <= nE)", S, nE,
                 G, p, Lt);
    return REDCLIFF_EINVAL;
  }
  if (S * G == 0) return 0;
  const size_t lds = (size_t)36 * p * p;
  if (lds > 64 * 1024) {
    const int e = rc_check(hipFuncSetAttribute(reinterpret_cast<const void*>(k_gc_progress),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                           "k_gc_progress LDS");
    if (e) return e;
  }
  hipLaunchKernelGGL(k_gc_progress, dim3(S * G), dim3(RC_BLOCK), lds, (hipStream_t)stream, S, nE, G, p, Lt, est, truth,
                     eps_pow, in_degree_coeff, out_degree_coeff, out);
  return rc_check(hipGetLastError(), "k_gc_progress");
}
