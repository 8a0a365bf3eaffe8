// rc_aux.hip -- cMLP group norms (GC extraction) and proximal steps on gfx950.
//
// Reference: models/cmlp.py:147-167 (cMLP.GC: ||W0[:, c, t]|| over hidden units, or over
// hidden units and lags) and models/cmlp.py:117-144 (perform_prox_update_on_GC_weights:
// GL / GSGL / H shrinkage with threshold lr*lam).  One workgroup per (factor, network).
#include "rc_common.h"

namespace {

// One WAVE per (factor, network) of a replica (four per workgroup): G[e] = ||W0[:, e]|| over the
// h hidden units (e = c * L + t) and G0[c] = the norm over hidden units and lags.  Lane l owns
// the outputs o = l + 64 k (o < Q: G columns, Q <= o < Q + p: G0 channels) and sums them in
// ascending (u[, t]) fmaf order straight from global memory (the G lanes' rows are one
// coalesced 4 Q-byte read per hidden unit; the G0 lanes re-read the same lines from cache).
// Short waves are dispatch-bound at a packed grid's size: a 256-thread workgroup per network
// (20,480 waves at R = 128 D4IC) ran 83-94 us, a quarter of the waves is the lever.
#define GN_WPG (RC_BLOCK / 64)
__global__ __launch_bounds__(RC_BLOCK) void k_gc_norms(RedcliffDims d, const float* fac, int64_t fs, FacOff fo,
                                                       float* G, float* G0) {
  const int r = blockIdx.y, lane = threadIdx.x & 63;
  const int kj = blockIdx.x * GN_WPG + (threadIdx.x >> 6);
  const int p = d.p, h = d.h, L = d.L, Q = p * L, nout = Q + p;
  if (kj >= d.K * p) return;
  const float* W = fac + r * fs + fo.W0 + (int64_t)kj * h * Q;
  float* Gr = G + ((int64_t)r * d.K * p + kj) * Q;
  float* G0r = G0 + ((int64_t)r * d.K * p + kj) * p;
  for (int o = lane; o < nout; o += 64) {
    float a = 0.f;
    if (o < Q) {
#pragma unroll 10
      for (int u = 0; u < h; ++u) {
        const float x = W[(int64_t)u * Q + o];
        a += x * x;
      }
      Gr[o] = sqrtf(a);
    } else {
      const float* wr = W + (o - Q) * L;
      for (int u = 0; u < h; ++u) {
#pragma unroll 4
        for (int t = 0; t < L; ++t) {
          const float x = wr[(int64_t)u * Q + t];
          a += x * x;
        }
      }
      G0r[o - Q] = sqrtf(a);
    }
  }
}

// W <- W / max(norm, thr) * max(norm - thr, 0) on the groups of one input channel.
__global__ __launch_bounds__(RC_BLOCK) void k_prox(RedcliffDims d, float* fac, int64_t fs, FacOff fo, float lam,
                                                   float lr, int penalty) {
  const int r = blockIdx.y, kj = blockIdx.x;
  const int p = d.p, h = d.h, L = d.L, Q = p * L;
  float* W = fac + r * fs + fo.W0 + (int64_t)kj * h * Q;
  const float thr = lr * lam;
  // one thread per input channel c (p <= 64): the groups never straddle channels
  const int cc = threadIdx.x;
  if (cc >= p) return;
  auto shrink = [&](int t0, int t1) {
    float s = 0.f;
    for (int u = 0; u < h; ++u)
      for (int t = t0; t < t1; ++t) s += W[(int64_t)u * Q + cc * L + t] * W[(int64_t)u * Q + cc * L + t];
    const float nrm = sqrtf(s);
    const float den = fmaxf(nrm, thr), num = fmaxf(nrm - thr, 0.f);
    for (int u = 0; u < h; ++u)
      for (int t = t0; t < t1; ++t) {
        const int64_t i = (int64_t)u * Q + cc * L + t;
        W[i] = (W[i] / den) * num;
      }
  };
  if (penalty == 0) {  // GL: one group per input channel (norm over hidden units and lags)
    shrink(0, L);
  } else if (penalty == 1) {  // GSGL: per (channel, lag) groups, then per channel
    for (int t = 0; t < L; ++t) shrink(t, t + 1);
    shrink(0, L);
  } else {  // H: nested prefixes of the lag axis, lowest index = most lagged (cmlp.py:138-141)
    for (int i = 0; i < L; ++i) shrink(0, i + 1);
  }
}

// Adam from a gradient buffer (data-parallel step, after the all-reduce).  grid (ceil(n/1024), R),
// 4 elements per thread, float4 loads when the rows are 16-byte aligned.
__global__ __launch_bounds__(RC_BLOCK) void k_adam_apply(float* P, float* M, float* V, const float* G, int64_t n,
                                                         int64_t stride, const RedcliffReplicaHyper* hyp, int group,
                                                         int t) {
  const int r = blockIdx.y;
  const RcAdamScalars s = rc_adam_scalars(group == 0 ? hyp[r].A : hyp[r].B, t);
  const int64_t off = (int64_t)r * stride;
  const int64_t i0 = ((int64_t)blockIdx.x * RC_BLOCK + threadIdx.x) * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = i0 + k;
    if (i >= n) break;
    float pp = P[off + i], mm = M[off + i], vv = V[off + i];
    rc_adam(pp, mm, vv, G[off + i], s);
    P[off + i] = pp; M[off + i] = mm; V[off + i] = vv;
  }
}

}  // namespace

extern "C" int redcliff_adam_apply(const RedcliffDims* d, float* params, float* exp_avg, float* exp_avg_sq,
                                   const float* grad, int64_t n, int64_t stride, const RedcliffReplicaHyper* hyper,
                                   int32_t group, int32_t t, void* stream) {
  if (!d || !params || !exp_avg || !exp_avg_sq || !grad || !hyper || n < 0 || t < 1 || (group != 0 && group != 1)) {
    rc_set_error("adam_apply: bad arguments");
    return REDCLIFF_EINVAL;
  }
  if (n == 0) return 0;
  const int64_t nb = (n + 4 * RC_BLOCK - 1) / (4 * RC_BLOCK);
  hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)nb, d->R), dim3(RC_BLOCK), 0, (hipStream_t)stream, params, exp_avg,
                     exp_avg_sq, grad, n, stride, hyper, group, t);
  return rc_check(hipGetLastError(), "k_adam_apply");
}

extern "C" int redcliff_gc_norms(const RedcliffDims* d, const float* fac, int64_t fac_stride, float* G, float* G0,
                                 void* stream) {
  if (!d || !fac || !G || !G0) { rc_set_error("gc_norms: null argument"); return REDCLIFF_EINVAL; }
  if (d->p > 64 || d->h > 4096) { rc_set_error("gc_norms: p > 64 or h > 4096"); return REDCLIFF_ELIMIT; }
  const int nwg = (d->K * d->p + GN_WPG - 1) / GN_WPG;
  hipLaunchKernelGGL(k_gc_norms, dim3(nwg, d->R), dim3(RC_BLOCK), 0, (hipStream_t)stream, *d, fac, fac_stride,
                     rc_fac_off(*d), G, G0);
  return rc_check(hipGetLastError(), "k_gc_norms");
}

extern "C" int redcliff_prox(const RedcliffDims* d, float* fac, int64_t fac_stride, float lam, float lr,
                             int32_t penalty, void* stream) {
  if (!d || !fac) { rc_set_error("prox: null argument"); return REDCLIFF_EINVAL; }
  if (penalty < 0 || penalty > 2) { rc_set_error("unsupported penalty %d", penalty); return REDCLIFF_EINVAL; }
  if (d->p > RC_BLOCK) { rc_set_error("prox: p > %d", RC_BLOCK); return REDCLIFF_ELIMIT; }
  hipLaunchKernelGGL(k_prox, dim3(d->K * d->p, d->R), dim3(RC_BLOCK), 0, (hipStream_t)stream, *d, fac, fac_stride,
                     rc_fac_off(*d), lam, lr, penalty);
  return rc_check(hipGetLastError(), "k_prox");
}
