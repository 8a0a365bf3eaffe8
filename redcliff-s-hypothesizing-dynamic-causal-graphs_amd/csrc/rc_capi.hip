// rc_capi.hip -- extern "C" entry points of libredcliff_hip.so (see include/redcliff_hip.h).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rc_common.h"

// ---- optional per-kernel HIP-event timing (bench / profiling only) -------------------------
namespace {
enum { KT_SUPPORTS = 0, KT_EMB_FWD, KT_FAC_FWD, KT_FAC_BWD, KT_EMB_BWD, KT_EMB_FINAL, KT_FAC_MIX, KT_EMB_COMB, KT_FAC_LEAD, KT_N };
struct TimedLaunch {
  int id;
  hipEvent_t a, b;
};
bool g_timing = false;
std::vector<TimedLaunch> g_launches;

template <class F>
int timed(int id, hipStream_t s, F&& launch) {
  if (!g_timing) return launch();
  TimedLaunch t{id, nullptr, nullptr};
  int e = rc_check(hipEventCreate(&t.a), "hipEventCreate");
  if (!e) e = rc_check(hipEventCreate(&t.b), "hipEventCreate");
  if (!e) e = rc_check(hipEventRecord(t.a, s), "hipEventRecord");
  if (e) return e;
  e = launch();
  const int e2 = rc_check(hipEventRecord(t.b, s), "hipEventRecord");
  g_launches.push_back(t);
  return e ? e : e2;
}
}  // namespace

// Second stream for the factor chain when the step splits into two independent kernel chains
// (GEMM-shaped embedder and / or matrix-core factor path), joined back into the caller's
// stream with events: per host thread and device, created on first use.
namespace {
struct AuxStream {
  hipStream_t s = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
};
thread_local AuxStream g_aux[16];

int aux_stream(AuxStream** out) {
  int dev = 0;
  int e = rc_check(hipGetDevice(&dev), "hipGetDevice");
  if (e) return e;
  if (dev < 0 || dev >= 16) { rc_set_error("device %d outside the auxiliary-stream table", dev); return REDCLIFF_ELIMIT; }
  AuxStream& a = g_aux[dev];
  if (!a.s) {
    // normal priority (round 3): a low- or high-priority stream needs a hardware queue of its
    // own class, and once RCCL's streams hold the process's queues (a torch.distributed "nccl"
    // group) a forked step on such a stream ran 3.5x slower (C1(K=4): 100 -> 353 us per step,
    // profiles/r03_dp_profile_c1k4_*.log); without RCCL normal and low measure the same (C1(K=4)
    // 1.29 M windows/s both, C5 288 K vs 281 K)
    const char* pv = getenv("REDCLIFF_AUX_PRIO");  // tuning knob: low | normal (default) | high
    if (!pv || (strcmp(pv, "low") && strcmp(pv, "high"))) {
      e = rc_check(hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
    } else {
      int least = 0, greatest = 0;
      e = rc_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
      const int prio = !strcmp(pv, "high") ? greatest : least;
      if (!e) e = rc_check(hipStreamCreateWithPriority(&a.s, hipStreamNonBlocking, prio), "hipStreamCreateWithPriority");
    }
    // fork / join events order work between two streams of ONE device: no system-scope fence on
    // their record (the host never inspects them; C1(K=4) 0.0905-0.0910 -> 0.0891-0.0896 ms per
    // step, TST unchanged).  REDCLIFF_EVENT_SCOPE=device | system (tuning knob)
    const char* ev = getenv("REDCLIFF_EVENT_SCOPE");
    unsigned ef = hipEventDisableTiming;
    if (!ev || !strcmp(ev, "nofence")) ef |= hipEventDisableSystemFence;
    else if (!strcmp(ev, "device")) ef |= hipEventReleaseToDevice;
    for (int i = 0; i < 3 && !e; ++i) e = rc_check(hipEventCreateWithFlags(&a.ev[i], ef), "hipEventCreate");
    if (e) return e;
  }
  *out = &a;
  return 0;
}

// `to` waits for everything enqueued on `from` so far
int stream_wait(hipStream_t to, hipStream_t from, hipEvent_t ev) {
  if (to == from) return 0;  // single-stream step (REDCLIFF_FORK=0)
  int e = rc_check(hipEventRecord(ev, from), "hipEventRecord");
  return e ? e : rc_check(hipStreamWaitEvent(to, ev, 0), "hipStreamWaitEvent");
}
}  // namespace

static thread_local char g_err[512] = "";
int rc_ws_guard_floats = 0;

void rc_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int rc_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  rc_set_error("%s: %s", what, hipGetErrorString(e));
  return (int)e;
}

size_t rc_emb_bwd_lds(const RedcliffDims& d, bool late);

// Shape limits of the kernels (LDS tiles, register-blocked accumulators).
static int check_dims(const RedcliffDims* d) {
  if (!d) { rc_set_error("null dims"); return REDCLIFF_EINVAL; }
  if (d->R < 1 || d->Bmax < 1 || d->p < 1 || d->L < 1 || d->K < 1 || d->h < 1 || d->F < 1 || d->n < 1 || d->H < 1 ||
      d->M1 < 1 || d->nsup < 0 || d->nsup > d->K || d->T < 1) {
    rc_set_error("invalid dims (R=%d Bmax=%d p=%d L=%d K=%d h=%d F=%d n=%d H=%d M1=%d nsup=%d T=%d)", d->R, d->Bmax,
                 d->p, d->L, d->K, d->h, d->F, d->n, d->H, d->M1, d->nsup, d->T);
    return REDCLIFF_EINVAL;
  }
  const int Lmax = rc_lmax(*d);
  if (d->T < Lmax) { rc_set_error("T=%d shorter than max(gen_lag, embed_lag)=%d", d->T, Lmax); return REDCLIFF_EINVAL; }
  if (d->p > 64 || d->K > 16 || d->h > 128 || d->F > 64 || d->n > 4 || d->M1 > 64 || d->Bmax > 512 ||
      d->p * d->H > 32 * RC_BLOCK || d->M1 * d->H > 32 * RC_BLOCK || d->F * d->H > 32 * RC_BLOCK || d->L > 64) {
    rc_set_error("dims outside kernel limits (p<=64 K<=16 h<=128 F<=64 n<=4 M1<=64 Bmax<=512 p*H,M1*H,F*H<=8192)");
    return REDCLIFF_ELIMIT;
  }
  if (d->F < d->L) {
    rc_set_error("fused path needs embed_lag >= gen_lag (forward and GC embedder windows coincide)");
    return REDCLIFF_ELIMIT;
  }
  if (rc_emb_bwd_lds(*d, false) > RC_LDS_MAX_FLOATS * sizeof(float)) {
    rc_set_error("embedder backward LDS budget exceeded for Bmax*K=%d", d->Bmax * d->K);
    return REDCLIFF_ELIMIT;
  }
  return 0;
}

extern "C" {

int redcliff_abi_version(void) { return REDCLIFF_ABI_VERSION; }

#ifndef REDCLIFF_BUILD_ID
#define REDCLIFF_BUILD_ID "unknown"
#endif
// build.py reads the id back from the file bytes (after the tag) without loading the library
__attribute__((used)) static const char kBuildTag[] = "REDCLIFF_BUILD_ID=" REDCLIFF_BUILD_ID;

const char* redcliff_build_id(void) { return kBuildTag + sizeof("REDCLIFF_BUILD_ID=") - 1; }

const char* redcliff_last_error(void) { return g_err; }

size_t redcliff_workspace_bytes(const RedcliffDims* d) {
  if (check_dims(d) != 0) return 0;
  return sizeof(float) * (size_t)rc_ws_off(*d).total * (size_t)d->R;
}

size_t redcliff_emb_param_count(const RedcliffDims* d) { return d ? (size_t)rc_emb_off(*d).total : 0; }
size_t redcliff_fac_param_count(const RedcliffDims* d) { return d ? (size_t)rc_fac_off(*d).total : 0; }

// Offsets (floats, per replica) of the workspace regions the host reads back:
// out[0..] = T R f1 w a y G G0 dwp dAadj dWi dS dgb S dZ amat lossp xsim gfc total
int redcliff_workspace_layout(const RedcliffDims* d, int64_t* out, int32_t n_out) {
  if (check_dims(d) != 0) return REDCLIFF_EINVAL;
  const WsOff o = rc_ws_off(*d);
  const int64_t v[] = {o.T, o.R, o.f1, o.w, o.a, o.y, o.G, o.G0, o.w1, o.gq, o.ebp, o.ecnt, o.gfc1, o.dwp, o.dAadj, o.dWi, o.dS, o.dgb, o.S, o.dZ,
                       o.amat, o.lossp, o.xsim, o.gfc, o.xw, o.dyl, o.dgs, o.errw, o.total};
  const int nv = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n_out && i < nv; ++i) out[i] = v[i];
  return nv;
}

int redcliff_device_status(const RedcliffDims* d, void* ws, uint32_t* out, void* stream) {
  if (check_dims(d) != 0 || !ws || !out) { rc_set_error("device_status: bad arguments"); return REDCLIFF_EINVAL; }
  const WsOff o = rc_ws_off(*d);
  hipStream_t s = (hipStream_t)stream;
  const size_t pitch = sizeof(float) * (size_t)o.total;
  char* base = (char*)ws + sizeof(float) * (size_t)o.errw;
  int e = rc_check(hipMemcpy2DAsync(out, sizeof(uint32_t), base, pitch, sizeof(uint32_t), (size_t)d->R,
                                    hipMemcpyDeviceToHost, s), "device_status copy");
  if (!e) e = rc_check(hipMemset2DAsync(base, pitch, 0, sizeof(uint32_t), (size_t)d->R, s), "device_status clear");
  if (!e) e = rc_check(hipStreamSynchronize(s), "device_status sync");
  if (e) return e;
  int bad = 0;
  for (int r = 0; r < d->R; ++r) bad += out[r] != 0;
  return bad;
}

// Verification mode: guard bands of `floats` floats after every workspace region (0 = off,
// the production layout).  Affects workspaces sized / laid out after the call.  Returns the
// previous setting.
int redcliff_debug_guard_bands(int32_t floats) {
  const int prev = rc_ws_guard_floats;
  rc_ws_guard_floats = floats < 0 ? 0 : (floats > 4096 ? 4096 : floats);
  return prev;
}

// (start, size) in floats of every region of one replica's workspace slice, in layout order;
// with guard bands on, region i's band is [start + size, start + size + guard).  Returns the
// number of regions.
int redcliff_workspace_regions(const RedcliffDims* d, int64_t* out, int32_t n_pairs) {
  if (check_dims(d) != 0) return REDCLIFF_EINVAL;
  int64_t ext[2 * RC_WS_MAX_REGIONS];
  int nr = 0;
  rc_ws_off(*d, ext, &nr);
  for (int i = 0; i < nr && i < n_pairs; ++i) {
    out[2 * i] = ext[2 * i];
    out[2 * i + 1] = ext[2 * i + 1];
  }
  return nr;
}

int redcliff_bn_batch_stats(const RedcliffDims* d, const float* X, int64_t x_rstride, int64_t N, int32_t B,
                            double* stats, int64_t stats_rstride, void* stream) {
  int e = check_dims(d);
  if (e) return e;
  if (!X || !stats || N < 1 || B < 1) { rc_set_error("bn_batch_stats: bad arguments"); return REDCLIFF_EINVAL; }
  return rc_launch_bn_stats(*d, X, x_rstride, N, B, stats, stats_rstride, (hipStream_t)stream);
}

int redcliff_dgcnn_supports(const RedcliffDims* d, const float* emb, int64_t emb_stride, void* ws, void* stream) {
  int e = check_dims(d);
  if (e) return e;
  const WsOff wo = rc_ws_off(*d);
  return rc_launch_supports(*d, emb, emb_stride, (float*)ws, wo.total, rc_emb_off(*d), wo, (hipStream_t)stream);
}

static int make_ctx(const RedcliffStepArgs* a, StepCtx& c) {
  int e = check_dims(&a->d);
  if (e) return e;
  const RedcliffDims& d = a->d;
  if (a->B < 1 || a->B > d.Bmax) { rc_set_error("batch %d outside [1, Bmax=%d]", a->B, d.Bmax); return REDCLIFF_EINVAL; }
  if (!a->X || !a->emb || !a->fac || !a->hyper || !a->ws || !a->bn_rm || !a->bn_rv) {
    rc_set_error("null buffer in step arguments");
    return REDCLIFF_EINVAL;
  }
  const WsOff wo = rc_ws_off(d);
  if (a->ws_bytes < sizeof(float) * (size_t)wo.total * (size_t)d.R) {
    rc_set_error("workspace too small: %zu < %zu", a->ws_bytes, sizeof(float) * (size_t)wo.total * (size_t)d.R);
    return REDCLIFF_EWORKSPACE;
  }
  if ((a->flags & (RC_LOSS_FORECAST | RC_VALUES)) && d.T < rc_lmax(d) + 1) {
    rc_set_error("forecast loss needs T > max(gen_lag, embed_lag)");
    return REDCLIFF_EINVAL;
  }
  if ((a->flags & RC_BN_TRAIN) && !a->bn_stats) { rc_set_error("train-mode BatchNorm needs bn_stats"); return REDCLIFF_EINVAL; }
  if ((a->flags & (RC_LOSS_FACTOR | RC_CONFUSION)) && d.nsup > 0 && !a->labels) {
    rc_set_error("factor-score loss needs labels");
    return REDCLIFF_EINVAL;
  }
  if ((a->flags & RC_VALUES) && !a->acc) { rc_set_error("RC_VALUES needs acc"); return REDCLIFF_EINVAL; }
  if ((a->flags & RC_CONFUSION) && d.nsup > 0 && !a->confusion) { rc_set_error("RC_CONFUSION needs confusion"); return REDCLIFF_EINVAL; }
  const bool grad_only = a->flags & RC_GRAD_ONLY;
  if ((a->flags & (RC_STEP_A | RC_STEP_B)) && !grad_only && (!a->emb_m || !a->emb_v || !a->fac_m || !a->fac_v)) {
    rc_set_error("optimizer state missing");
    return REDCLIFF_EINVAL;
  }
  if (grad_only && (((a->flags & RC_STEP_A) && !a->grad_emb) || ((a->flags & RC_STEP_B) && !a->grad_fac))) {
    rc_set_error("RC_GRAD_ONLY needs grad_emb / grad_fac for the stepped groups");
    return REDCLIFF_EINVAL;
  }
  if (a->B_global != 0 && a->B_global < a->B) {
    rc_set_error("B_global=%d smaller than the shard B=%d", a->B_global, a->B);
    return REDCLIFF_EINVAL;
  }
  memset(&c, 0, sizeof(c));
  if (a->replicas) {
    if (a->n_replicas < 0 || a->n_replicas > RC_MAX_ACTIVE || a->n_replicas > d.R) {
      rc_set_error("active replica list of %d entries (at most min(R=%d, %d))", a->n_replicas, d.R, RC_MAX_ACTIVE);
      return REDCLIFF_ELIMIT;
    }
    for (int i = 0; i < a->n_replicas; ++i) {
      const int r = a->replicas[i];
      if (r < 0 || r >= d.R || (i > 0 && r <= a->replicas[i - 1])) {
        rc_set_error("active replica list must be strictly increasing indices < R=%d (entry %d = %d)", d.R, i, r);
        return REDCLIFF_EINVAL;
      }
      c.rmap[i] = (uint8_t)r;
    }
    c.nrep = a->n_replicas;
    c.rident = 0;
  } else {
    c.nrep = d.R;
    c.rident = 1;
  }
  c.d = d;
  c.B = a->B;
  c.Bg = a->B_global ? a->B_global : a->B;
  c.gE = a->grad_emb;
  c.gF = a->grad_fac;
  c.Lmax = rc_lmax(d);
  c.Ls = rc_ls(d);
  c.flags = a->flags;
  c.nbn = a->n_bn_updates;
  c.defer = 0;
  c.tA = a->tA;
  c.tB = a->tB;
  c.X = a->X; c.xr = a->x_rstride; c.row0 = a->row0;
  c.lab = a->labels; c.labr = a->lab_rstride;
  c.bns = a->bn_stats; c.bnsr = a->bn_stats_rstride;
  c.emb = a->emb; c.embM = a->emb_m; c.embV = a->emb_v; c.es = a->emb_stride;
  c.fac = a->fac; c.facM = a->fac_m; c.facV = a->fac_v; c.fs = a->fac_stride;
  c.rm = a->bn_rm; c.rv = a->bn_rv;
  c.hyp = a->hyper;
  c.ws = (float*)a->ws; c.wss = wo.total;
  c.acc = a->acc;
  c.conf = a->confusion;
  c.eo = rc_emb_off(d);
  c.fo = rc_fac_off(d);
  c.wo = wo;
  rc_emb_partial_layout(c, rc_emb_use_gemm(d));
  c.fslots = rc_fac_slots(d);
  rc_ctx_magics(c);
  return 0;
}

int redcliff_train_step(const RedcliffStepArgs* a, void* stream) {
  if (!a) { rc_set_error("null step arguments"); return REDCLIFF_EINVAL; }
  StepCtx c;
  int e = make_ctx(a, c);
  if (e) return e;
  if (c.nrep == 0) return 0;  // every replica of the pack has stopped
  static const bool wait_dbg = [] {
    const char* v = getenv("REDCLIFF_DEBUG_WAIT_TIMEOUT");
    return v && strcmp(v, "0") != 0;
  }();
  c.wait_dbg = wait_dbg;
  hipStream_t s = (hipStream_t)stream;
  const int fl = a->flags;
  const bool emb_grad = fl & RC_STEP_A;
  const bool fac = (fl & (RC_STEP_B | RC_VALUES | RC_STORE_OUTPUTS)) || (emb_grad && (fl & (RC_LOSS_FORECAST | RC_LOSS_ADJ)));
  if (fl & RC_REFRESH_SUPPORTS) {
    if ((e = timed(KT_SUPPORTS, s, [&] { return rc_launch_supports(c.d, c.emb, c.es, c.ws, c.wss, c.eo, c.wo, s); })))
      return e;
  }
  const bool mfma = fac && rc_fac_use_mfma(c.d);
  const bool egemm = rc_emb_use_gemm(c.d);
  // Two chains when either side is a multi-kernel chain -- stream s: embedder forward, mixing
  // (needs w and the factor forward), embedder backward and optimizer; stream sf: factor
  // forward, then (after the mixing) dW0 + Adam, which overlaps the embedder backward; joined
  // at the end.  Otherwise everything runs on s.
  const bool fork = fac && (egemm || mfma);
  static AuxStream none;  // single-stream step: null events, stream_wait(s, s) is a no-op
  AuxStream* aux = &none;
  hipStream_t sf = s;
  // A single fit is latency-bound: the factor chain on a second stream fills idle CUs (C5 201K ->
  // 233K windows/s).  Packs of 32 or more replicas gain as well since round 4 (the chains' launch
  // tails and short kernels -- head, k_emb_final, supports -- overlap the other chain's work:
  // D4IC R = 32 / 64 / 128 0.282 / 0.444 / 0.774 -> 0.267 / 0.421 / 0.732 ms per step,
  // profiles/r04_grid_fork_sweep.log); at R = 8 one stream stays ahead (0.160 vs 0.161).  Forked
  // and single-stream steps give the same bits (tests/test_gpu_forked.py); the intermittent A
  // mismatch once blamed on the fork was a missing barrier in k_emb_final's adjacency
  // workgroup, which concurrent work only made likelier.  REDCLIFF_FORK=0 / 1 overrides (tuning).
  const char* fv = getenv("REDCLIFF_FORK");
  const bool two = fv ? strcmp(fv, "0") != 0 : (c.d.R == 1 || c.nrep >= 32);
  if (fork && two) {
    if ((e = aux_stream(&aux))) return e;
    sf = aux->s;
    if ((e = stream_wait(sf, s, aux->ev[0]))) return e;
  }
  // Merged backward (vector factor path + fused embedder, one stream, training without loss
  // values): factor and embedder backward in one launch, the embedder workgroups waiting only
  // for the factor-lead workgroups' dL/dw / dL/dA records (k_bwd_merged), when its grid fits the
  // chip at once (rc_bwd_merged_grid: D4IC 0.097 -> 0.083 ms per step).  REDCLIFF_MERGE=0 / 1
  // forces the two launches / the merged one (same bits).
  const char* mv = getenv("REDCLIFF_MERGE");
  const char* dv0 = getenv("REDCLIFF_DEFER");
  const bool merged = fac && !mfma && !fork && !egemm && emb_grad && !(fl & RC_VALUES) && !(dv0 && strcmp(dv0, "1") != 0) &&
                      (mv ? strcmp(mv, "0") != 0 : rc_bwd_merged_grid(c) > 0);
  // Split lead (vector factor path when the merged launch does not fit, e.g. TST: K*p = 108
  // networks): the K*p lead workgroups' records (dL/dw, dL/dA, group norms) are all the embedder
  // backward needs, and the factor update needs only the forward, so the records get their own
  // short launch on s and the update runs on the second stream beside the embedder backward,
  // joined before k_emb_final (which rewrites A, an operand of the update).  Same workgroup
  // arithmetic as the one launch, so the same bits (tests/test_gpu_forked.py).  Default: single
  // fits (a pack fills the chip) whose update grid leaves at least half of the CUs to the
  // embedder backward (C1(K=4): 80 update workgroups, 1.23 -> 1.30 M windows/s; TST: 216, the
  // embedder backward is slowed by more than the split saves, 1.07 -> 1.01 M).
  // REDCLIFF_SPLIT_LEAD=0 / 1 overrides.
  // Not for data-parallel shard steps (RC_GRAD_ONLY): their process holds an RCCL communicator, and
  // with one the second stream runs serialised behind the first -- the split step is then slower
  // than one launch (C1(K=4): 0.104 -> 0.132 ms, profiles/r04_ns_probe.log).
  const char* slv = getenv("REDCLIFF_SPLIT_LEAD");
  const bool split_ok = !mfma && fac && !merged && !fork && emb_grad && (fl & RC_STEP_B) && !(fl & RC_GRAD_ONLY);
  const bool split = split_ok && (slv ? strcmp(slv, "0") != 0
                                      : c.d.R == 1 && 2 * rc_fac_bwd_grid(c) <= rc_cu_count());
  // In a split-lead step the forward and the factor update complete the fork / join events
  // themselves (hipExtLaunchKernel stop events) instead of an event-record packet on the stream
  // after them: C1(K=4) 0.0892-0.0898 -> 0.0872-0.0874 ms per step, TST unchanged, the same bits
  // (tests/test_gpu_forked.py).  REDCLIFF_EXT_EVENT=0 records the events as packets (read per step).
  const char* xev = getenv("REDCLIFF_EXT_EVENT");
  const bool ext_ev = !xev || strcmp(xev, "0") != 0;
  if (split && ext_ev && (e = aux_stream(&aux))) return e;
  // forward: the fused launch runs the embedder and (vector path, no fork) the factor networks
  if (egemm) {
    if ((e = timed(KT_EMB_FWD, s, [&] { return rc_launch_emb_fwd_gemm(c, s); }))) return e;
  } else if ((e = timed(KT_EMB_FWD, s, [&] {
               return rc_launch_forward(c, s, true, fac && !mfma && !fork, split && ext_ev ? aux->ev[1] : nullptr);
             }))) {
    return e;
  }
  if (mfma) {
    if ((e = timed(KT_FAC_FWD, sf, [&] { return rc_launch_fac_fwd_mfma(c, sf); }))) return e;
  } else if (fork) {
    if ((e = timed(KT_FAC_FWD, sf, [&] { return rc_launch_forward(c, sf, false, true); }))) return e;
  }
  if (mfma) {
    if ((e = stream_wait(s, sf, aux->ev[1]))) return e;  // the mixing needs the factor forward
    if ((e = timed(KT_FAC_MIX, s, [&] { return rc_launch_fac_mix(c, s); }))) return e;
    if ((e = stream_wait(sf, s, aux->ev[0]))) return e;  // dW0 needs the mixing's dL/dy
    if ((e = timed(KT_FAC_BWD, sf, [&] { return rc_launch_fac_dw0(c, sf); }))) return e;
  }
  if (split) {
    if ((e = aux_stream(&aux))) return e;
    sf = aux->s;
    if (ext_ev) {  // the forward completed ev[1] itself
      if ((e = rc_check(hipStreamWaitEvent(sf, aux->ev[1], 0), "hipStreamWaitEvent"))) return e;
    } else if ((e = stream_wait(sf, s, aux->ev[1]))) {  // the update needs the forward
      return e;
    }
    if ((e = timed(KT_FAC_BWD, sf, [&] { return rc_launch_fac_bwd(c, sf, RC_FB_UPDATE, ext_ev ? aux->ev[0] : nullptr); })))
      return e;
    if ((e = timed(KT_FAC_LEAD, s, [&] { return rc_launch_fac_bwd(c, s, RC_FB_RECORDS); }))) return e;
  } else if (!mfma && fac && !merged) {
    if (fork && (e = stream_wait(sf, s, aux->ev[1]))) return e;  // the mixing needs the embedder output w
    if ((e = timed(KT_FAC_BWD, sf, [&] { return rc_launch_fac_bwd(c, sf, RC_FB_ALL); }))) return e;
    if (fork && (e = stream_wait(s, sf, aux->ev[0]))) return e;
  }
  if ((fl & RC_VALUES) && (e = rc_launch_cos_values(c, s))) return e;  // before the head workgroup
  // k_emb_combine + k_emb_final as one launch (k_emb_tail) when its grid is resident: the
  // adjacency chain starts with the combine instead of after it, and one kernel boundary goes.
  // REDCLIFF_TAIL=0 keeps the two launches.
  const char* tlv = getenv("REDCLIFF_TAIL");
  bool tail = false;
  auto tail_ok = [&]() {
    return !egemm && emb_grad && c.defer == 1 && !(fl & RC_VALUES) && !(tlv && strcmp(tlv, "0") == 0) &&
           rc_emb_tail_grid(c) > 0;
  };
  if (emb_grad && egemm) {
    // GEMM chain, then the fused kernel without node workgroups (head / adjacency-L1 reduce)
    if ((e = timed(KT_EMB_BWD, s, [&] {
           const int e2 = rc_launch_emb_bwd_gemm(c, s);
           return e2 ? e2 : rc_launch_emb_bwd(c, s, false);
         })))
      return e;
  } else if (merged) {
    c.defer = 1;
    if ((e = timed(KT_EMB_BWD, s, [&] { return rc_launch_bwd_merged(c, s); }))) return e;
    tail = tail_ok();
    if (!tail && (e = timed(KT_EMB_COMB, s, [&] { return rc_launch_emb_combine(c, s); }))) return e;
  } else if (emb_grad) {
    // The node blocks' window-block partials are summed by a separate k_emb_combine launch
    // instead of the in-kernel last arriver (ticket + agent-scope fences): the fences cost the
    // packed grid ~20 % (D4IC R=32 6.8M -> 8.1M windows/s).  Same sums in the same order, so
    // every variant gives the same bits (tests/test_gpu_replicas.py, tests/test_gpu_forked.py).
    // defer 2: k_emb_final reads the partials in place (same order, no combine launch) --
    // measured slower for the single fit (k_emb_final 10 -> 20.5 us: p * nbw dependent loads
    // per element on its critical path), +1 % on the R = 32 grid, so not the default.
    // REDCLIFF_DEFER=0 / 1 / 2 overrides (tuning).
    const char* dv = getenv("REDCLIFF_DEFER");
    c.defer = dv ? atoi(dv) : 1;
    if (c.defer < 0 || c.defer > 2) c.defer = 1;
    if ((e = timed(KT_EMB_BWD, s, [&] { return rc_launch_emb_bwd(c, s, true); }))) return e;
    tail = tail_ok();
    if (c.defer == 1 && !tail && (e = timed(KT_EMB_COMB, s, [&] { return rc_launch_emb_combine(c, s); }))) return e;
  } else if (fl & (RC_VALUES | RC_CONFUSION)) {
    if ((e = timed(KT_EMB_BWD, s, [&] { return rc_launch_emb_bwd(c, s, false); }))) return e;
  }
  if (split) {  // join before A changes
    if (ext_ev)
      e = rc_check(hipStreamWaitEvent(s, aux->ev[0], 0), "hipStreamWaitEvent");
    else
      e = stream_wait(s, sf, aux->ev[0]);
    if (e) return e;
  }
  if (emb_grad || c.nbn > 0) {
    if ((e = timed(KT_EMB_FINAL, s, [&] { return tail ? rc_launch_emb_tail(c, s) : rc_launch_emb_final(c, s); }))) return e;
  }
  if (fork && (e = stream_wait(s, sf, aux->ev[2]))) return e;  // join: the caller's stream sees both chains
  return 0;
}

// Data-parallel update (reference: the optimizer steps of batch_update, models/redcliff_s_cmlp_
// withStateSmoothing.py:741-759, applied to gradients summed over the ranks): the same step
// arguments the shard step ran with, after the all-reduce of grad_emb / grad_fac.
int redcliff_dp_update(const RedcliffStepArgs* a, int64_t n_emb, int64_t n_fac, void* stream) {
  if (!a) { rc_set_error("null step arguments"); return REDCLIFF_EINVAL; }
  StepCtx c;
  int e = make_ctx(a, c);
  if (e) return e;
  if (c.nrep == 0) return 0;
  const bool sa = a->flags & RC_STEP_A, sb = a->flags & RC_STEP_B;
  if ((sa && (!a->grad_emb || n_emb < (int64_t)c.d.p * c.d.p || n_emb > c.es)) || (sb && (!a->grad_fac || n_fac < 0 || n_fac > c.fs))) {
    rc_set_error("dp_update: gradient buffers / group sizes do not match the step arguments");
    return REDCLIFF_EINVAL;
  }
  if (c.eo.A + (int64_t)c.d.p * c.d.p > n_emb && sa) { rc_set_error("dp_update: A outside the embedder group"); return REDCLIFF_EINVAL; }
  if (!sa && !sb) return 0;
  return rc_launch_dp_update(c, n_emb, n_fac, (hipStream_t)stream);
}

int redcliff_train_steps(const RedcliffStepArgs* a, int32_t nsteps, const int64_t* rows, const int32_t* sizes,
                         int32_t bn_stats_step, void* stream) {
  if (!a || nsteps < 0 || (nsteps > 0 && (!rows || !sizes))) { rc_set_error("train_steps: bad arguments"); return REDCLIFF_EINVAL; }
  RedcliffStepArgs s = *a;
  for (int32_t i = 0; i < nsteps; ++i) {
    s.row0 = rows[i];
    s.B = sizes[i];
    s.flags = (i == 0) ? a->flags : (a->flags & ~RC_REFRESH_SUPPORTS);
    s.tA = a->tA + ((a->flags & RC_STEP_A) ? i : 0);
    s.tB = a->tB + ((a->flags & RC_STEP_B) ? i : 0);
    if (a->bn_stats) s.bn_stats = a->bn_stats + (int64_t)i * bn_stats_step;
    const int e = redcliff_train_step(&s, stream);
    if (e) return e;
  }
  return 0;
}

// Per-kernel timing: while enabled every launch of redcliff_train_step is bracketed by
// HIP events on its stream.  redcliff_kernel_times() waits for the recorded events,
// adds the elapsed milliseconds per kernel (ids: supports, emb_fwd, fac_fwd, fac_bwd,
// emb_bwd, emb_final, fac_mix, emb_combine, fac_lead) into total_ms[]/counts[] and clears the record.
int redcliff_kernel_timing(int32_t enable) {
  g_timing = enable != 0;
  return 0;
}

int redcliff_kernel_times(double* total_ms, int64_t* counts, int32_t n) {
  for (int i = 0; i < n; ++i) { total_ms[i] = 0.0; counts[i] = 0; }
  int err = 0;
  for (auto& t : g_launches) {
    float ms = 0.f;
    if (!err) err = rc_check(hipEventSynchronize(t.b), "kernel_times");
    if (!err) err = rc_check(hipEventElapsedTime(&ms, t.a, t.b), "kernel_times");
    if (!err && t.id < n) { total_ms[t.id] += ms; counts[t.id] += 1; }
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  g_launches.clear();
  return err ? err : KT_N;
}

}  // extern "C"
