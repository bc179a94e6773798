// Context, memory, error and timing plumbing of libgpr_hip.so.
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

int set_err(gpr_ctx* ctx, int code, const char* fmt, ...) {
  if (ctx) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return code;
}

int ensure_buf(gpr_ctx* ctx, double** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return 0;
  if (*p) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(*p));
    *p = nullptr;
    *cap = 0;
  }
  if (need == 0) need = 1;
  if (hipMalloc((void**)p, need * sizeof(double)) != hipSuccess) {
    *p = nullptr;
    return set_err(ctx, GPR_E_NOMEM, "hipMalloc of %zu bytes failed", need * sizeof(double));
  }
  *cap = need;
  return 0;
}

int ensure_winv(gpr_ctx* ctx, int n, int nb) {
  size_t nblk = (size_t)((n + nb - 1) / nb);
  return ensure_buf(ctx, &ctx->winv, &ctx->winv_cap, nblk * nb * nb);
}

// ---- timing ----------------------------------------------------------------------------
static hipEvent_t get_event(gpr_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

TimerScope::TimerScope(gpr_ctx* c, int cls, double flops) : ctx(c), on(c->timing) {
  if (!on) return;
  st = ctx->ls ? ctx->ls : ctx->stream;
  tl.cls = cls;
  tl.flops = flops;
  tl.a = get_event(ctx);
  tl.b = get_event(ctx);
  hipEventRecord(tl.a, st);
}

TimerScope::~TimerScope() {
  if (!on) return;
  hipEventRecord(tl.b, st);
  ctx->pending.push_back(tl);
}

static void drain_timing(gpr_ctx* ctx) {
  if (ctx->pending.empty()) return;
  hipStreamSynchronize(ctx->stream);
  for (auto& t : ctx->pending) {
    float ms = 0;
    hipEventElapsedTime(&ms, t.a, t.b);
    ctx->t_ms[t.cls] += ms;
    ctx->t_launches[t.cls] += 1;
    ctx->t_flops[t.cls] += t.flops;
    ctx->event_pool.push_back(t.a);
    ctx->event_pool.push_back(t.b);
  }
  ctx->pending.clear();
}

// ---- kernel description ------------------------------------------------------------------
int make_kparams(gpr_ctx* ctx, const int* kinds, int nk, const double* hp, int d, double eps,
                 KParams* kp, int* D_total) {
  if (!kinds || nk <= 0 || nk > GPR_MAX_PARTS) return set_err(ctx, GPR_E_ARG, "bad kinds/nk (%d)", nk);
  if (!hp) return set_err(ctx, GPR_E_ARG, "hp is NULL");
  if (d <= 0 || d > KMAXD) return set_err(ctx, GPR_E_UNSUP, "d=%d unsupported (1..%d)", d, KMAXD);
  memset(kp, 0, sizeof *kp);
  kp->exptab = ctx->dexptab;
  kp->d = d;
  kp->eps = eps;
  int off = 0;
  for (int i = 0; i < nk; ++i) {
    if (kinds[i] == GPR_SE) {
      if (kp->nse >= KMAXP) return set_err(ctx, GPR_E_UNSUP, "more than %d SquaredExp parts", KMAXP);
      kp->sigma[kp->nse] = hp[off];
      kp->hp_off[kp->nse] = off;
      for (int k = 0; k < d; ++k) {
        kp->l[kp->nse][k] = hp[off + 1 + k];
        kp->l2[kp->nse][k] = hp[off + 1 + k] * hp[off + 1 + k];
      }
      kp->nse++;
      off += d + 1;
    } else if (kinds[i] == GPR_WN) {
      if (!kp->has_noise) {  // findfirst(WhiteNoise) -- src/compose_covar.jl:64-68
        kp->has_noise = 1;
        kp->noise_sigma = hp[off];
        kp->noise2 = hp[off] * hp[off];
        kp->hp_off_noise = off;
      }
      off += 1;
    } else {
      return set_err(ctx, GPR_E_ARG, "unknown kernel kind %d", kinds[i]);
    }
  }
  if (kp->nse == 0) return set_err(ctx, GPR_E_ARG, "kernel needs at least one SquaredExp part");
  if (D_total) *D_total = off;
  return 0;
}

// ---- knobs ---------------------------------------------------------------------------------
// Every run-time switch of the library: a GPR_* environment variable read once by
// gpr_ctx_create, or gpr_set_knob on a live context.  Documented in include/gpr_hip.h; none of
// them changes a result beyond rounding (they pick between equivalent code paths or tune
// memory budgets).  Test-only fault injection exists only in libgpr_hip_testing.so
// (-DGPR_TESTING).
namespace {
struct Knob {
  const char* name;
  int gpr_ctx::*ip;     // an int field, or
  double gpr_ctx::*dp;  // a double field
};
const Knob kKnobs[] = {
    {"GPR_DAG", &gpr_ctx::dag_mode, nullptr},
    {"GPR_DAG_TAIL", &gpr_ctx::dag_tail, nullptr},
    {"GPR_DAG_SOLVE", &gpr_ctx::dag_solve, nullptr},
    {"GPR_DAG_GRAM", &gpr_ctx::dag_gram, nullptr},
    {"GPR_DAG_ZLAG", &gpr_ctx::dag_zlag, nullptr},
    {"GPR_FUSED_RHS", &gpr_ctx::fused_rhs, nullptr},
    {"GPR_FUSE_Y", &gpr_ctx::fuse_y, nullptr},
    {"GPR_FUSE_KINV", &gpr_ctx::fuse_kinv, nullptr},
    {"GPR_KBUILD_UPPER", &gpr_ctx::kbuild_upper, nullptr},
    {"GPR_KBUILD_EXACT", &gpr_ctx::kbuild_exact, nullptr},
    {"GPR_KBUILD_COLSTORE", &gpr_ctx::kbuild_colstore, nullptr},
    {"GPR_CV_STREAMS", &gpr_ctx::cv_streams, nullptr},
    {"GPR_CV_BATCH", &gpr_ctx::cv_batch, nullptr},
    {"GPR_CV_BATCH_GB", nullptr, &gpr_ctx::cv_batch_gb},
    {"GPR_QUAD_BATCH_GB", nullptr, &gpr_ctx::quad_batch_gb},
    {"GPR_QUAD_EIGEN", &gpr_ctx::quad_eigen, nullptr},
    {"GPR_QUAD_SEQ", &gpr_ctx::quad_seq, nullptr},
};

void knob_set(gpr_ctx* ctx, const Knob& k, double v) {
  if (k.ip) {
    int iv = (int)v;
    if (k.ip == &gpr_ctx::dag_zlag) iv = std::max(0, iv);
    if (k.ip == &gpr_ctx::cv_streams) iv = std::max(1, std::min(iv, (int)gpr_ctx::CV_MAX_SUB));
    ctx->*k.ip = iv;
  } else {
    ctx->*k.dp = v;
  }
}

const Knob* knob_find(const char* name) {
  if (!name) return nullptr;
  for (const Knob& k : kKnobs)
    if (!strcmp(k.name, name)) return &k;
  return nullptr;
}
}  // namespace

void copy_knobs(const gpr_ctx* from, gpr_ctx* to) {
  for (const Knob& k : kKnobs) {
    if (k.ip) to->*k.ip = from->*k.ip;
    else to->*k.dp = from->*k.dp;
  }
  to->dag_spin_limit = from->dag_spin_limit;
}

extern "C" {

const char* gpr_version(void) { return "gpr_hip 0.1.0 (gfx950)"; }

int gpr_ctx_create(int device, void* stream, gpr_ctx_t* out) {
  if (!out) return GPR_E_ARG;
  *out = nullptr;
  gpr_ctx* ctx = new gpr_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete ctx;
    return GPR_E_HIP;
  }
  if (stream) {
    ctx->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      delete ctx;
      return GPR_E_HIP;
    }
    ctx->own_stream = true;
  }
  ctx->ls = ctx->stream;
  // the lookahead panel stream gets the highest priority: its latency-bound chain
  // (diag factor + panel TRSM) must win CUs over the big trailing SYRK it overlaps
  int prio_lo = 0, prio_hi = 0;
  hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->srhs, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->ssq, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return GPR_E_HIP;
  }
  // Concurrent child contexts of cv_batch / integrate_noise: each drives its own stream, so
  // by default no more of them than the process has hardware queues (GPU_MAX_HW_QUEUES,
  // HIP's default 4); more only multiplex onto the same queues.
  if (const char* e = getenv("GPU_MAX_HW_QUEUES")) {
    const int q = atoi(e);
    if (q > 0) ctx->cv_streams = std::min(ctx->cv_streams, q);
  }
  // the documented knobs (include/gpr_hip.h), read once here; gpr_set_knob changes them
  for (const Knob& k : kKnobs)
    if (const char* e = getenv(k.name)) knob_set(ctx, k, atof(e));
  if (hipMalloc((void**)&ctx->dinfo, 64) != hipSuccess) {
    delete ctx;
    return GPR_E_NOMEM;
  }
  {
    // 2^(j/256) in extended precision, rounded once to double (assembly kexp_neg table)
    double tab[256];
    for (int j = 0; j < 256; ++j) tab[j] = (double)exp2l((long double)j / 256.0L);
    if (hipMalloc((void**)&ctx->dexptab, sizeof tab) != hipSuccess ||
        hipMemcpy(ctx->dexptab, tab, sizeof tab, hipMemcpyHostToDevice) != hipSuccess) {
      hipFree(ctx->dinfo);
      delete ctx;
      return GPR_E_NOMEM;
    }
  }
  *out = ctx;
  return 0;
}

int gpr_ctx_destroy(gpr_ctx_t ctx) {
  if (!ctx) return 0;
  for (auto* sub : ctx->cv_sub) gpr_ctx_destroy(sub);
  hipStreamSynchronize(ctx->stream);
  if (ctx->dag_sync_readers) {  // a hook's readers of dag_sync (freed below)
    hipEventSynchronize(ctx->dag_sync_readers);
    hipEventDestroy(ctx->dag_sync_readers);
  }
  drain_timing(ctx);
  for (auto e : ctx->event_pool) hipEventDestroy(e);
  for (auto e : ctx->sync_events) hipEventDestroy(e);
  if (ctx->stream2) hipStreamDestroy(ctx->stream2);
  if (ctx->srhs) hipStreamDestroy(ctx->srhs);
  if (ctx->ssq) hipStreamDestroy(ctx->ssq);
  if (ctx->dpanel_rhs) hipFree(ctx->dpanel_rhs);
  if (ctx->dscr_wt) hipFree(ctx->dscr_wt);
  if (ctx->dag_tasks) hipFree(ctx->dag_tasks);
  if (ctx->dag_sync) hipFree(ctx->dag_sync);
  if (ctx->dpadA) hipFree(ctx->dpadA);
  if (ctx->dpadB) hipFree(ctx->dpadB);
  if (ctx->rb_handle && ctx->rb_destroy) ctx->rb_destroy(ctx->rb_handle);
  if (ctx->winv) hipFree(ctx->winv);
  if (ctx->dinfo) hipFree(ctx->dinfo);
  if (ctx->dexptab) hipFree(ctx->dexptab);
  if (ctx->dscratch) hipFree(ctx->dscratch);
  if (ctx->dbig) hipFree(ctx->dbig);
  if (ctx->dbig2) hipFree(ctx->dbig2);
  if (ctx->dtrsv) hipFree(ctx->dtrsv);
  if (ctx->dsqinv) hipFree(ctx->dsqinv);
  if (ctx->dpanel) hipFree(ctx->dpanel);
  if (ctx->dxs) hipFree(ctx->dxs);
  if (ctx->dxps) hipFree(ctx->dxps);
  if (ctx->dgA) hipFree(ctx->dgA);
  if (ctx->dgB) hipFree(ctx->dgB);
  if (ctx->dgc) hipFree(ctx->dgc);
  for (auto& e : ctx->kup)
    if (e.d) hipFree(e.d);
  if (ctx->deig) hipFree(ctx->deig);
  if (ctx->ddc) hipFree(ctx->ddc);
  if (ctx->dc_tab_ev) hipEventDestroy(ctx->dc_tab_ev);
  if (ctx->dc_tab_host) hipHostFree(ctx->dc_tab_host);
  if (ctx->dtri) hipFree(ctx->dtri);
  if (ctx->dagb) hipFree(ctx->dagb);
  if (ctx->own_stream) hipStreamDestroy(ctx->stream);
  delete ctx;
  return 0;
}

const char* gpr_last_error(gpr_ctx_t ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int gpr_sync(gpr_ctx_t ctx) {
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

void* gpr_ctx_stream(gpr_ctx_t ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int gpr_malloc(gpr_ctx_t ctx, size_t bytes, void** dptr) {
  if (!dptr) return set_err(ctx, GPR_E_ARG, "dptr is NULL");
  if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess)
    return set_err(ctx, GPR_E_NOMEM, "hipMalloc(%zu) failed", bytes);
  return 0;
}

int gpr_free(gpr_ctx_t ctx, void* dptr) {
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (dptr) HIP_TRY(ctx, hipFree(dptr));
  return 0;
}

int gpr_upload(gpr_ctx_t ctx, void* dst, const void* src, size_t bytes) {
  HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int gpr_download(gpr_ctx_t ctx, void* dst, const void* src, size_t bytes) {
  HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int gpr_set_block(gpr_ctx_t ctx, int nb) {
  if (nb != 64 && nb != 128) return set_err(ctx, GPR_E_ARG, "nb must be 64 or 128 (got %d)", nb);
  ctx->nb = nb;
  if (ctx->nb2 % nb) ctx->nb2 = 4 * nb;
  ctx->fac_valid = false;
  return 0;
}

int gpr_set_outer_block(gpr_ctx_t ctx, int nb2) {
  if (nb2 < ctx->nb || nb2 % ctx->nb)
    return set_err(ctx, GPR_E_ARG, "outer block %d must be a multiple of nb=%d", nb2, ctx->nb);
  ctx->nb2 = nb2;
  return 0;
}

int gpr_set_knob(gpr_ctx_t ctx, const char* name, double value) {
  if (!ctx) return GPR_E_ARG;
  const Knob* k = knob_find(name);
  if (!k) return set_err(ctx, GPR_E_ARG, "unknown knob %s", name ? name : "(null)");
  knob_set(ctx, *k, value);
  if (k->ip == &gpr_ctx::dag_zlag) ctx->dag_lag_built = -1;  // (the task list depends on it)
  return 0;
}

int gpr_get_knob(gpr_ctx_t ctx, const char* name, double* value) {
  if (!ctx || !value) return GPR_E_ARG;
  const Knob* k = knob_find(name);
  if (!k) return set_err(ctx, GPR_E_ARG, "unknown knob %s", name ? name : "(null)");
  *value = k->ip ? (double)(ctx->*k->ip) : ctx->*k->dp;
  return 0;
}

int gpr_forget_factor(gpr_ctx_t ctx) {
  ctx->fac_valid = false;
  ctx->fac_ptr = nullptr;
  ctx->sqinv_nb2 = 0;
  ctx->sq_ptr = nullptr;
  return 0;
}

int gpr_timing_enable(gpr_ctx_t ctx, int on) {
  ctx->timing = on != 0;
  return 0;
}

int gpr_timing_get(gpr_ctx_t ctx, int cls, double* ms, long long* launches, double* flops) {
  if (cls < 0 || cls >= TC_N) return set_err(ctx, GPR_E_ARG, "bad timing class %d", cls);
  drain_timing(ctx);
  if (ms) *ms = ctx->t_ms[cls];
  if (launches) *launches = ctx->t_launches[cls];
  if (flops) *flops = ctx->t_flops[cls];
  return 0;
}

int gpr_timing_reset(gpr_ctx_t ctx) {
  drain_timing(ctx);
  for (int i = 0; i < TC_N; ++i) {
    ctx->t_ms[i] = 0;
    ctx->t_launches[i] = 0;
    ctx->t_flops[i] = 0;
  }
  return 0;
}

}  // extern "C"
