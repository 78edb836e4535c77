// libttk runtime: error reporting, launch accounting, pinned staging for host scalars.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "ttk_common.h"
#include "ttk_internal.h"

namespace ttk {

static thread_local char g_err[512] = "";
static std::atomic<long long> g_launches{0};
static std::atomic<long long> g_syncs{0};

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void note_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }
void note_sync() { g_syncs.fetch_add(1, std::memory_order_relaxed); }

struct Stage {
  double *p = nullptr;
  size_t n = 0;
  ~Stage() {
    if (p) (void)hipHostFree(p);
  }
};
static thread_local Stage g_stage;

double *pinned_stage(size_t n) {
  if (g_stage.n < n) {
    if (g_stage.p) (void)hipHostFree(g_stage.p);
    size_t want = n < 4096 ? 4096 : n;
    if (hipHostMalloc(reinterpret_cast<void **>(&g_stage.p), want * sizeof(double), 0) != hipSuccess) {
      g_stage.p = nullptr;
      g_stage.n = 0;
      return nullptr;
    }
    g_stage.n = want;
  }
  return g_stage.p;
}

// host-coherent mapped buffer (per context): small results are written there by a kernel and read
// by the host after the stream synchronises (no runtime blit + staging copy per read)
double *mapped_stage(size_t n, double **dev) {
  Ctx &c = ctx();
  if (c.mapped_n < n) {
    if (c.mapped_h) (void)hipHostFree(c.mapped_h);
    c.mapped_h = c.mapped_d = nullptr;
    c.mapped_n = 0;
    const size_t want = n < 8192 ? 8192 : n;
    if (hipHostMalloc(reinterpret_cast<void **>(&c.mapped_h), want * sizeof(double),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c.mapped_d), c.mapped_h, 0) != hipSuccess) {
      (void)hipHostFree(c.mapped_h);
      c.mapped_h = nullptr;
      return nullptr;
    }
    c.mapped_n = want;
  }
  *dev = c.mapped_d;
  return c.mapped_h;
}

static Ctx g_default_ctx;
static thread_local Ctx *g_cur_ctx = nullptr;
Ctx &ctx() { return g_cur_ctx ? *g_cur_ctx : g_default_ctx; }

}  // namespace ttk

namespace {
__global__ void to_host_kernel(const double *__restrict__ src, int64_t n, double *__restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
}  // namespace

extern "C" {

const char *ttk_last_error(void) { return ttk::g_err; }
int ttk_version(void) { return 1; }
long long ttk_launch_count(void) { return ttk::g_launches.load(); }
long long ttk_sync_count(void) { return ttk::g_syncs.load(); }

int ttk_upload(void *stream, const double *host, double *dev, int64_t n) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0) return TTK_OK;
  ttk::Ctx &c = ttk::ctx();  // host -> device through the context's ring of pinned slots
  ttk::UpSlot &sl = c.up[c.up_next];
  c.up_next = (c.up_next + 1) % ttk::UP_SLOTS;
  if (sl.pending) {
    TTK_HIP(hipEventSynchronize(sl.ev));  // the slot's previous copy has left it (normally long ago)
    sl.pending = false;
  }
  if (sl.n < (size_t)n) {
    if (sl.p) (void)hipHostFree(sl.p);
    sl.p = nullptr;
    sl.n = 0;
    const size_t want = (size_t)n < 4096 ? 4096 : (size_t)n;
    TTK_HIP(hipHostMalloc(reinterpret_cast<void **>(&sl.p), want * sizeof(double), 0));
    sl.n = want;
  }
  if (!sl.ev) TTK_HIP(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
  std::memcpy(sl.p, host, (size_t)n * sizeof(double));
  TTK_HIP(hipMemcpyAsync(dev, sl.p, (size_t)n * sizeof(double), hipMemcpyHostToDevice, TTK_STREAM(stream)));
  TTK_HIP(hipEventRecord(sl.ev, TTK_STREAM(stream)));
  sl.pending = true;
  return TTK_OK;
}

static int g_mapped_reads = getenv("TTK_MAPPED_READS") ? atoi(getenv("TTK_MAPPED_READS")) : 1;

int ttk_read_sync(void *stream, const double *src, double *host_dst, int64_t n) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0) return TTK_OK;
  if (n <= 65536 && g_mapped_reads) {  // small reads: one copy kernel into host-coherent memory
    double *dev = nullptr;
    double *h = ttk::mapped_stage(static_cast<size_t>(n), &dev);
    if (h) {
      const int grid = (int)((n + 255) / 256 < 64 ? (n + 255) / 256 : 64);
      hipLaunchKernelGGL(to_host_kernel, dim3(grid), dim3(256), 0, TTK_STREAM(stream), src, n, dev);
      TTK_LAUNCH_CHECK();
      ttk::note_sync();
      TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
      std::memcpy(host_dst, h, n * sizeof(double));
      return TTK_OK;
    }
  }
  double *st = ttk::pinned_stage(static_cast<size_t>(n));
  if (!st) {
    ttk::set_error("ttk_read_sync: pinned allocation failed");
    return TTK_ERR_HIP;
  }
  TTK_HIP(hipMemcpyAsync(st, src, n * sizeof(double), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  std::memcpy(host_dst, st, n * sizeof(double));
  return TTK_OK;
}

}  // extern "C"

// ---- contexts
namespace ttk {
void ctx_bind(Ctx *c) { g_cur_ctx = c; }
Ctx *ctx_swap(Ctx *c) {
  Ctx *p = g_cur_ctx;
  g_cur_ctx = c;
  return p;
}
}  // namespace ttk

int ttk::dep_counter(void *stream) {
  ttk::Ctx &cx = ttk::ctx();
  if (cx.dep) return TTK_OK;
  TTK_HIP(hipMalloc(reinterpret_cast<void **>(&cx.dep), 256));
  TTK_HIP(hipMemsetAsync(cx.dep, 0, 256, TTK_STREAM(stream)));
  cx.dep_total = 0;
  cx.tick_total = 0;
  return TTK_OK;
}

extern "C" {

int ttk_ctx_create(void *stream, ttk_ctx *out) {
  *out = nullptr;
  ttk_ctx_s *h = new (std::nothrow) ttk_ctx_s();
  if (!h) {
    ttk::set_error("ttk_ctx_create: out of host memory");
    return TTK_ERR_ARG;
  }
  h->c.stream = TTK_STREAM(stream);
  // TTK_EAGER_SIDE=1: create the context's second stream now instead of at its first forked dgecon
  // (diagnostics: whether a process's second HW queue changes how concurrent processes share the GPU)
  static const int eager = getenv("TTK_EAGER_SIDE") ? atoi(getenv("TTK_EAGER_SIDE")) : 0;
  if (eager && !h->c.side) {
    if (hipStreamCreateWithFlags(&h->c.side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->c.ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->c.ev_join, hipEventDisableTiming) != hipSuccess) {
      delete h;
      ttk::set_error("ttk_ctx_create: side stream creation failed");
      return TTK_ERR_HIP;
    }
  }
  {  // scratch at its initial sizes now (this entry point releases the GIL; the launch-only ones that
     // would grow it later keep it, _lib.py), and the hand-off counter
    ttk::Ctx *prev = ttk::ctx_swap(&h->c);
    int rc = ttk::presize_splitk();
    if (!rc) rc = ttk::presize_lgmres();
    if (!rc) rc = ttk::presize_schur();
    if (!rc) rc = ttk::dep_counter(stream);
    if (!rc && hipStreamSynchronize(TTK_STREAM(stream)) != hipSuccess) rc = TTK_ERR_HIP;
    ttk::ctx_swap(prev);
    if (rc) {
      ttk_ctx_destroy(h);
      return rc;
    }
  }
  *out = h;
  return TTK_OK;
}

int ttk_ctx_set_knob(ttk_ctx h, int knob, int value, int *old) {
  if (knob < 0 || knob >= TTK_KNOB_COUNT) {
    ttk::set_error("ttk_ctx_set_knob: unknown knob %d", knob);
    return TTK_ERR_ARG;
  }
  if (knob == TTK_KNOB_SPLITK_MINK && value <= 0) {
    ttk::set_error("ttk_ctx_set_knob: SPLITK_MINK must be > 0 (got %d)", value);
    return TTK_ERR_ARG;
  }
  ttk::Ctx &c = h ? h->c : ttk::ctx();
  if (old) *old = c.knob[knob];
  c.knob[knob] = value;
  return TTK_OK;
}

int ttk_ctx_get_knob(ttk_ctx h, int knob, int *value) {
  if (knob < 0 || knob >= TTK_KNOB_COUNT) {
    ttk::set_error("ttk_ctx_get_knob: unknown knob %d", knob);
    return TTK_ERR_ARG;
  }
  *value = (h ? h->c : ttk::ctx()).knob[knob];
  return TTK_OK;
}

void *ttk_ctx_stream(ttk_ctx h) { return h ? reinterpret_cast<void *>(h->c.stream) : nullptr; }

int ttk_ctx_bind(ttk_ctx h) {
  ttk::ctx_bind(h ? &h->c : nullptr);
  return TTK_OK;
}

int ttk_ctx_destroy(ttk_ctx h) {
  if (!h) return TTK_OK;
  ttk::Ctx &c = h->c;
  TTK_HIP(hipStreamSynchronize(c.stream));
  ttk::Ctx *prev = ttk::g_cur_ctx;
  ttk::g_cur_ctx = &c;
  ttk::ctx_free_einsum(c);
  ttk::g_cur_ctx = prev == &c ? nullptr : prev;
  for (double *p : {c.scratch, c.splitk, c.dev_scalar, c.schur_w, c.lgmres, c.rcond}) if (p) (void)hipFree(p);
  ttk::schur_release(c);
  if (c.status) (void)hipFree(c.status);
  if (c.dep) (void)hipFree(c.dep);
  if (c.splitk_cnt) (void)hipFree(c.splitk_cnt);
  if (c.colr) (void)hipFree(c.colr);
  if (c.mapped_h) (void)hipHostFree(c.mapped_h);
  if (c.side) {
    (void)hipStreamSynchronize(c.side);
    (void)hipStreamDestroy(c.side);
    (void)hipEventDestroy(c.ev_fork);
    (void)hipEventDestroy(c.ev_join);
  }
  for (ttk::UpSlot &u : c.up) {
    if (u.p) (void)hipHostFree(u.p);
    if (u.ev) (void)hipEventDestroy(u.ev);
  }
  delete h;
  return TTK_OK;
}

}  // extern "C"
