// libttk runtime: error reporting, launch accounting, pinned staging for host scalars.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "ttk_common.h"

namespace ttk {

static thread_local char g_err[512] = "";
static std::atomic<long long> g_launches{0};

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void note_launch() { g_launches.fetch_add(1, std::memory_order_relaxed); }

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

}  // namespace ttk

extern "C" {

const char *ttk_last_error(void) { return ttk::g_err; }
int ttk_version(void) { return 1; }
long long ttk_launch_count(void) { return ttk::g_launches.load(); }

int ttk_read_sync(void *stream, const double *src, double *host_dst, int64_t n) {
  if (n <= 0) return TTK_OK;
  double *st = ttk::pinned_stage(static_cast<size_t>(n));
  if (!st) {
    ttk::set_error("ttk_read_sync: pinned allocation failed");
    return TTK_ERR_HIP;
  }
  TTK_HIP(hipMemcpyAsync(st, src, n * sizeof(double), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  std::memcpy(host_dst, st, n * sizeof(double));
  return TTK_OK;
}

}  // extern "C"
