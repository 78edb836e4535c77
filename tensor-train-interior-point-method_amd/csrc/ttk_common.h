// Shared helpers for libttk (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ttk.h"

namespace ttk {

void set_error(const char *fmt, ...);
void note_launch();
double *pinned_stage(size_t n_doubles);  // per-thread pinned host staging buffer

constexpr int WAVE = 64;
constexpr int MAXD = 6;

struct NdDesc {
  int ndim;
  int64_t total;
  int64_t shape[MAXD];
  int64_t s0[MAXD];
  int64_t s1[MAXD];
  int64_t s2[MAXD];
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// block-wide sum; `red` must hold blockDim.x/64 doubles; result valid on all threads
__device__ __forceinline__ double block_sum(double v, double *red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

}  // namespace ttk

#define TTK_HIP(call)                                                                    \
  do {                                                                                   \
    hipError_t _e = (call);                                                              \
    if (_e != hipSuccess) {                                                              \
      ttk::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(_e)); \
      return TTK_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define TTK_LAUNCH_CHECK()                                                               \
  do {                                                                                   \
    ttk::note_launch();                                                                  \
    hipError_t _e = hipGetLastError();                                                   \
    if (_e != hipSuccess) {                                                              \
      ttk::set_error("%s:%d launch: %s", __FILE__, __LINE__, hipGetErrorString(_e));     \
      return TTK_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define TTK_STREAM(s) (reinterpret_cast<hipStream_t>(s))
