// Latency microbenchmark of the primitives one-workgroup factorisations are built from.
// Build: hipcc -O3 --offload-arch=gfx950 latency.hip -o latency ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../tensor-train-interior-point-method_amd/csrc/ttk_common.h"

__global__ void k_sync(int iters, unsigned long long *out, int mode, int div) {
  __shared__ double buf[1024];
  const int tid = threadIdx.x;
  double acc = tid;
  buf[tid] = tid;
  __syncthreads();
  const unsigned long long t0 = wall_clock64(), c0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (mode == 0) {  // barrier only
      __syncthreads();
    } else if (mode == 1) {  // LDS write -> barrier -> LDS read (neighbour)
      buf[tid] = acc;
      __syncthreads();
      acc = buf[(tid + 1) % blockDim.x] * 0.5 + 1.0;
      __syncthreads();
    } else if (mode == 2) {  // integer modulo by runtime divisor (dependent chain)
      acc += (double)(((int)acc + it) % div);
    } else if (mode == 3) {  // DPP wave_sum (dependent chain)
      acc = ttk::wave_sum(acc) * 1e-3 + 1.0;
    } else if (mode == 4) {  // fp64 division chain
      acc = 1.0 / (acc + 1.0) + 0.5;
    } else if (mode == 5) {  // fp64 sqrt chain
      acc = sqrt(acc + 1.0);
    } else if (mode == 6) {  // group_sum_rt(g=2)
      acc = ttk::group_sum_rt(acc, 2) * 0.5 + 1.0;
    } else if (mode == 7) {  // 8 dependent fp64 FMAs
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fma(acc, 0.999999, 1e-9);
    } else if (mode == 8) {  // 8 dependent fp32 FMAs
      float f = (float)acc;
#pragma unroll
      for (int u = 0; u < 8; ++u) f = fmaf(f, 0.999999f, 1e-9f);
      acc = f;
    } else if (mode == 9) {  // 2 x 8 independent fp64 FMA chains
      double b2 = acc + 1.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc = fma(acc, 0.999999, 1e-9);
        b2 = fma(b2, 0.999999, 1e-9);
      }
      acc += b2;
    }
  }
  const unsigned long long t1 = wall_clock64(), c1 = clock64();
  if (tid == 0) {
    out[0] = t1 - t0;
    out[1] = c1 - c0;
    out[2] = (unsigned long long)acc;
  }
}

int main() {
  unsigned long long *d, h[3];
  hipMalloc(&d, 3 * sizeof(unsigned long long));
  const char *names[] = {"barrier", "lds+2 barriers", "int modulo", "wave_sum (DPP)", "fp64 div", "fp64 sqrt",
                         "group_sum g=2", "8 dep fp64 fma", "8 dep fp32 fma", "2x8 fp64 fma"};
  const int iters = 20000;
  for (int threads : {64, 256, 1024}) {
    for (int mode = 0; mode < 10; ++mode) {
      hipLaunchKernelGGL(k_sync, dim3(1), dim3(threads), 0, 0, iters, d, mode, 7);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      const double ns = h[0] * 10.0 / iters;  // wall_clock64 = 100 MHz
      printf("threads %4d %-16s %8.1f ns/iter  %7.0f cycles/iter  (shader clock %.0f MHz)\n", threads, names[mode], ns,
             (double)h[1] / iters, (double)h[1] / (h[0] * 10.0) * 1e3);
    }
  }
  return 0;
}
