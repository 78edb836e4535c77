// Isolated cost of one one-sided Jacobi round (jacobi_round<G> from ttk_linalg.hip) on a small
// LDS-resident matrix.  Build: hipcc -O3 --offload-arch=gfx950 jround.hip -o jround
#include "../../tensor-train-interior-point-method_amd/csrc/ttk_linalg.hip"
#include "../../tensor-train-interior-point-method_amd/csrc/ttk_runtime.hip"

template <int G>
__global__ void k_round(int p, int L, int rounds, int mode, unsigned long long *out) {
  __shared__ double X[64 * 65], V[64 * 65];
  __shared__ int any;
  const int tid = threadIdx.x;
  const int ldx = L | 1, ldv = p | 1;
  for (int e = tid; e < ldx * p; e += blockDim.x) X[e] = 1.0 / (1.0 + (e * 7919 % 101));
  for (int e = tid; e < ldv * p; e += blockDim.x) V[e] = (e % (ldv + 1)) == 0 ? 1.0 : 0.0;
  __syncthreads();
  const int P = (p % 2) ? p + 1 : p;
  const unsigned long long t0 = wall_clock64();
  for (int it = 0; it < rounds; ++it) {
    const int r = it % (P - 1);
    if (mode == 0) {
      jacobi_round<G>(X, ldx, V, ldv, p, L, P, r, 0.0, &any);  // tol 0: always rotates
    } else {
      jacobi_round<G>(X, ldx, V, ldv, p, L, P, r, 1e300, &any);  // never rotates
    }
    __syncthreads();
  }
  const unsigned long long t1 = wall_clock64();
  if (tid == 0) out[0] = t1 - t0;
}

int main() {
  unsigned long long *d, h;
  (void)hipMalloc(&d, sizeof(h));
  const int rounds = 20000;
  struct C { int p, L, nt; };
  for (C c : {C{8, 8, 64}, C{16, 16, 64}, C{48, 48, 192}}) {
    for (int mode = 0; mode < 2; ++mode) {
      if (c.p == 8) hipLaunchKernelGGL(k_round<1>, dim3(1), dim3(c.nt), 0, 0, c.p, c.L, rounds, mode, d);
      if (c.p == 16) hipLaunchKernelGGL(k_round<2>, dim3(1), dim3(c.nt), 0, 0, c.p, c.L, rounds, mode, d);
      if (c.p == 48) hipLaunchKernelGGL(k_round<8>, dim3(1), dim3(c.nt), 0, 0, c.p, c.L, rounds, mode, d);
      (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("p=%2d L=%2d threads %4d %-12s %8.1f ns/round\n", c.p, c.L, c.nt, mode ? "no-rotate" : "rotate",
             h * 10.0 / rounds);
    }
  }
  return 0;
}
