// Occupancy probe: one-wave blocks of a kernel pinned at 168 VGPRs
// (waves_per_eu 3) -- how many fit a CU as the dynamic LDS per block grows.
// Prints the LDS sizes at which the resident-block count changes, i.e. the
// LDS allocation granularity the level kernel's tile sizing has to respect.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) k_probe(int* p) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p) p[threadIdx.x] = s[63 - threadIdx.x];
}
int main() {
  int prev = -1;
  for (int lds = 8192; lds <= 20480; lds += 64) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_probe, 64, lds) != hipSuccess) return 1;
    if (nb != prev) printf("dynamic LDS %6d B -> %d blocks/CU\n", lds, nb);
    prev = nb;
  }
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, (const void*)k_probe) == hipSuccess)
    printf("probe kernel: %d VGPRs(numRegs), static LDS %zu\n", a.numRegs, a.sharedSizeBytes);
  return 0;
}
