// Launch-to-launch time of back-to-back small kernels vs grid / block shape (tuning probe, not product).
//   hipcc -O3 --offload-arch=gfx950 tools/launch_micro.hip -o /tmp/launch_micro && /tmp/launch_micro
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_touch(const double* __restrict__ a, double* __restrict__ b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] + 1.0;
}
int main() {
  const int n = 1 << 20;
  double *a, *b;
  hipMalloc(&a, n * sizeof(double)); hipMalloc(&b, n * sizeof(double));
  hipMemset(a, 0, n * sizeof(double));
  hipStream_t s; hipStreamCreate(&s);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int shapes[][2] = {{260, 128}, {130, 256}, {260, 64}, {520, 64}, {65, 512}, {1, 64}, {1040, 64}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& sh : shapes) {
      const int grid = sh[0], block = sh[1], N = 2000;
      for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(block), 0, s, a, b, n);
      hipEventRecord(e0, s);
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(block), 0, s, a, b, n);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("grid %5d block %4d: %.3f us per launch\n", grid, block, ms * 1e3 / N);
    }
  return 0;
}
