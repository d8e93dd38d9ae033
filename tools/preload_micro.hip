// Probe (not product): does kernarg preloading (-mllvm -amdgpu-kernarg-preload-count) shorten a chain of dependent
// launches on this box? Each launch of k_chain reads a list entry through a pointer argument, then gathers one row
// through it (twelve dependent trips, so the GPU and not the host's enqueue sets the pace), and writes one value; 256 workgroups of 128
// threads, launched back to back. Build twice (with / without the flag) and compare the launch-to-launch time:
//   hipcc --offload-arch=gfx950 -O3 tools/preload_micro.hip -o tools/stampslib/pm_base
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 tools/preload_micro.hip -o tools/stampslib/pm_pre
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(128) void k_chain(const int* __restrict__ list, const double* __restrict__ rows,
                                               double* __restrict__ out, int n) {
  const int i = blockIdx.x * 128 + threadIdx.x;
  int j = list[i];                    // trip 1: through a pointer argument
#pragma unroll 1
  for (int r = 0; r < 10; ++r) j = list[j];   // ten more dependent trips: the GPU, not the host, sets the pace
  const double v = rows[j];           // gathered through the list
  out[i] = v + (double)n;
}

int main() {
  const int nwg = 256, n = nwg * 128, launches = 4000;
  int* list;
  double *rows, *out;
  hipMalloc(&list, n * sizeof(int));
  hipMalloc(&rows, n * sizeof(double));
  hipMalloc(&out, n * sizeof(double));
  std::vector<int> h(n);
  for (int i = 0; i < n; ++i) h[i] = (i * 7919) % n;
  hipMemcpy(list, h.data(), n * sizeof(int), hipMemcpyHostToDevice);
  hipMemset(rows, 0, n * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 4; ++rep) {
    for (int k = 0; k < 200; ++k) hipLaunchKernelGGL(k_chain, dim3(nwg), dim3(128), 0, 0, list, rows, out, k);
    hipEventRecord(e0, 0);
    for (int k = 0; k < launches; ++k) hipLaunchKernelGGL(k_chain, dim3(nwg), dim3(128), 0, 0, list, rows, out, k);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("rep %d: %.3f us per launch\n", rep, 1e3 * ms / launches);
  }
  return 0;
}
