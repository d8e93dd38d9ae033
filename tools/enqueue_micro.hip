// Host enqueue cost vs GPU launch-to-launch time for back-to-back small kernels (tuning probe, not product).
// Does the host keep up with a ~4 us dependent PCG launch? Forms compared, each N launches of a kernel that spins for
// a given time on the GPU (so the GPU side is fixed):
//   a) hipLaunchKernelGGL, 2 pointer args             b) hipLaunchKernelGGL, + a 256-B struct arg
//   c) hipExtLaunchKernel (same 256-B args)           d) a hipGraph of 100 launches (captured once, replayed)
//   e) a hipGraph of 8 launches, replayed              f) a hipGraph of 2 launches, replayed
//   hipcc -O3 --offload-arch=gfx950 tools/enqueue_micro.hip -o tools/stampslib/enqueue_micro && tools/stampslib/enqueue_micro
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

struct Big {
  double* p[28];
  int a, b;
};
__device__ __forceinline__ void spin(long long cyc) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < cyc) {}
}
__global__ void k_small(double* a, long long cyc) {
  spin(cyc);
  if (threadIdx.x == 0 && blockIdx.x == 0) a[0] += 1.0;
}
__global__ void k_big(double* a, Big b, long long cyc) {
  spin(cyc);
  if (threadIdx.x == 0 && blockIdx.x == 0) a[0] += (double)b.a;
}

int main() {
  double* a;
  hipMalloc(&a, 64);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  Big big{};
  big.a = 1;
  const int N = 2000;
  int grid = 250, block = 128;
  if (const char* e = getenv("GRID")) grid = atoi(e);
  if (const char* e = getenv("BLOCK")) block = atoi(e);
  printf("grid %d x block %d\n", grid, block);
  for (long long cyc : {0LL, 5000LL, 7500LL}) {   // s_memtime ticks at 2.4 GHz on gfx950 (reported, see below)
    for (int form = 0; form < 6; ++form) {
      hipGraphExec_t ge = nullptr;
      const int glen = form == 3 ? 100 : form == 4 ? 8 : 2;
      if (form >= 3) {
        hipGraph_t gr;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < glen; ++i) hipLaunchKernelGGL(k_big, dim3(grid), dim3(block), 0, s, a, big, cyc);
        hipStreamEndCapture(s, &gr);
        hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        hipGraphDestroy(gr);
      }
      auto launch = [&](int n) {
        for (int i = 0; i < n; ++i) {
          if (form == 0) hipLaunchKernelGGL(k_small, dim3(grid), dim3(block), 0, s, a, cyc);
          else if (form == 1) hipLaunchKernelGGL(k_big, dim3(grid), dim3(block), 0, s, a, big, cyc);
          else if (form == 2) {
            void* args[] = {&a, &big, &cyc};
            hipExtLaunchKernel((const void*)k_big, dim3(grid), dim3(block), args, 0, s, nullptr, nullptr, 0);
          } else if (i % glen == 0) hipGraphLaunch(ge, s);
        }
      };
      launch(200);
      hipStreamSynchronize(s);
      hipEventRecord(e0, s);
      const auto h0 = std::chrono::steady_clock::now();
      launch(N);
      const auto h1 = std::chrono::steady_clock::now();
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double host = std::chrono::duration<double, std::micro>(h1 - h0).count() / N;
      printf("spin %5lld form %c: host enqueue %.3f us/launch, GPU %.3f us/launch\n", cyc, "abcdef"[form], host,
             ms * 1e3 / N);
      if (ge) hipGraphExecDestroy(ge);
    }
  }
  // the spin clock: one launch of 1e6 ticks
  hipEventRecord(e0, s);
  hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, a, 1000000LL);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("1e6 s_memtime ticks = %.3f ms\n", ms);
  return 0;
}
