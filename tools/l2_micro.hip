// Does a back-to-back launch find last launch's data in L2? (tuning probe, not product). Each launch of k_probe reads
// one static line per wave (the same line every launch: the same workgroup runs on the same XCD) and times that first
// load, then a second load of a line it has not touched in this launch but that an earlier launch read (same XCD), and
// a third load of the first line again (now an L1/L2 hit). s_memtime cycles, median over the waves and launches.
//   hipcc -O3 --offload-arch=gfx950 tools/l2_micro.hip -o tools/stampslib/l2_micro && tools/stampslib/l2_micro
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void k_probe(const int* __restrict__ stat, const int* __restrict__ stat2, long long* __restrict__ out,
                        int launch) {
  const int w = blockIdx.x;
  const int lane = threadIdx.x;
  const int* p1 = stat + w * 64 + lane;
  const int* p2 = stat2 + ((w + launch) % gridDim.x) * 64 + lane;
  const int* p3 = stat + (w * 64 + lane + 16) % (64 * gridDim.x);
  asm volatile("" :: "v"(p1), "v"(p2), "v"(p3) : "memory");   // addresses (and the kernel arguments) ready before t0
  const long long t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int v = *p1;                       // static, read by this workgroup in every launch
  asm volatile("" : "+v"(v) :: "memory");            // (forces the wait for the load here)
  const long long t1 = __builtin_amdgcn_s_memtime();
  asm volatile("" ::: "memory");
  int v2 = *p2;   // static, but read by another workgroup last launch
  asm volatile("" : "+v"(v2) :: "memory");
  const long long t2 = __builtin_amdgcn_s_memtime();
  asm volatile("" ::: "memory");
  int v3 = *p3;   // a line this wave just read (hit)
  asm volatile("" : "+v"(v3) :: "memory");
  const long long t3 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    long long* o = out + ((long long)launch * gridDim.x + w) * 4;
    o[0] = t1 - t0; o[1] = t2 - t1; o[2] = t3 - t2; o[3] = v + v2 + v3;
  }
}

int main() {
  const int nwg = 256, L = 400;
  int *stat, *stat2;
  long long* out;
  (void)hipMalloc(&stat, nwg * 64 * sizeof(int));
  (void)hipMalloc(&stat2, nwg * 64 * sizeof(int));
  (void)hipMalloc(&out, (size_t)L * nwg * 4 * sizeof(long long));
  (void)hipMemset(stat, 0, nwg * 64 * sizeof(int));
  (void)hipMemset(stat2, 0, nwg * 64 * sizeof(int));
  for (int l = 0; l < L; ++l) hipLaunchKernelGGL(k_probe, dim3(nwg), dim3(64), 0, 0, stat, stat2, out, l);
  (void)hipDeviceSynchronize();
  std::vector<long long> h((size_t)L * nwg * 4);
  (void)hipMemcpy(h.data(), out, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
  for (int k = 0; k < 3; ++k) {
    std::vector<long long> x;
    for (int l = 50; l < L; ++l)
      for (int w = 0; w < nwg; ++w) x.push_back(h[((size_t)l * nwg + w) * 4 + k]);
    std::sort(x.begin(), x.end());
    printf("%s: median %lld cycles, p10 %lld, p90 %lld\n",
           k == 0 ? "first load (static line, same XCD last launch)" : k == 1 ? "second load (static, other WG last launch)"
                                                                      : "third load (line just read)",
           x[x.size() / 2], x[x.size() / 10], x[x.size() * 9 / 10]);
  }
  return 0;
}
