// Tuning probe (not product): a GN step's hand-off from the converging PCG launch to the next step's first kernel
// on ANOTHER stream gated by hipStreamWaitValue32 on signal memory, instead of the same stream behind the chunk's
// drained launches.
//   hipcc -O3 --offload-arch=gfx950 tools/waitvalue_micro.hip -o tools/bin/waitvalue_micro && tools/bin/waitvalue_micro
//
// Stream A: 40 launches of a ~3 us kernel (260 workgroups of 128 threads spinning on the wall clock); launch 20 is the
// "converging" one: its last-arriving workgroup stores the step number into the signal word (release, system
// scope) and records the wall clock; launches 21..39 end at once (the drained launches). Stream B: waits for the
// signal (>= step) and runs a probe kernel that records its start. Reported: signal -> probe start, and for
// comparison the same probe enqueued on stream A behind the drained launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef unsigned long long u64;

// mode 0: spin ~spin ticks; mode 1: converging (spin, then the last workgroup signals); mode 2: drained (return)
__global__ __launch_bounds__(128) void k_work(int mode, u64 spin, unsigned* __restrict__ arrive, unsigned* sig,
                                              unsigned step, u64* __restrict__ t_sig) {
  if (mode == 2) return;
  const u64 t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) {
  }
  if (mode == 1) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned old = atomicAdd(arrive, 1u);
      if (old == gridDim.x - 1) {
        *arrive = 0;
        *t_sig = wall_clock64();
        __hip_atomic_store(sig, step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

__global__ void k_probe(u64* __restrict__ t_start) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *t_start = wall_clock64();
}

int main() {
  int dev = 0, can = 0, rate_khz = 0;
  CHECK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev));
  CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
  printf("{\"can_wait_value\": %d, \"wall_clock_khz\": %d", can, rate_khz);
  const double us_per_tick = 1000.0 / rate_khz;
  unsigned* sig = nullptr;
  const char* kind = "signal";
  if (hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    kind = "host_coherent";
    CHECK(hipHostMalloc((void**)&sig, 64, hipHostMallocCoherent | hipHostMallocMapped));
  }
  CHECK(hipMemset(sig, 0, 8));
  printf(", \"sig_memory\": \"%s\"", kind);
  unsigned* arrive = nullptr;
  u64 *t_sig = nullptr, *t_probe = nullptr;
  CHECK(hipMalloc(&arrive, 64));
  CHECK(hipMemset(arrive, 0, 64));
  CHECK(hipMalloc(&t_sig, 64 * sizeof(u64)));
  CHECK(hipMalloc(&t_probe, 64 * sizeof(u64)));
  hipStream_t A, B;
  CHECK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  const u64 spin = (u64)(3.0 / us_per_tick);
  std::vector<double> lat_b, lat_a;
  for (int rep = 0; rep < 24; ++rep) {
    const unsigned step = rep + 1;
    const bool cross = rep % 2 == 0;
    if (cross) CHECK(hipStreamWaitValue32(B, sig, step, hipStreamWaitValueGte, 0xFFFFFFFFu));
    if (cross) hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, B, t_probe + rep);
    for (int i = 0; i < 40; ++i)
      hipLaunchKernelGGL(k_work, dim3(260), dim3(128), 0, A, i < 20 ? 0 : (i == 20 ? 1 : 2), spin, arrive, sig, step,
                         t_sig + rep);
    if (!cross) hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, A, t_probe + rep);
    CHECK(hipStreamSynchronize(A));
    CHECK(hipStreamSynchronize(B));
  }
  std::vector<u64> ts(64), tp(64);
  CHECK(hipMemcpy(ts.data(), t_sig, 64 * sizeof(u64), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(tp.data(), t_probe, 64 * sizeof(u64), hipMemcpyDeviceToHost));
  for (int rep = 2; rep < 24; ++rep) {   // first two: warm-up
    const double d = (double)((long long)(tp[rep] - ts[rep])) * us_per_tick;
    (rep % 2 == 0 ? lat_b : lat_a).push_back(d);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  auto mn = [](const std::vector<double>& v) { return *std::min_element(v.begin(), v.end()); };
  auto mx = [](const std::vector<double>& v) { return *std::max_element(v.begin(), v.end()); };
  printf(", \"signal_to_probe_other_stream_us\": {\"median\": %.2f, \"min\": %.2f, \"max\": %.2f}", med(lat_b), mn(lat_b),
         mx(lat_b));
  printf(", \"signal_to_probe_same_stream_after_19_drained_us\": {\"median\": %.2f, \"min\": %.2f, \"max\": %.2f}}\n",
         med(lat_a), mn(lat_a), mx(lat_a));
  return 0;
}
