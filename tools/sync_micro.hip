// Tuning probe (not product): what one PCG iteration's cross-workgroup traffic costs on this part, as a kernel
// boundary vs inside one persistent launch, at the PCG's real geometry (260 cluster workgroups of 128 threads).
//   hipcc -O3 --offload-arch=gfx950 tools/sync_micro.hip -o tools/bin/sync_micro && tools/bin/sync_micro
//
// 1. boundary: back-to-back launches of a kernel whose every workgroup reads its own 44 KB slice of a 11.4 MB
//    buffer (the PCG's per-cluster bytes), for grids of 256 / 260 / 264 workgroups, slice = blockIdx, and for 256
//    with slice = (XCC id, blockIdx / 8) (the same slices on the same XCD every launch). Records each workgroup's
//    XCC id for the first launches (is the block -> XCD map stable across launches?).
// 2. persistent: ONE launch of 260 workgroups looping K iterations; per iteration each workgroup publishes its
//    cluster's 48 doubles (m rows) and 3 partial sums as tagged 8-byte granules (a double = two {tag, 32-bit half}
//    granules, sc1 stores), then waits for (a) its 16 neighbours' rows, (b) all 260 x 3 partials (every workgroup
//    sweeps them: an all-gather), or (c) both, sums the partials in a fixed order, and goes on. Bounded spins.
//    Reports us per iteration.
#include <hip/hip_runtime.h>

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

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

constexpr int kSlice = 44 * 1024;   // bytes per workgroup per iteration (the PCG's ~44 KB per cluster)

// mode 0: slice = blockIdx; mode 1: slice = xcc * (gridDim / 8) + blockIdx / 8 (needs gridDim % 8 == 0)
__global__ __launch_bounds__(128) void k_slice(const float4* __restrict__ buf, float* __restrict__ out, int mode,
                                               int* __restrict__ xcc_log, int log_launch) {
  const int b = blockIdx.x;
  const int x = xcc_id();
  const int slice = mode == 0 ? b : x * (int)(gridDim.x / 8) + b / 8;
  const float4* p = buf + (size_t)slice * (kSlice / 16);
  float a = 0.f;
#pragma unroll 4
  for (int i = threadIdx.x; i < kSlice / 16; i += 128) {
    const float4 v = p[i];
    a += (v.x + v.y) + (v.z + v.w);
  }
  if (threadIdx.x == 0) {
    out[b] = a;
    if (xcc_log && log_launch >= 0) xcc_log[log_launch * 1024 + b] = x;
  }
}

typedef unsigned long long u64;
__device__ __forceinline__ void put_granule(u64* g, unsigned tag, unsigned v) {
  __hip_atomic_store(g, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 get_granule(u64* g) { return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

constexpr int kG = 260, kRows = 48, kNb = 16;
constexpr unsigned kSpinLimit = 1u << 22;

// granule layout: rows[(wg * 48 + r) * 2 + half], parts[(wg * 3 + k) * 2 + half]
__global__ __launch_bounds__(128) void k_persist(u64* rows, u64* parts, const int* __restrict__ nbr, int iters,
                                                 int mode, int* err, double* sink, int G) {
  const int wg = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ double s_part[3];
  __shared__ int s_fail;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    const unsigned tag = (unsigned)it + 1;
    // publish: 48 row doubles (lanes 0..47 of wave 0: two granules each) + 3 partials (wave 1 lanes 0..2)
    const double val = (double)(wg * 1000 + it) + 0.25 * tid + acc * 1e-30;
    if (w == 0 && lane < kRows) {
      const u64 bits = (u64)__double_as_longlong(val);
      put_granule(rows + ((size_t)wg * kRows + lane) * 2, tag, (unsigned)bits);
      put_granule(rows + ((size_t)wg * kRows + lane) * 2 + 1, tag, (unsigned)(bits >> 32));
    }
    if (w == 1 && lane < 3) {
      const u64 bits = (u64)__double_as_longlong(val + lane);
      put_granule(parts + ((size_t)wg * 3 + lane) * 2, tag, (unsigned)bits);
      put_granule(parts + ((size_t)wg * 3 + lane) * 2 + 1, tag, (unsigned)(bits >> 32));
    }
    // consume (mode 1: neighbours, 2: partials, 3: both); wave 0 gathers neighbour rows (lane = one of 16
    // neighbours x 4 of its rows' ... every lane reads 6 granule pairs of one neighbour row block), wave 1 sweeps the
    // partials (lane reads entries lane, lane + 64, ... of 780)
    double got = 0.0;
    if (w == 0 && (mode & 1)) {
      const int nb = nbr[wg * kNb + (lane & 15)];
      const int r0 = (lane >> 4) * 12;
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 12; r += 2) {
          const u64 lo = get_granule(rows + ((size_t)nb * kRows + r0 + r) * 2);
          const u64 hi = get_granule(rows + ((size_t)nb * kRows + r0 + r) * 2 + 1);
          ok &= (unsigned)(lo >> 32) >= tag && (unsigned)(hi >> 32) >= tag;   // producers may run ahead
          s += __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
        }
        if (__all(ok)) { got = s; break; }
        if (++spins > kSpinLimit || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          if (lane == 0) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); s_fail = 1; }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (w == 1 && (mode & 2)) {
      unsigned spins = 0;
      for (;;) {
        bool ok = true;
        double s[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int u = 0; u < 5; ++u) {          // 5 x 64 >= 260 producers (x 3 partials as a,b,c per producer)
          const int p = lane + 64 * u;
          if (p < G) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const u64 lo = get_granule(parts + ((size_t)p * 3 + k) * 2);
              const u64 hi = get_granule(parts + ((size_t)p * 3 + k) * 2 + 1);
              ok &= (unsigned)(lo >> 32) >= tag && (unsigned)(hi >> 32) >= tag;   // producers may run ahead
              s[k] += __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
            }
          }
        }
        if (__all(ok)) {
          for (int k = 0; k < 3; ++k)
            for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
          if (lane == 0) { s_part[0] = s[0]; s_part[1] = s[1]; s_part[2] = s[2]; }
          break;
        }
        if (++spins > kSpinLimit || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          if (lane == 0) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); s_fail = 1; }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (s_fail) break;
    acc += got + (mode & 2 ? s_part[0] : 0.0);
    __syncthreads();
  }
  if (tid == 0) sink[wg] = acc;
}

int main(int argc, char** argv) {
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // ---- 1. boundary + slice reads
  const size_t nbuf = (size_t)264 * kSlice;
  float4* buf;
  float* out;
  int* xlog;
  CHECK(hipMalloc(&buf, nbuf));
  CHECK(hipMemset(buf, 0, nbuf));
  CHECK(hipMalloc(&out, 1024 * sizeof(float)));
  CHECK(hipMalloc(&xlog, 16 * 1024 * sizeof(int)));
  CHECK(hipMemset(xlog, 0xff, 16 * 1024 * sizeof(int)));
  struct Case { int grid, mode; } cases[] = {{256, 0}, {260, 0}, {264, 0}, {256, 1}, {264, 1}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto c : cases) {
      const int N = 3000;
      for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_slice, dim3(c.grid), dim3(128), 0, s, buf, out, c.mode, nullptr, -1);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_slice, dim3(c.grid), dim3(128), 0, s, buf, out, c.mode, nullptr, -1);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"probe\": \"slice\", \"grid\": %d, \"mode\": \"%s\", \"us_per_launch\": %.3f}\n", c.grid,
             c.mode ? "xcc-stable" : "blockIdx", ms * 1e3 / N);
    }
  for (int gi = 0; gi < 3; ++gi) {   // XCC id of every workgroup over 8 consecutive launches
    const int grid = gi == 0 ? 256 : gi == 1 ? 260 : 264;
    for (int l = 0; l < 8; ++l) hipLaunchKernelGGL(k_slice, dim3(grid), dim3(128), 0, s, buf, out, 0, xlog, l);
    CHECK(hipStreamSynchronize(s));
    std::vector<int> h(16 * 1024);
    CHECK(hipMemcpy(h.data(), xlog, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    printf("{\"probe\": \"xcc_map\", \"grid\": %d, \"block0_xcc_per_launch\": [", grid);
    for (int l = 0; l < 8; ++l) printf("%d%s", h[l * 1024], l < 7 ? ", " : "");
    int rr = 1;                    // round robin within each launch: xcc(b) == (xcc(0) + b) % 8 ?
    for (int l = 0; l < 8; ++l)
      for (int b = 0; b < grid; ++b) rr &= h[l * 1024 + b] == (h[l * 1024] + b) % 8;
    printf("], \"round_robin\": %d}\n", rr);
  }
  // ---- 2. persistent iterations
  u64 *rows, *parts;
  int *nbr, *err;
  double* sink;
  CHECK(hipMalloc(&rows, (size_t)kG * kRows * 2 * sizeof(u64)));
  CHECK(hipMalloc(&parts, (size_t)kG * 3 * 2 * sizeof(u64)));
  CHECK(hipMalloc(&nbr, kG * kNb * sizeof(int)));
  CHECK(hipMalloc(&err, sizeof(int)));
  CHECK(hipMalloc(&sink, kG * sizeof(double)));
  {
    std::vector<int> h(kG * kNb);
    for (int g = 0; g < kG; ++g)
      for (int k = 0; k < kNb; ++k) h[g * kNb + k] = (g + (k - kNb / 2) * 3 + 2 * kG) % kG;   // spread neighbours
    CHECK(hipMemcpy(nbr, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_persist, 128, 0));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("{\"probe\": \"persist_occupancy\", \"blocks_per_cu\": %d, \"cus\": %d}\n", occ, prop.multiProcessorCount);
  if (occ * prop.multiProcessorCount < kG) { printf("not co-resident\n"); return 1; }
  const char* names[] = {"", "neighbour rows", "partials all-gather", "both"};
  for (int G : {260, 128, 64})
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 1; mode <= 3; ++mode) {
      {
        std::vector<int> h(kG * kNb);
        for (int g = 0; g < kG; ++g)
          for (int k = 0; k < kNb; ++k) h[g * kNb + k] = ((g + (k - kNb / 2) * 3) % G + 2 * G) % G;
        CHECK(hipMemcpy(nbr, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
      }
      float t[2];
      const int its[2] = {200, 1200};
      int bad = 0;
      for (int q = 0; q < 2; ++q) {
        CHECK(hipMemsetAsync(rows, 0, (size_t)kG * kRows * 2 * sizeof(u64), s));
        CHECK(hipMemsetAsync(parts, 0, (size_t)kG * 3 * 2 * sizeof(u64), s));
        CHECK(hipMemsetAsync(err, 0, sizeof(int), s));
        CHECK(hipEventRecord(e0, s));
        int it = its[q];
        void* args[] = {&rows, &parts, &nbr, &it, &mode, &err, &sink, &G};
        CHECK(hipLaunchCooperativeKernel((const void*)k_persist, dim3(G), dim3(128), args, 0, s));
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&t[q], e0, e1));
        int h = 0;
        CHECK(hipMemcpy(&h, err, sizeof(int), hipMemcpyDeviceToHost));
        bad |= h;
      }
      printf("{\"probe\": \"persist\", \"workgroups\": %d, \"wait_for\": \"%s\", \"us_per_iteration\": %.3f, "
             "\"timeout\": %d}\n", G, names[mode], (t[1] - t[0]) * 1e3 / (its[1] - its[0]), bad);
    }
  return 0;
}
