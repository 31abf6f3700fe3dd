// Measurement tool (not product): achievable rate of random row gathers on this GPU.
// table of R rows x W bytes; each lane-group (W/16 lanes) fetches one random row per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int LPR, int U>  // lanes per row (16 B each), rows in flight per lane-group
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ tab, const uint32_t* __restrict__ idx,
                                              int64_t n, float4* __restrict__ out) {
  const int g = threadIdx.x % LPR;
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int64_t ngrp = (int64_t)gridDim.x * 256 / LPR;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t i = grp * U; i < n; i += ngrp * U) {
    uint32_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = (i + u < n) ? idx[i + u] : 0;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[(int64_t)r[u] * LPR + g];
#pragma unroll
    for (int u = 0; u < U; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int LPR, int U>
void run(const char* name, const float4* tab, const uint32_t* idx, int64_t n, float4* out, hipStream_t st) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int grid = 256 * 16;
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((gather<LPR, U>), dim3(grid), dim3(256), 0, st, tab, idx, n, out);
  CK(hipEventRecord(a, st));
  const int R = 10;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL((gather<LPR, U>), dim3(grid), dim3(256), 0, st, tab, idx, n, out);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= R;
  printf("%-28s LPR=%2d U=%d: %.3f ms  %.2f Grows/s  %.0f GB/s (useful)\n", name, LPR, U, ms, n / ms / 1e6,
         n * 16.0 * LPR / ms / 1e6);
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 100000000;
  const int64_t n = 10223616;
  float4* tab; float4* out; uint32_t* idx;
  CK(hipMalloc(&tab, rows * 64 + 64));
  CK(hipMemset(tab, 0, rows * 64));
  CK(hipMalloc(&out, 256 * 16 * 256 * 16));
  CK(hipMalloc(&idx, 4 * n));
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h(n);
  hipStream_t st; CK(hipStreamCreate(&st));
  for (int mode = 0; mode < 2; ++mode) {
    for (int64_t i = 0; i < n; ++i) {
      uint64_t r = rng();
      h[i] = (mode == 0) ? (uint32_t)(r % rows) : ((r % 10 < 4) ? (uint32_t)((r >> 8) % 1000 * 99991u % rows) : (uint32_t)((r >> 8) % rows));
    }
    CK(hipMemcpy(idx, h.data(), 4 * n, hipMemcpyHostToDevice));
    const char* nm = mode == 0 ? "uniform random rows" : "40% hot rows";
    run<4, 1>(nm, tab, idx, n, out, st);
    run<4, 4>(nm, tab, idx, n, out, st);
    run<4, 8>(nm, tab, idx, n, out, st);
    run<1, 4>(nm, tab, idx, n, out, st);
    run<1, 8>(nm, tab, idx, n, out, st);
  }
  return 0;
}
