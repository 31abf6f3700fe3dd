// Measurement tool (not product): the memory floor of the update's row traffic.
// Table 100M records x 128 B (the k = 16 record stride).  U = 6M distinct rows, visited in
// ascending slot order (as the sorted update visits them) or in random order.  One 8-lane group
// per row, 16 B per lane (the whole 128-B line), U rows in flight per group.
//   rd   : read the line
//   wr   : write the line
//   rmw  : read, modify, write the line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int64_t kRows = 100000000;

template <int MODE, int LPR, int UF>
__global__ __launch_bounds__(256) void k_rows(float4* tab, const uint32_t* __restrict__ idx, int64_t n, float4* out) {
  const int g = threadIdx.x % LPR;
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int64_t ngrp = (int64_t)gridDim.x * 256 / LPR;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t i = grp * UF; i < n; i += ngrp * UF) {
    uint32_t r[UF];
#pragma unroll
    for (int u = 0; u < UF; ++u) r[u] = i + u < n ? idx[i + u] : 0xFFFFFFFFu;
    float4 v[UF];
    if (MODE != 1) {
#pragma unroll
      for (int u = 0; u < UF; ++u) v[u] = r[u] != 0xFFFFFFFFu ? tab[(int64_t)r[u] * 8 + g] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      if (MODE == 0) {
        acc.x += v[u].x; acc.y += v[u].y;
      } else if (r[u] != 0xFFFFFFFFu) {
        float4 w = MODE == 1 ? make_float4(1.f, 2.f, 3.f, (float)i) : make_float4(v[u].x * 0.5f, v[u].y + 1.f, v[u].z, v[u].w);
        tab[(int64_t)r[u] * 8 + g] = w;
      }
    }
  }
  if (MODE == 0) out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int64_t U = argc > 1 ? atoll(argv[1]) : 6000000;
  float4* tab; float4* out; uint32_t* idx;
  CK(hipMalloc(&tab, kRows * 128));
  CK(hipMemset(tab, 0, kRows * 128));
  CK(hipMalloc(&out, 4096 * 256 * 16));
  CK(hipMalloc(&idx, 4 * U));
  std::mt19937_64 rng(5);
  std::vector<uint32_t> h(U);
  for (auto& x : h) x = (uint32_t)(rng() % kRows);
  std::sort(h.begin(), h.end());
  h.erase(std::unique(h.begin(), h.end()), h.end());
  const int64_t n = (int64_t)h.size();
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms;
  const int grid = 4096;
  for (int order = 0; order < 2; ++order) {
    if (order == 1) std::shuffle(h.begin(), h.end(), rng);
    CK(hipMemcpy(idx, h.data(), 4 * n, hipMemcpyHostToDevice));
    const char* on = order == 0 ? "sorted" : "random";
#define TIME(name, launch) do { launch(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a)); for (int r_ = 0; r_ < 5; ++r_) launch(); \
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); ms /= 5; \
    printf("%-6s %-10s rows %lld  %.3f ms  %.2f Grows/s  %.0f GB/s of lines\n", on, name, (long long)n, ms, n / ms / 1e6, n * 128.0 / ms / 1e6); } while (0)
    TIME("rd U1", ([&] { k_rows<0, 8, 1><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("rd U4", ([&] { k_rows<0, 8, 4><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("wr U1", ([&] { k_rows<1, 8, 1><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("wr U4", ([&] { k_rows<1, 8, 4><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("rmw U1", ([&] { k_rows<2, 8, 1><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("rmw U4", ([&] { k_rows<2, 8, 4><<<grid, 256>>>(tab, idx, n, out); }));
    TIME("rmw4 U4", ([&] { k_rows<2, 4, 4><<<grid, 256>>>(tab, idx, n, out); }));
  }
  return 0;
}
