// Measurement tool (not product): calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// patterns of the FM kernels (MI355X_MICROARCH.md: "calibrate on a known byte count in your own
// access pattern").  Table of 100M records x 128 B (the k = 16 record stride), n = 10.2M random
// record indices (no reuse to speak of).  Kernels, one launch each, known bytes printed:
//   rd64   4 lanes x 16 B read the record's first 64 B (V row)
//   rd80   rd64 + one lane reads the 16-B header at +64 (the forward's / update's row read)
//   wr80   the same 80 B written (the update's row write-back)
//   stream 16 B/lane coalesced read of 1.28 GB (the guide's reference pattern)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int64_t kRows = 100000000, kStride = 32;  // floats per record (128 B)

template <int MODE>
__global__ __launch_bounds__(256) void k_rows(float* tab, const uint32_t* __restrict__ idx, int64_t n, float4* out) {
  const int g = threadIdx.x & 3;
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
  const int64_t ngrp = (int64_t)gridDim.x * 64;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t i = grp; i < n; i += ngrp) {
    float* rec = tab + (int64_t)idx[i] * kStride;
    if (MODE == 2) {  // 64 B V + 16 B header, separate instructions (the update's write-back)
      reinterpret_cast<float4*>(rec)[g] = make_float4(1.f, 2.f, 3.f, (float)i);
      if (g == 0) reinterpret_cast<float4*>(rec + 16)[0] = make_float4(5.f, 6.f, 7.f, 8.f);
    } else if (MODE == 3) {  // 64 B only
      reinterpret_cast<float4*>(rec)[g] = make_float4(1.f, 2.f, 3.f, (float)i);
    } else if (MODE == 4) {  // 64 B + 32 B (header + 16 B pad)
      reinterpret_cast<float4*>(rec)[g] = make_float4(1.f, 2.f, 3.f, (float)i);
      if (g < 2) reinterpret_cast<float4*>(rec + 16)[g] = make_float4(5.f, 6.f, 7.f, 8.f);
    } else if (MODE == 5) {  // full 128-B line: 64 B, then 64 B (header + pad) by the same 4 lanes
      reinterpret_cast<float4*>(rec)[g] = make_float4(1.f, 2.f, 3.f, (float)i);
      reinterpret_cast<float4*>(rec + 16)[g] = make_float4(5.f, 6.f, 7.f, 8.f);
    } else {
      float4 v = reinterpret_cast<const float4*>(rec)[g];
      if (MODE == 1 && g == 0) {
        const float4 h = reinterpret_cast<const float4*>(rec + 16)[0];
        v.x += h.x; v.y += h.y;
      }
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  if (MODE != 2) out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ a, int64_t n4, float4* out) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = a[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int64_t n = 10223616;
  float* tab; float4* out; uint32_t* idx;
  CK(hipMalloc(&tab, kRows * kStride * 4));
  CK(hipMemset(tab, 0, kRows * kStride * 4));
  CK(hipMalloc(&out, 4096 * 256 * 16));
  CK(hipMalloc(&idx, 4 * n));
  std::mt19937_64 rng(11);
  std::vector<uint32_t> h(n);
  for (auto& x : h) x = (uint32_t)(rng() % kRows);
  CK(hipMemcpy(idx, h.data(), 4 * n, hipMemcpyHostToDevice));
  const int grid = 4096;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms;
#define TIME(name, bytes, launch) do { launch; CK(hipDeviceSynchronize()); CK(hipEventRecord(a)); launch; \
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); \
    printf("%-8s known %.1f MB per launch  %.3f ms  %.0f GB/s\n", name, (bytes) / 1e6, ms, (bytes) / ms / 1e6); } while (0)
  TIME("rd64", n * 64.0, hipLaunchKernelGGL(k_rows<0>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  TIME("rd80", n * 80.0, hipLaunchKernelGGL(k_rows<1>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  TIME("wr80", n * 80.0, hipLaunchKernelGGL(k_rows<2>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  TIME("wr64", n * 64.0, hipLaunchKernelGGL(k_rows<3>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  TIME("wr96", n * 96.0, hipLaunchKernelGGL(k_rows<4>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  TIME("wr128", n * 128.0, hipLaunchKernelGGL(k_rows<5>, dim3(grid), dim3(256), 0, 0, tab, idx, n, out));
  const int64_t n4 = 1280000000 / 16;
  TIME("stream", n4 * 16.0, hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const float4*)tab, n4, out));
  CK(hipDeviceSynchronize());
  return 0;
}
