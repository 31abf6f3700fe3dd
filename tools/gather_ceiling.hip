// Measurement tool (not product): the L2 request rate that random row gathers saturate on this GPU,
// for the ceiling bench.py's roofline.requests quotes (profiles/gather_ceiling.json).
//
// A table of R records of STRIDE floats (R = 100M at STRIDE 32: the c3 table's 128-B records), and
// 10.2M random record indices (a c3 batch's entries): uniform, or 40 % of them on 1000 hot rows.
// Each lane group of LPR lanes (16 B each) gathers U records in flight, as the step's forward does.
// Every variant is its own kernel instantiation (the MODE argument only names it), launched 2 + 10
// times; the tool prints the event time per launch; tools/gather_ceiling.py joins it with the
// TCC_HIT + TCC_MISS counts of a rocprofv3 --pmc pass over the same binary.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);               \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <int LPR, int U, int STRIDE, int MODE>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ tab, const uint32_t* __restrict__ idx, int64_t n,
                                              float4* __restrict__ out) {
  constexpr int Q = STRIDE / 4;  // float4 quads per record
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
    for (int u = 0; u < U; ++u) v[u] = tab[(int64_t)r[u] * Q + g];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += v[u].x;
      acc.y += v[u].y;
      acc.z += v[u].z;
      acc.w += v[u].w;
    }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int LPR, int U, int STRIDE, int MODE>
void run(const float4* tab, const uint32_t* idx, int64_t n, float4* out, hipStream_t st) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 2048;
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((gather<LPR, U, STRIDE, MODE>), dim3(grid), dim3(256), 0, st, tab, idx, n, out);
  CK(hipEventRecord(a, st));
  const int R = 10;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL((gather<LPR, U, STRIDE, MODE>), dim3(grid), dim3(256), 0, st, tab, idx, n, out);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= R;
  printf("VARIANT gather<%d, %d, %d, %d> ms=%.5f rows=%ld\n", LPR, U, STRIDE, MODE, ms, (long)n);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 100000000;
  const int64_t n = 10223616;  // a c3 batch's entries (256K rows x 39)
  float4* tab;
  float4* out;
  uint32_t* idx;
  CK(hipMalloc(&tab, rows * 128 + 128));
  CK(hipMemset(tab, 0, rows * 128));
  CK(hipMalloc(&out, 2048 * 256 * 16));
  CK(hipMalloc(&idx, 4 * n));
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h(n);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int mode = 0; mode < 2; ++mode) {
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t r = rng();
      h[i] = mode == 0 ? (uint32_t)(r % rows)
                       : ((r % 10 < 4) ? (uint32_t)((r >> 8) % 1000 * 99991u % rows) : (uint32_t)((r >> 8) % rows));
    }
    CK(hipMemcpy(idx, h.data(), 4 * n, hipMemcpyHostToDevice));
    if (mode == 0) {
      run<4, 8, 32, 0>(tab, idx, n, out, st);   // 64 B of a 128-B record (the forward's V quads)
      run<8, 4, 32, 0>(tab, idx, n, out, st);   // the whole 128-B record
      run<4, 8, 16, 0>(tab, idx, n, out, st);   // 64-B records
      run<1, 8, 32, 0>(tab, idx, n, out, st);   // 16 B of a 128-B record
    } else {
      run<4, 8, 32, 1>(tab, idx, n, out, st);
      run<8, 4, 32, 1>(tab, idx, n, out, st);
      run<4, 8, 16, 1>(tab, idx, n, out, st);
      run<1, 8, 32, 1>(tab, idx, n, out, st);
    }
  }
  CK(hipFree(tab));
  CK(hipFree(out));
  CK(hipFree(idx));
  return 0;
}
