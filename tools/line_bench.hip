// Measurement tool (not product): random gathers of 128-B row records (V 64 B + 16-B header +
// pad, the k = 16 table layout of DESIGN §2) in the instruction shapes the forward could use.
//   A  two loads per row: V as float4 by 4 lanes, header 16 B by the same 4 lanes (k_forward now)
//   B  one load per row: 8 lanes per row, lanes 0-3 V quads, lane 4 the header, lanes 5-7 idle
//   C  V only, 4 lanes per row (lower bound: no header)
//   D  one load per row: 5 lanes of 16 B (V + header), 12 rows per wave, 4 lanes idle
// Index streams: uniform over the table, and Zipf-like (40 % of picks from 1000 hot rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int kU = 4;

template <int MODE>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ tab, const uint32_t* __restrict__ idx,
                                              int64_t n, float4* __restrict__ out) {
  constexpr int LPR = MODE == 0 ? 4 : MODE == 1 ? 8 : MODE == 2 ? 4 : 5;
  constexpr int RPW = 64 / LPR;  // rows per wave-instruction
  const int lane = threadIdx.x & 63;
  const int g = lane % LPR;
  const int slot = lane / LPR;
  const bool act = slot < RPW;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int64_t i = wave * RPW * kU; i < n; i += nwaves * RPW * kU) {
    uint32_t r[kU];
    bool ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t e = i + (int64_t)u * RPW + slot;
      ok[u] = act && e < n;
      r[u] = ok[u] ? idx[e] : 0u;
    }
    float4 v[kU], h[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const float4* row = tab + (int64_t)r[u] * 8;
      if (MODE == 0) {
        v[u] = ok[u] ? row[g] : make_float4(0, 0, 0, 0);
        h[u] = ok[u] ? row[4] : make_float4(0, 0, 0, 0);
      } else if (MODE == 1) {
        v[u] = (ok[u] && g <= 4) ? row[g] : make_float4(0, 0, 0, 0);
        h[u] = make_float4(0, 0, 0, 0);
      } else if (MODE == 2) {
        v[u] = ok[u] ? row[g] : make_float4(0, 0, 0, 0);
        h[u] = make_float4(0, 0, 0, 0);
      } else {
        v[u] = ok[u] ? row[g] : make_float4(0, 0, 0, 0);
        h[u] = make_float4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      acc.x += v[u].x + h[u].x; acc.y += v[u].y + h[u].y;
      acc.z += v[u].z + h[u].z; acc.w += v[u].w + h[u].w;
    }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// random record writes.  MODE 0: V by 4 lanes + header by 1 lane (two stores, 80 B);
// 1: 5 lanes one store (80 B); 2: 8 lanes one store (whole 128-B line, pad written);
// 3: 4 lanes, two float4 stores each (quads g and g + 4: whole line in two instructions);
// 4: read V + header (two loads), write them back (two stores): the update's row RMW;
// 5: read as 4, write the whole line with 8 lanes
template <int MODE>
__global__ __launch_bounds__(256) void scatter(float4* __restrict__ tab, const uint32_t* __restrict__ idx, int64_t n) {
  constexpr int LPR = (MODE == 0 || MODE == 3 || MODE == 4) ? 4 : 8;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane % LPR;
  const int slot = lane / LPR;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t i = wave * RPW; i < n; i += nwaves * RPW) {
    const int64_t e = i + slot;
    if (e >= n) continue;
    float4* row = tab + (int64_t)idx[e] * 8;
    float4 val = make_float4((float)g, 1.f, 2.f, 3.f);
    if (MODE == 0) {
      row[g] = val;
      if (g == 0) row[4] = val;
    } else if (MODE == 1) {
      if (g <= 4) row[g] = val;
    } else if (MODE == 2) {
      row[g] = val;
    } else if (MODE == 3) {
      row[g] = val;
      row[g + 4] = val;
    } else if (MODE == 4) {
      float4 v = row[g];
      float4 h = row[4];
      v.x += 1.f; h.x += 1.f;
      row[g] = v;
      if (g == 0) row[4] = h;
    } else {
      float4 v = row[g & 3];
      float4 h = row[4];
      v.x += h.y;
      row[g] = g < 4 ? v : (g == 4 ? h : make_float4(0, 0, 0, 0));
    }
  }
}

template <class F>
float time_it(F f, hipStream_t st) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) f();
  CK(hipEventRecord(a, st));
  const int R = 10;
  for (int r = 0; r < R; ++r) f();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / R;
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 100000000;
  const int64_t n = 10223616;
  float4* tab; float4* out; uint32_t* idx;
  CK(hipMalloc(&tab, rows * 128 + 128));
  CK(hipMemset(tab, 0, rows * 128));
  CK(hipMalloc(&out, 256 * 2048 * 16));
  CK(hipMalloc(&idx, 4 * n));
  std::mt19937_64 rng(7);
  std::vector<uint32_t> h(n);
  hipStream_t st; CK(hipStreamCreate(&st));
  const int grid = 2048;
  const char* names[4] = {"A V+hdr two loads", "B 8 lanes one load", "C V only", "D 5 lanes one load"};
  for (int mode = 0; mode < 2; ++mode) {
    for (int64_t i = 0; i < n; ++i) {
      uint64_t r = rng();
      h[i] = (mode == 0) ? (uint32_t)(r % rows)
                         : ((r % 10 < 4) ? (uint32_t)((r >> 8) % 1000 * 99991u % rows) : (uint32_t)((r >> 8) % rows));
    }
    CK(hipMemcpy(idx, h.data(), 4 * n, hipMemcpyHostToDevice));
    const char* dist = mode == 0 ? "uniform" : "40% hot";
    float t[4];
    t[0] = time_it([&] { hipLaunchKernelGGL(gather<0>, dim3(grid), dim3(256), 0, st, tab, idx, n, out); }, st);
    t[1] = time_it([&] { hipLaunchKernelGGL(gather<1>, dim3(grid), dim3(256), 0, st, tab, idx, n, out); }, st);
    t[2] = time_it([&] { hipLaunchKernelGGL(gather<2>, dim3(grid), dim3(256), 0, st, tab, idx, n, out); }, st);
    t[3] = time_it([&] { hipLaunchKernelGGL(gather<3>, dim3(grid), dim3(256), 0, st, tab, idx, n, out); }, st);
    for (int m = 0; m < 4; ++m)
      printf("gather  %-8s %-20s %.3f ms  %.2f G rows/s\n", dist, names[m], t[m], n / t[m] / 1e6);
    const char* snames[6] = {"V + hdr, two stores", "5 lanes, one store", "8 lanes, whole line",
                             "4 lanes x 2 stores", "RMW V+hdr (update)", "RMW, whole-line store"};
    float s[6];
    s[0] = time_it([&] { hipLaunchKernelGGL(scatter<0>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    s[1] = time_it([&] { hipLaunchKernelGGL(scatter<1>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    s[2] = time_it([&] { hipLaunchKernelGGL(scatter<2>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    s[3] = time_it([&] { hipLaunchKernelGGL(scatter<3>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    s[4] = time_it([&] { hipLaunchKernelGGL(scatter<4>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    s[5] = time_it([&] { hipLaunchKernelGGL(scatter<5>, dim3(grid), dim3(256), 0, st, tab, idx, n); }, st);
    for (int m = 0; m < 6; ++m)
      printf("scatter %-8s %-24s %.3f ms  %.2f G rows/s\n", dist, snames[m], s[m], n / s[m] / 1e6);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
