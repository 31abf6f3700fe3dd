// Measurement tool (not product): the L2 request rate that random row gathers saturate on this GPU,
// for the ceiling bench.py's roofline.requests quotes (profiles/gather_ceiling.json).
//
// A table of R records of STRIDE floats (R = 100M at STRIDE 32: the c3 table's 128-B records), and
// 10.2M random record indices (a c3 batch's entries): uniform, or 40 % of them on 1000 hot rows.
// Each lane group of LPR lanes (16 B each) gathers U records in flight, as the step's forward does.
// Every variant is its own kernel instantiation (the MODE argument only names it), launched 2 + 10
// times; the tool prints the event time per launch; tools/gather_ceiling.py joins it with the
// TCC_HIT + TCC_MISS counts of a rocprofv3 --pmc pass over the same binary.
//
// With a stream file (argv[2], tools/c3_stream.py: one c3 batch's row_ptr and feature ids in CSR
// order, bit 31 = the id has one entry in the batch) two more variants replay c3's own forward
// address stream: MODE 2 gathers its ids in CSR order (as the uniform variants do), MODE 3
// (`gather_skel`) is the fused forward's memory skeleton without its arithmetic -- one wave per
// sample, its row_ptr, ids and x read, every row's whole 128-B record gathered (8 lanes x 16 B, all
// of a 39-entry sample's rows in flight), the singleton rows' records written back (one 8-lane
// store each) and the sample's 128-B S record written.  Its time is the floor of the forward's
// own access stream on this chip.
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


// MODE 3: the fused forward's memory skeleton over c3's own stream (see the header)
template <int LPR, int U, int STRIDE, int MODE>
__global__ __launch_bounds__(256) void gather_skel(float4* __restrict__ tab, const int64_t* __restrict__ rp,
                                                   const uint32_t* __restrict__ col, const float* __restrict__ xs,
                                                   int64_t B, float4* __restrict__ srec) {
  constexpr int Q = STRIDE / 4;
  constexpr int RPP = 64 / LPR;  // rows per pass of the wave
  const int lane = threadIdx.x & 63;
  const int g = lane % LPR, row_in = lane / LPR;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const int64_t nwaves = (int64_t)gridDim.x * 256 / 64;
  for (int64_t s = wave; s < B; s += nwaves) {
    const int64_t e0 = rp[s], e1 = rp[s + 1];
    uint32_t id[U];
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u * RPP + row_in;
      id[u] = e < e1 ? col[e] : 0xFFFFFFFFu;
      x[u] = e < e1 ? xs[e] : 0.f;
    }
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = id[u] != 0xFFFFFFFFu ? tab[(int64_t)(id[u] & 0x7FFFFFFFu) * Q + g] : make_float4(0, 0, 0, 0);
    float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += v[u].x * x[u];
      acc.y += v[u].y * x[u];
      acc.z += v[u].z * x[u];
      acc.w += v[u].w * x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (id[u] != 0xFFFFFFFFu && (id[u] >> 31)) {
        float4 w = v[u];
        w.x += 1e-7f * acc.x;
        tab[(int64_t)(id[u] & 0x7FFFFFFFu) * Q + g] = w;
      }
    if (lane < Q) srec[s * Q + lane] = acc;
  }
}


// MODE 4: the same skeleton in the forward's lane shape -- 4 lanes per row carry the 64-B V quads, the
// 16-B header is a second load (every lane of the group), a singleton's record leaves as V (4 lanes)
// plus header + pad (4 lanes) in two stores: what the shape costs against the 8-lane whole-record one
template <int LPR, int U, int STRIDE, int MODE>
__global__ __launch_bounds__(256) void gather_skel4(float4* __restrict__ tab, const int64_t* __restrict__ rp,
                                                    const uint32_t* __restrict__ col, const float* __restrict__ xs,
                                                    int64_t B, float4* __restrict__ srec) {
  constexpr int Q = STRIDE / 4;
  constexpr int RPP = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane % LPR, row_in = lane / LPR;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const int64_t nwaves = (int64_t)gridDim.x * 256 / 64;
  for (int64_t s = wave; s < B; s += nwaves) {
    const int64_t e0 = rp[s], e1 = rp[s + 1];
    uint32_t id[U];
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u * RPP + row_in;
      id[u] = e < e1 ? col[e] : 0xFFFFFFFFu;
      x[u] = e < e1 ? xs[e] : 0.f;
    }
    float4 v[U], h[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = id[u] != 0xFFFFFFFFu;
      const int64_t r = (int64_t)(id[u] & 0x7FFFFFFFu) * Q;
      h[u] = ok ? tab[r + 4] : make_float4(0, 0, 0, 0);
      v[u] = ok ? tab[r + g] : make_float4(0, 0, 0, 0);
    }
    float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += v[u].x * x[u] + h[u].x;
      acc.y += v[u].y * x[u];
      acc.z += v[u].z * x[u];
      acc.w += v[u].w * x[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (id[u] != 0xFFFFFFFFu && (id[u] >> 31)) {
        const int64_t r = (int64_t)(id[u] & 0x7FFFFFFFu) * Q;
        float4 w = v[u];
        w.x += 1e-7f * acc.x;
        tab[r + g] = w;
        tab[r + 4 + g] = g == 0 ? h[u] : make_float4(0, 0, 0, 0);
      }
    if (lane < Q) srec[s * Q + lane] = acc;
  }
}

template <int LPR, int U, int STRIDE, int MODE>
void run_skel(float4* tab, const int64_t* rp, const uint32_t* col, const float* xs, int64_t B, int64_t n,
              float4* srec, hipStream_t st) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 2048;
  auto launch = [&] {
    if (MODE == 4)
      hipLaunchKernelGGL((gather_skel4<LPR, U, STRIDE, MODE>), dim3(grid), dim3(256), 0, st, tab, rp, col, xs, B, srec);
    else
      hipLaunchKernelGGL((gather_skel<LPR, U, STRIDE, MODE>), dim3(grid), dim3(256), 0, st, tab, rp, col, xs, B, srec);
  };
  for (int w = 0; w < 2; ++w) launch();
  CK(hipEventRecord(a, st));
  const int R = 10;
  for (int r = 0; r < R; ++r) launch();
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
  if (argc > 2) {  // c3's own stream (tools/c3_stream.py)
    FILE* f = fopen(argv[2], "rb");
    if (!f) {
      printf("cannot open %s\n", argv[2]);
      return 1;
    }
    int64_t hdr[2];
    if (fread(hdr, sizeof(int64_t), 2, f) != 2) return 1;
    const int64_t B = hdr[0], N = hdr[1];
    if (N > n || B < 1) return 1;  // the index buffer holds a c3 batch's entries
    std::vector<int64_t> hrp(B + 1);
    std::vector<uint32_t> hcol(N);
    std::vector<float> hxs(N);
    if (fread(hrp.data(), sizeof(int64_t), B + 1, f) != (size_t)(B + 1) || fread(hcol.data(), 4, N, f) != (size_t)N ||
        fread(hxs.data(), 4, N, f) != (size_t)N)
      return 1;
    fclose(f);
    for (int64_t e = 0; e < N; ++e)
      if ((int64_t)(hcol[e] & 0x7FFFFFFFu) >= rows) return 1;
    int64_t* drp;
    uint32_t* dcol;
    float* dxs;
    float4* srec;
    CK(hipMalloc(&drp, 8 * (B + 1)));
    CK(hipMalloc(&dcol, 4 * N));
    CK(hipMalloc(&dxs, 4 * N));
    CK(hipMalloc(&srec, 128 * B));
    CK(hipMemcpy(drp, hrp.data(), 8 * (B + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(dcol, hcol.data(), 4 * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxs, hxs.data(), 4 * N, hipMemcpyHostToDevice));
    int64_t nsingle = 0;
    for (int64_t e = 0; e < N; ++e) {
      nsingle += hcol[e] >> 31;
      h[e] = hcol[e] & 0x7FFFFFFFu;
    }
    printf("STREAM rows=%ld entries=%ld singleton_entries=%ld\n", (long)B, (long)N, (long)nsingle);
    CK(hipMemcpy(idx, h.data(), 4 * N, hipMemcpyHostToDevice));
    run<4, 8, 32, 2>(tab, idx, N, out, st);  // c3's ids in CSR order: 64 B of each 128-B record
    run<8, 4, 32, 2>(tab, idx, N, out, st);  // the whole record
    run_skel<8, 5, 32, 3>(tab, drp, dcol, dxs, B, N, srec, st);  // the fused forward's memory skeleton
    run_skel<4, 3, 32, 4>(tab, drp, dcol, dxs, B, N, srec, st);  // the same in the forward's lane shape
    CK(hipFree(drp));
    CK(hipFree(dcol));
    CK(hipFree(dxs));
    CK(hipFree(srec));
  }
  CK(hipFree(tab));
  CK(hipFree(out));
  CK(hipFree(idx));
  return 0;
}
