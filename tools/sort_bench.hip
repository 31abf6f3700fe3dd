// Measurement tool (not product): time the library's LSD sort against rocPRIM's device radix sort
// on the same 10M (uint32 key, uint64 payload) pairs, 27-bit keys, and check its output against it.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../fm_spark_amd/csrc/fm_internal.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_gather_payload(const uint32_t* __restrict__ idx, const uint2* __restrict__ ent, uint2* __restrict__ out,
                                 int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = ent[idx[i]];
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 10223616;
  const int bits = argc > 2 ? atoi(argv[2]) : 27;
  std::mt19937_64 rng(1);
  std::vector<uint32_t> keys(n);
  std::vector<uint2> vals(n);
  // skew: 0 = 40% of keys from 1000 hot keys, the rest uniform; 1 = uniform; 2 = 60% on one key
  const int skew = argc > 3 ? atoi(argv[3]) : 0;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t r = rng();
    const uint32_t uni = (uint32_t)((r >> 8) % (1ull << bits));
    if (skew == 0)
      keys[i] = (r % 10 < 4) ? (uint32_t)((r >> 8) % 1000) * 99991u % (1u << bits) : uni;
    else if (skew == 2)
      keys[i] = (r % 10 < 6) ? 12345u % (1u << bits) : uni;
    else if (skew == 3) {  // c3-like: 39 fields, rank with the Zipf(1.05) tail P(rank >= r) = r^-0.05, hashed
      const double u = (double)(rng() >> 11) * (1.0 / 9007199254740992.0);
      double rk = std::pow(1.0 - u, -20.0);
      if (rk > 1e12) rk = 1e12;
      uint64_t z = ((uint64_t)(i % 39) << 40) + (uint64_t)rk + 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      keys[i] = (uint32_t)(z % (1ull << bits));
    }
    else
      keys[i] = uni;
    vals[i] = make_uint2((uint32_t)i, (uint32_t)(r >> 32));
  }
  uint32_t *dk, *dk2;
  uint2 *dv, *dv2;
  CK(hipMalloc(&dk, 4 * n)); CK(hipMalloc(&dk2, 4 * n));
  CK(hipMalloc(&dv, 8 * n)); CK(hipMalloc(&dv2, 8 * n));
  CK(hipMemcpy(dk, keys.data(), 4 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, vals.data(), 8 * n, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  // rocPRIM
  size_t tmp = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tmp, dk, dk2, dv, dv2, (size_t)n, 0, bits, st));
  void* dtmp;
  CK(hipMalloc(&dtmp, tmp));
  for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_pairs(dtmp, tmp, dk, dk2, dv, dv2, (size_t)n, 0, bits, st));
  const int R = 20;
  CK(hipEventRecord(a, st));
  for (int r = 0; r < R; ++r) CK(rocprim::radix_sort_pairs(dtmp, tmp, dk, dk2, dv, dv2, (size_t)n, 0, bits, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("rocprim radix_sort_pairs n=%lld bits=%d: %.3f ms\n", (long long)n, bits, ms / R);
  // ours: the LSD passes (mode 0; the multi-view check below served the bucket sort's split, removed)
  std::vector<uint32_t> k1(n), k2(n);
  std::vector<uint2> v1(n), v2(n);
  CK(hipMemcpy(k1.data(), dk2, 4 * n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(v1.data(), dv2, 8 * n, hipMemcpyDeviceToHost));
  std::vector<uint32_t> mk;
  std::vector<uint2> mv;
  int64_t singles = 0;
  for (int64_t i = 0; i < n; ++i) {
    const bool m = (i > 0 && k1[i - 1] == k1[i]) || (i + 1 < n && k1[i + 1] == k1[i]);
    if (m) {
      mk.push_back(k1[i]);
      mv.push_back(v1[i]);
    } else {
      ++singles;
    }
  }
  int64_t bad_total = 0;
  uint32_t* fk;
  uint2* fv;
  int64_t* dn;
  CK(hipMalloc(&fk, 4 * n));
  CK(hipMalloc(&fv, 8 * n));
  CK(hipMalloc(&dn, 16));
  for (int mode = 0; mode < 1; ++mode) {  // (modes 1-2 timed the bucket sort, removed in round 5)
    fmhip::SortWork sw;
    const uint32_t* ok = fk;
    const uint2* ov = fv;
    auto run = [&] { fmhip::radix_sort_pairs64(sw, dk, dv, n, bits, st, &ok, &ov); };
    for (int w = 0; w < 3; ++w) run();
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; ++r) run();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    const char* nm = mode == 0 ? "lsd" : mode == 1 ? "bucket" : "bucket-split";
    printf("fm_hip %s n=%lld bits=%d skew=%d: %.3f ms\n", nm, (long long)n, bits, skew, ms / R);
    int64_t cnt = n, hn[2] = {0, 0};
    if (mode == 2) {
      CK(hipMemcpy(hn, dn, 16, hipMemcpyDeviceToHost));
      cnt = hn[0];
    }
    CK(hipMemcpy(k2.data(), ok, 4 * cnt, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v2.data(), ov, 8 * cnt, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    const std::vector<uint32_t>& wk = mode == 2 ? mk : k1;
    const std::vector<uint2>& wv = mode == 2 ? mv : v1;
    if (mode == 2 && (hn[0] != (int64_t)mk.size() || hn[1] != singles)) {
      printf("split counts %lld / %lld, expected %lld / %lld\n", (long long)hn[0], (long long)hn[1],
             (long long)mk.size(), (long long)singles);
      bad += 1;
    }
    for (int64_t i = 0; i < (int64_t)wk.size() && i < cnt; ++i)
      bad += (wk[i] != k2[i]) || (wv[i].x != v2[i].x) || (wv[i].y != v2[i].y);
    printf("mismatches vs rocprim (%s): %lld\n", nm, (long long)bad);
    bad_total += bad;
  }
  if (getenv("SORT_CHECK_ONLY")) return bad_total ? 1 : 0;
  // rocPRIM keys-only sort of packed 64-bit words (key << 24 | entry index): one stream per pass
  {
    std::vector<uint64_t> pk(n);
    for (int64_t i = 0; i < n; ++i) pk[i] = ((uint64_t)keys[i] << 24) | (uint64_t)i;
    uint64_t *dp, *dp2;
    CK(hipMalloc(&dp, 8 * n)); CK(hipMalloc(&dp2, 8 * n));
    CK(hipMemcpy(dp, pk.data(), 8 * n, hipMemcpyHostToDevice));
    size_t tmp2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tmp2, dp, dp2, (size_t)n, 24, 24 + bits, st));
    void* dtmp2;
    CK(hipMalloc(&dtmp2, tmp2));
    for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_keys(dtmp2, tmp2, dp, dp2, (size_t)n, 24, 24 + bits, st));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; ++r) CK(rocprim::radix_sort_keys(dtmp2, tmp2, dp, dp2, (size_t)n, 24, 24 + bits, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("rocprim radix_sort_keys uint64 (key<<24|index) bits 24..%d: %.3f ms\n", 24 + bits, ms / R);
    // 16-byte pairs: 4-B key + 16-B payload would be one more stream; here 4-B keys only
    CK(hipEventRecord(a, st));
    size_t tmp3 = 0;
    uint32_t* dk3;
    CK(hipMalloc(&dk3, 4 * n));
    CK(rocprim::radix_sort_keys(nullptr, tmp3, dk, dk3, (size_t)n, 0, bits, st));
    void* dtmp3;
    CK(hipMalloc(&dtmp3, tmp3));
    for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_keys(dtmp3, tmp3, dk, dk3, (size_t)n, 0, bits, st));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; ++r) CK(rocprim::radix_sort_keys(dtmp3, tmp3, dk, dk3, (size_t)n, 0, bits, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("rocprim radix_sort_keys uint32 bits 0..%d: %.3f ms\n", bits, ms / R);
  }
  // (key, index) sort + payload gather
  {
    fmhip::SortWork sw2;
    const uint32_t* ok2;
    const uint32_t* oi2;
    uint2* dg;
    CK(hipMalloc(&dg, 8 * n));
    auto run = [&] {
      fmhip::radix_sort_pairs(sw2, dk, nullptr, n, bits, st, &ok2, &oi2);
      hipLaunchKernelGGL(k_gather_payload, dim3(4096), dim3(256), 0, st, oi2, dv, dg, n);
    };
    for (int w = 0; w < 3; ++w) run();
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; ++r) run();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("fm_hip radix_sort_pairs(key, index) + payload gather n=%lld: %.3f ms\n", (long long)n, ms / R);
    std::vector<uint2> v3(n);
    CK(hipMemcpy(v3.data(), dg, 8 * n, hipMemcpyDeviceToHost));
    int64_t bad3 = 0;
    for (int64_t i = 0; i < n; ++i) bad3 += (v1[i].x != v3[i].x) || (v1[i].y != v3[i].y);
    printf("mismatches (index sort + gather vs rocprim): %lld\n", (long long)bad3);
  }
  return 0;
}
