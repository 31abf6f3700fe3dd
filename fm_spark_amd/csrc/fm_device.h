// Device helpers shared by the step kernels (fm_kernels.hip) and the sharded path
// (fm_shard.hip).
#pragma once

#include "fm_internal.h"

namespace fmhip {

// Plain cached loads and stores throughout: nontemporal variants of the row write-back, the sorted
// entry stream, the CSR stream and the sort's streams were measured (round 2) and
// were neutral or slower in the step.

// Block barrier that orders LDS only: the waits it implies are lgkmcnt, not vmcnt, so global
// loads issued ahead and global stores still draining stay in flight across it (__syncthreads'
// workgroup fence waits for every outstanding global access of the wave).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void st_row4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ float shrink_f(float z, double a) {
  // signum(z) * max(0, |z| - a) (FactorizationMachinesSGD.scala:104, :179), in fp64.
  const double az = fabs((double)z) - a;
  return az > 0.0 ? (float)copysign(az, (double)z) : 0.0f * z;
}

__device__ __forceinline__ double shrink_d(double z, double a) {
  const double az = fabs(z) - a;
  return az > 0.0 ? copysign(az, z) : 0.0 * z;
}

__device__ __forceinline__ float4 shrink4(float4 v, double a) {
  return make_float4(shrink_f(v.x, a), shrink_f(v.y, a), shrink_f(v.z, a), shrink_f(v.w, a));
}

// fp32 soft-threshold, for the row catch-up and the update's final rounding: the operands are
// fp32 values and fp32-rounded shrink amounts, the result differs from the fp64 form by at most
// one rounding of the fp32 result.
__device__ __forceinline__ float shrink1f(float z, float a) { return copysignf(fmaxf(fabsf(z) - a, 0.f), z); }
__device__ __forceinline__ float4 shrink4f(float4 v, float a) {
  return make_float4(shrink1f(v.x, a), shrink1f(v.y, a), shrink1f(v.z, a), shrink1f(v.w, a));
}

// Inclusive segmented scan over lanes [start_lane, lane] in a fixed tree order.  nsteps is the
// wave-uniform depth the longest piece needs; the skipped steps would add nothing, so the
// result is bitwise that of the full 6-step scan.
__device__ __forceinline__ double seg_scan(double v, int lane, int start_lane, int nsteps) {
  for (int i = 0; i < nsteps; ++i) {
    const int o = 1 << i;
    const double t = __shfl_up(v, o);
    if (lane - o >= start_lane) v += t;
  }
  return v;
}

// Header store that completes the 64-B memory granule holding it: the header, then zero
// padding to the granule's end.  A partly written granule costs a read-modify-write in HBM
// (measured on MI355X, tools/traffic_cal.hip: random 80-B row writes 0.58 ms per 10M rows, the
// same rows written as whole 128-B lines 0.37 ms); the V quads that share the granule are
// written by the same kernel, so the granule leaves L2 whole.
__device__ __forceinline__ void store_hdr(const TableView& T, int64_t slot, const RowHdr& o) {
  float* r = T.rec + slot * T.stride + T.kp;
  *reinterpret_cast<RowHdr*>(r) = o;
  const int pad = (16 - ((T.kp + 4) & 15)) & 15;  // floats from the header's end to the granule's
  for (int i = 0; i < pad; i += 4) *reinterpret_cast<float4*>(r + 4 + i) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Row update of SGD.scala:150-181, fp64:
//   vec' = S_lambda(vec - sum * (eta / m));  strength' = S_lambda(strength - (sum / m) * eta)
__device__ __forceinline__ float upd_v(float v, double g, const StepParams& p) {
  return (float)shrink_d((double)v - g * p.scale_v, p.lam);
}
__device__ __forceinline__ float upd_w(float w, double g, const StepParams& p) {
  return (float)shrink_d((double)w - (g / p.m) * p.eta, p.lam);
}

}  // namespace fmhip
