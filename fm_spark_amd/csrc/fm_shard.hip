// Row-sharded FM SGD step (one context per rank, owner of feature id = id % R, local slot =
// id / R).  The fused single-table step of fm_kernels.hip split at its two data-dependence
// points so the caller can exchange over RCCL all-to-all between phases:
//
//   fm_shard_plan        sort the batch's entries by (owner, slot); dedupe -> request list
//                        (owner-major, one entry per distinct id) + each entry's unique index
//   -- all-to-all requests -->
//   fm_shard_serve       owner: gather the requested rows, pending L1 applied
//   -- all-to-all rows <--
//   fm_shard_local_grad  forward from the received rows + per-distinct-id partial gradient
//                        (segmented reduction over the plan's sorted order; fp64 sums, fp32 wire)
//   -- all-to-all gradients -->
//   fm_shard_apply       owner: merge the <= R partials per slot in fixed rank order, apply the
//                        update + L1 of SGD.scala:150-181, advance the epoch.
//
// Semantics equal the single-table step over the ranks' batches concatenated in rank order
// (global miniBatchSize m = sum of the ranks' rows), up to fp summation order.
// Wire formats: rows [V(kp) | w | 0 0 0] fp32, gradients [gV(kp) | gw | 0 0 0] fp32; kp + 4
// floats per distinct id.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "fm_context.h"
#include "fm_device.h"

namespace fmhip {

namespace {

constexpr int kBlock = 256;
constexpr int kTileS = 4096;  // entries per block in the run-index scan

__global__ void k_shard_keys(const uint32_t* __restrict__ col, int64_t n, uint32_t R, uint32_t rpsh,
                             uint32_t* __restrict__ ck) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t id = col[i];
    ck[i] = (id % R) * rpsh + id / R;
  }
}

__device__ __forceinline__ uint32_t run_flag(const uint32_t* skeys, int64_t p, int64_t n) {
  return (p < n && (p == 0 || skeys[p - 1] != skeys[p])) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_runs_count(const uint32_t* __restrict__ skeys, int64_t n,
                                                       uint32_t* __restrict__ bsum) {
  __shared__ uint32_t ws[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kTileS;
  uint32_t c = 0;
  for (int i = threadIdx.x; i < kTileS; i += kBlock) c += run_flag(skeys, base + i, n);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
    bsum[blockIdx.x] = t;
  }
}

// single block: exclusive scan of the block sums in place, total -> *total
__global__ __launch_bounds__(kBlock) void k_runs_scan(uint32_t* __restrict__ bsum, int64_t nb,
                                                      uint64_t* __restrict__ total) {
  __shared__ uint32_t ws[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t b = 0; b < nb; b += kBlock) {
    const int64_t i = b + threadIdx.x;
    const uint32_t v = i < nb ? bsum[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      pre += w < wave ? ws[w] : 0u;
      tot += ws[w];
    }
    if (i < nb) bsum[i] = carry + pre + inc - v;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// Per sorted position: run index (= distinct-id index u), the request list, each entry's
// unique index (CSR order) and the per-owner request counts.
__global__ __launch_bounds__(kBlock) void k_plan_apply(const uint32_t* __restrict__ skeys,
                                                       const uint32_t* __restrict__ sidx, int64_t n,
                                                       const uint32_t* __restrict__ boff, uint32_t rpsh, int R,
                                                       int32_t* __restrict__ req, uint32_t* __restrict__ run_of,
                                                       uint32_t* __restrict__ uidx,
                                                       unsigned long long* __restrict__ counts) {
  __shared__ uint32_t ws[kBlock / 64];
  __shared__ uint32_t ocount[1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = threadIdx.x; o < R; o += kBlock) ocount[o] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTileS;
  uint32_t carry = boff[blockIdx.x];
  for (int r = 0; r < kTileS / kBlock; ++r) {
    const int64_t p = base + (int64_t)r * kBlock + threadIdx.x;
    const uint32_t f = run_flag(skeys, p, n);
    uint32_t inc = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      pre += w < wave ? ws[w] : 0u;
      tot += ws[w];
    }
    if (p < n) {
      const uint32_t u = carry + pre + inc - 1u;  // run containing p
      const uint32_t key = skeys[p];
      run_of[p] = u;
      uidx[sidx[p]] = u;
      if (f) {
        req[u] = (int32_t)(key % rpsh);
        atomicAdd(&ocount[key / rpsh], 1u);
      }
    }
    carry += tot;
    __syncthreads();
  }
  for (int o = threadIdx.x; o < R; o += kBlock)
    if (ocount[o]) atomicAdd(&counts[o], (unsigned long long)ocount[o]);
}

// owner side: requested slots -> rows [V(kp) | w | 0 0 0], pending L1 applied
template <int G>
__global__ __launch_bounds__(kBlock) void k_shard_serve(TableView T, const int32_t* __restrict__ req, int64_t n,
                                                        double cumE, float* __restrict__ rows) {
  const int g = threadIdx.x % G;
  const int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  if (i >= n) return;
  const int kp = T.kp, nq = kp >> 2, RW = kp + 4;
  const int64_t slot = req[i];
  const RowHdr h = *T.hdr(slot);
  const bool present = h.t >= 0;
  const double a = present ? cumE - h.cum : 0.0;
  float* out = rows + i * RW;
  for (int q = g; q < nq; q += G) {
    float4 v = present ? reinterpret_cast<const float4*>(T.v(slot))[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (a > 0.0) v = shrink4(v, a);
    reinterpret_cast<float4*>(out)[q] = v;
  }
  if (g == 0) {
    float w = present ? h.w : 0.f;
    if (a > 0.0) w = shrink_f(w, a);
    reinterpret_cast<float4*>(out)[nq] = make_float4(w, 0.f, 0.f, 0.f);
  }
}

struct EmitArgs {
  const uint32_t* skeys;  // composite keys, sorted
  const uint32_t* sidx;   // entry index e per sorted position
  const uint32_t* run_of; // distinct-id index u per sorted position
  const uint2* ent;       // batch entries {sample, x}
  const float* rows;      // received rows [U][kp+4]
  const float* S;
  const float2* yl;
  float* grads;           // [U][kp+4]
  double* part;           // [nchunks][2][kp+1]
  int64_t N, nchunks;
  int kp;
};

// Per-distinct-id partial gradient of this rank's entries (the k_segment_update reduction
// with the row taken from the received rows and the result written out instead of applied).
template <int G>
__global__ __launch_bounds__(kBlock) void k_segment_emit(EmitArgs a) {
  constexpr int E = 64 / G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t chunk = (int64_t)blockIdx.x * (kBlock / 64) + wave;
  const int kp = a.kp, nq = kp >> 2, RW = kp + 4;
  const int64_t p0 = chunk * 64;
  const int64_t pp = p0 + lane;
  const bool valid = chunk < a.nchunks && pp < a.N;
  const uint32_t kNone = 0xFFFFFFFFu;
  const uint32_t key = valid ? a.skeys[pp] : kNone;
  const uint32_t e = valid ? a.sidx[pp] : 0u;
  const uint32_t u = valid ? a.run_of[pp] : 0u;
  uint32_t prev_key = __shfl_up(key, 1);
  uint32_t next_key = __shfl_down(key, 1);
  if (lane == 0) prev_key = (valid && p0 > 0) ? a.skeys[p0 - 1] : kNone;
  if (lane == 63) next_key = (valid && p0 + 64 < a.N) ? a.skeys[p0 + 64] : kNone;
  if (pp == a.N - 1) next_key = kNone;
  const uint2 en = valid ? a.ent[e] : make_uint2(0u, 0u);
  const int s = (int)en.x;
  const float xf = __uint_as_float(en.y);
  const double x = (double)xf;
  const float2 yl = valid ? a.yl[s] : make_float2(0.f, 0.f);

  const bool seg_start = valid && key != prev_key;
  const bool seg_end = valid && key != next_key;
  const bool piece_head = valid && (lane == 0 || seg_start);
  const bool piece_tail = valid && (lane == 63 || seg_end);
  const uint64_t heads = __ballot(piece_head);
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const uint64_t hm = heads & upto;
  const int start_lane = hm ? 63 - __clzll(hm) : 0;
  const uint64_t starts = __ballot(seg_start);
  const int dist = valid ? lane - start_lane : 0;
  int nsteps = 0;
  while (nsteps < 6 && __ballot(dist >= (1 << nsteps))) ++nsteps;
  const bool head_is_start = (starts >> start_lane) & 1ull;
  const bool complete = head_is_start && seg_end;
  const int slot = (start_lane == 0 && !head_is_start) ? 0 : 1;
  const double yhat = yl.x, y = yl.y;
  const double r = yhat - y;

  double gw = valid ? x * yhat - y : 0.0;  // SGD.scala:145
  gw = seg_scan(gw, lane, start_lane, nsteps);
  if (piece_tail) {
    if (complete) reinterpret_cast<float4*>(a.grads + (int64_t)u * RW)[nq] = make_float4((float)gw, 0.f, 0.f, 0.f);
    else a.part[(chunk * 2 + slot) * (int64_t)(kp + 1)] = gw;
  }
  const int flags = (valid ? 1 : 0) | (piece_tail ? 2 : 0) | (complete ? 4 : 0) | (slot << 4) | (start_lane << 8);
  const float4* __restrict__ S4 = reinterpret_cast<const float4*>(a.S);
  const int q_in = lane % G, j_in = lane / G;
  for (int qc = 0; qc < nq; qc += G) {
    const int q = qc + q_in;
    const bool qok = q < nq;
    double carry0 = 0.0, carry1 = 0.0, carry2 = 0.0, carry3 = 0.0;
    for (int rd = 0; rd < G; ++rd) {
      const int j = rd * E + j_in;
      const int fl = __shfl(flags, j);
      const uint32_t uj = __shfl(u, j);
      const int sj = __shfl(s, j);
      const float xj = __shfl(xf, j);
      const double rj = __shfl(r, j);
      const bool vj = (fl & 1) && qok;
      const int sl = fl >> 8;
      const float4 sq = vj ? S4[(int64_t)sj * nq + q] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 v = vj ? reinterpret_cast<const float4*>(a.rows + (int64_t)uj * RW)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      const double xd = xj;
      double c0 = vj ? ((double)sq.x * xd - ((double)v.x * xd) * xd) * rj : 0.0;
      double c1 = vj ? ((double)sq.y * xd - ((double)v.y * xd) * xd) * rj : 0.0;
      double c2 = vj ? ((double)sq.z * xd - ((double)v.z * xd) * xd) * rj : 0.0;
      double c3 = vj ? ((double)sq.w * xd - ((double)v.w * xd) * xd) * rj : 0.0;
      const int lo = sl > rd * E ? sl : rd * E;
#pragma unroll
      for (int o = 1; o < E; o <<= 1) {
        if (o >= (1 << nsteps)) break;
        const double t0 = __shfl_up(c0, o * G), t1 = __shfl_up(c1, o * G);
        const double t2 = __shfl_up(c2, o * G), t3 = __shfl_up(c3, o * G);
        if (j - o >= lo) {
          c0 += t0; c1 += t1; c2 += t2; c3 += t3;
        }
      }
      if (sl < rd * E) {
        c0 += carry0; c1 += carry1; c2 += carry2; c3 += carry3;
      }
      const int last = (E - 1) * G + q_in;
      carry0 = __shfl(c0, last); carry1 = __shfl(c1, last);
      carry2 = __shfl(c2, last); carry3 = __shfl(c3, last);
      if (vj && (fl & 2)) {
        if (fl & 4) {
          reinterpret_cast<float4*>(a.grads + (int64_t)uj * RW)[q] = make_float4((float)c0, (float)c1, (float)c2, (float)c3);
        } else {
          double* prow = a.part + (((chunk * 2 + ((fl >> 4) & 1)) * (int64_t)(kp + 1)) + 1 + 4 * q);
          prow[0] = c0;
          prow[1] = c1;
          prow[2] = c2;
          prow[3] = c3;
        }
      }
    }
  }
}

// Crossing runs of the emit pass: chunk-order sums of the partials -> grads[u].  Block 0 also
// closes the rank's loss statistics {loss, n_loss, U}.
__global__ __launch_bounds__(kBlock) void k_segment_emit_combine(EmitArgs a, const double2* __restrict__ loss_part,
                                                                 int64_t n_loss_blocks, const uint64_t* __restrict__ U,
                                                                 double* __restrict__ stats_out) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int kp = a.kp, RW = kp + 4;
  const int64_t W = kp + 1;
  if (blockIdx.x == 0) {
    __shared__ double rl[kBlock], rc[kBlock];
    double l = 0.0, c = 0.0;
    for (int64_t i = tid; i < n_loss_blocks; i += kBlock) {
      l += loss_part[i].x;
      c += loss_part[i].y;
    }
    rl[tid] = l;
    rc[tid] = c;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
      if (tid < o) {
        rl[tid] += rl[tid + o];
        rc[tid] += rc[tid + o];
      }
      __syncthreads();
    }
    if (tid == 0) {
      stats_out[0] = rl[0];
      stats_out[1] = rc[0];
      stats_out[2] = (double)*U;
    }
  }
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + tid;
  bool owner = false;
  uint32_t key = 0;
  if (chunk < a.nchunks) {
    const int64_t p0 = chunk * 64;
    const int64_t p1 = p0 + 64 < a.N ? p0 + 64 : a.N;
    if (p1 < a.N) {
      key = a.skeys[p1 - 1];
      owner = a.skeys[p1] == key && !(a.skeys[p0] == key && p0 > 0 && a.skeys[p0 - 1] == key);
    }
  }
  uint64_t owners = __ballot(owner);
  while (owners) {
    const int l = __ffsll((unsigned long long)owners) - 1;
    owners &= owners - 1;
    const int64_t c0 = __shfl(chunk, l);
    const uint32_t k0 = __shfl(key, l);
    int64_t cend = c0 + 1;
    for (;;) {
      const int64_t c = cend + lane;
      const bool cont = c < a.nchunks && a.skeys[c * 64] == k0;
      const uint64_t m = __ballot(cont);
      if (m == ~0ull) {
        cend += 64;
        continue;
      }
      cend += __ffsll((unsigned long long)~m) - 1;
      break;
    }
    const uint32_t u0 = a.run_of[(c0 + 1) * 64 - 1];
    for (int f0 = 0; f0 < W; f0 += 64) {
      const int f = f0 + lane;
      if (f < W) {
        double g = a.part[(c0 * 2 + 1) * W + f];
        for (int64_t c = c0 + 1; c < cend; ++c) g += a.part[(c * 2) * W + f];
        // part column 0 is gw, 1.. are gV; the wire row is [gV(kp) | gw | pad]
        a.grads[(int64_t)u0 * RW + (f == 0 ? kp : f - 1)] = (float)g;
      }
    }
  }
}

// owner side: received (slot, gradient) pairs grouped by slot (stable radix sort keeps the
// rank order), summed in fp64 in that order, then the update + L1 of SGD.scala:150-181.
template <int G>
__global__ __launch_bounds__(kBlock) void k_shard_apply(TableView T, const uint32_t* __restrict__ sslots,
                                                        const uint32_t* __restrict__ sidx, int64_t n,
                                                        const float* __restrict__ grads, StepParams p) {
  const int g = threadIdx.x % G;
  const int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G;
  if (i >= n) return;
  const uint32_t slot = sslots[i];
  if (i > 0 && sslots[i - 1] == slot) return;  // not the first of its run
  int64_t j1 = i + 1;
  while (j1 < n && sslots[j1] == slot) ++j1;
  const int kp = T.kp, nq = kp >> 2, RW = kp + 4;
  const RowHdr h = *T.hdr(slot);
  const bool present = h.t >= 0;
  const double ac = present ? p.cumE - h.cum : 0.0;
  for (int q = g; q < nq; q += G) {
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
    for (int64_t j = i; j < j1; ++j) {
      const float4 gr = reinterpret_cast<const float4*>(grads + (int64_t)sidx[j] * RW)[q];
      g0 += gr.x; g1 += gr.y; g2 += gr.z; g3 += gr.w;
    }
    float4 v = present ? reinterpret_cast<const float4*>(T.v(slot))[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (ac > 0.0) v = shrink4(v, ac);
    reinterpret_cast<float4*>(T.v(slot))[q] =
        make_float4(upd_v(v.x, g0, p), upd_v(v.y, g1, p), upd_v(v.z, g2, p), upd_v(v.w, g3, p));
  }
  if (g == 0) {
    double gw = 0.0;
    for (int64_t j = i; j < j1; ++j) gw += grads[(int64_t)sidx[j] * RW + kp];
    float w = present ? h.w : 0.f;
    if (ac > 0.0) w = shrink_f(w, ac);
    RowHdr o;
    o.w = upd_w(w, gw, p);
    o.t = p.epoch + 1;
    o.cum = p.cum_next;
    store_hdr(T, slot, o);
  }
}

inline int lanes_per_row(int nq) {
  int G = 1;
  while (G < nq && G < 16) G <<= 1;
  return G;
}

inline unsigned blocks_for(int64_t threads) {
  int64_t b = (threads + kBlock - 1) / kBlock;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

}  // namespace fmhip

using namespace fmhip;

namespace {

void require_plan(fm_ctx* ctx, const fm_batch* b) {
  FM_REQUIRE(ctx->plan_batch == b && ctx->plan_nnz == (b ? b->dev.nnz : -1),
             "fm_shard_plan must run on this batch first");
}

}  // namespace

extern "C" {

int fm_shard_plan(fm_ctx* ctx, const fm_batch* b, int64_t* send_counts) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b != nullptr && b->owner == ctx && send_counts != nullptr, "bad arguments");
    const int R = ctx->cfg.shard_count;
    FM_REQUIRE(R <= 1024, "shard_count > 1024");
    const int64_t N = b->dev.nnz;
    const uint32_t rpsh = (uint32_t)((ctx->cfg.num_features + R - 1) / R);
    ctx->plan_ck.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
    ctx->plan_run.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 1));
    ctx->plan_uidx.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 1));
    ctx->plan_req.ensure(sizeof(int32_t) * std::max<int64_t>(N, 1));
    ctx->plan_counts.ensure(sizeof(unsigned long long) * R + sizeof(uint64_t));
    const int64_t nb = (N + kTileS - 1) / kTileS;
    ctx->plan_bsum.ensure(sizeof(uint32_t) * std::max<int64_t>(nb, 1));
    hipStream_t st = ctx->stream;
    hipEvent_t e0 = ctx->prof_begin(st);
    unsigned long long* counts = ctx->plan_counts.as<unsigned long long>();
    uint64_t* total = reinterpret_cast<uint64_t*>(counts + R);
    FM_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(unsigned long long) * R + sizeof(uint64_t), st));
    if (N > 0) {
      hipLaunchKernelGGL(k_shard_keys, dim3(blocks_for(N) > 4096 ? 4096 : blocks_for(N)), dim3(kBlock), 0, st,
                         b->dev.col.as<uint32_t>(), N, (uint32_t)R, rpsh, ctx->plan_ck.as<uint32_t>());
      const uint32_t *sk = nullptr, *si = nullptr;
      radix_sort_pairs(ctx->work.sort, ctx->plan_ck.as<uint32_t>(), nullptr, N,
                       bits_for((int64_t)R * rpsh - 1), st, &sk, &si);
      ctx->plan_skeys = sk;
      ctx->plan_sidx = si;
      hipLaunchKernelGGL(k_runs_count, dim3((unsigned)nb), dim3(kBlock), 0, st, sk, N, ctx->plan_bsum.as<uint32_t>());
      hipLaunchKernelGGL(k_runs_scan, dim3(1), dim3(kBlock), 0, st, ctx->plan_bsum.as<uint32_t>(), nb, total);
      hipLaunchKernelGGL(k_plan_apply, dim3((unsigned)nb), dim3(kBlock), 0, st, sk, si, N,
                         ctx->plan_bsum.as<uint32_t>(), rpsh, R, ctx->plan_req.as<int32_t>(),
                         ctx->plan_run.as<uint32_t>(), ctx->plan_uidx.as<uint32_t>(), counts);
      FM_HIP_CHECK(hipGetLastError());
    }
    ctx->prof_end("plan", e0, st);
    ctx->pinned.ensure(sizeof(unsigned long long) * (R + 1));
    FM_HIP_CHECK(hipMemcpyAsync(ctx->pinned.p, counts, sizeof(unsigned long long) * (R + 1), hipMemcpyDeviceToHost, st));
    FM_HIP_CHECK(hipStreamSynchronize(st));
    const unsigned long long* hc = reinterpret_cast<const unsigned long long*>(ctx->pinned.p);
    int64_t U = 0;
    for (int o = 0; o < R; ++o) {
      send_counts[o] = (int64_t)hc[o];
      U += (int64_t)hc[o];
    }
    FM_REQUIRE(U == (int64_t)hc[R], "plan: inconsistent distinct-id count");
    ctx->plan_unique = U;
    ctx->plan_nnz = N;
    ctx->plan_batch = b;
    return FM_OK;
  });
}

int fm_shard_request_copy(fm_ctx* ctx, void* dst) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(ctx->plan_batch != nullptr, "no plan");
    if (ctx->plan_unique == 0) return FM_OK;
    FM_REQUIRE(dst != nullptr, "null destination");
    FM_HIP_CHECK(hipMemcpyAsync(dst, ctx->plan_req.p, sizeof(int32_t) * ctx->plan_unique, hipMemcpyDeviceToDevice,
                                ctx->stream));
    return FM_OK;
  });
}

int fm_shard_serve_device(fm_ctx* ctx, const void* req, int64_t n, void* rows_out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0, "negative n");
    if (n == 0) return FM_OK;
    FM_REQUIRE(req && rows_out, "null buffer");
    const TableView T = ctx->view();
    const int G = lanes_per_row(ctx->kp / 4);
    const unsigned blocks = blocks_for(n * G);
    const double cumE = ctx->cum_host.back();
    const int32_t* r = reinterpret_cast<const int32_t*>(req);
    float* o = reinterpret_cast<float*>(rows_out);
    hipEvent_t e0 = ctx->prof_begin(ctx->stream);
    switch (G) {
      case 1: hipLaunchKernelGGL(k_shard_serve<1>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, r, n, cumE, o); break;
      case 2: hipLaunchKernelGGL(k_shard_serve<2>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, r, n, cumE, o); break;
      case 4: hipLaunchKernelGGL(k_shard_serve<4>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, r, n, cumE, o); break;
      case 8: hipLaunchKernelGGL(k_shard_serve<8>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, r, n, cumE, o); break;
      default: hipLaunchKernelGGL(k_shard_serve<16>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, r, n, cumE, o); break;
    }
    FM_HIP_CHECK(hipGetLastError());
    ctx->prof_end("serve", e0, ctx->stream);
    return FM_OK;
  });
}

int fm_shard_local_grad_device(fm_ctx* ctx, fm_batch* b, const void* rows_in, void* grads_out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b != nullptr, "null batch");
    require_plan(ctx, b);
    const int64_t B = b->dev.n_rows, N = b->dev.nnz;
    const int64_t U = ctx->plan_unique;
    FM_REQUIRE(U == 0 || (rows_in && grads_out), "null buffer");
    reserve_work(ctx, B, N);
    ctx->ensure_hist(ctx->epoch + 1);
    double* stats = ctx->loss_hist.as<double>() + 3 * (int64_t)ctx->epoch;
    StepParams p{};
    p.w0 = ctx->cfg.w0;
    p.cumE = ctx->cum_host.back();
    int64_t nfwd = 0;
    hipEvent_t e0 = ctx->prof_begin(ctx->stream);
    if (B > 0)
      launch_forward(ctx->view(), b->dev, ctx->work, p, ctx->stream, &nfwd, reinterpret_cast<const float*>(rows_in),
                     ctx->plan_uidx.as<uint32_t>());
    ctx->prof_end("forward", e0, ctx->stream);
    e0 = ctx->prof_begin(ctx->stream);
    EmitArgs a;
    a.skeys = ctx->plan_skeys;
    a.sidx = ctx->plan_sidx;
    a.run_of = ctx->plan_run.as<uint32_t>();
    a.ent = b->dev.ent.as<uint2>();
    a.rows = reinterpret_cast<const float*>(rows_in);
    a.S = ctx->work.S.as<float>();
    a.yl = ctx->work.yl.as<float2>();
    a.grads = reinterpret_cast<float*>(grads_out);
    a.part = ctx->work.part.as<double>();
    a.N = N;
    a.nchunks = (N + 63) / 64;
    a.kp = ctx->kp;
    const int G = lanes_per_row(ctx->kp / 4);
    if (a.nchunks > 0) {
      const unsigned blocks = (unsigned)((a.nchunks + 3) / 4);
      switch (G) {
        case 1: hipLaunchKernelGGL(k_segment_emit<1>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a); break;
        case 2: hipLaunchKernelGGL(k_segment_emit<2>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a); break;
        case 4: hipLaunchKernelGGL(k_segment_emit<4>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a); break;
        case 8: hipLaunchKernelGGL(k_segment_emit<8>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a); break;
        default: hipLaunchKernelGGL(k_segment_emit<16>, dim3(blocks), dim3(kBlock), 0, ctx->stream, a); break;
      }
    }
    const uint64_t* Ud = reinterpret_cast<const uint64_t*>(ctx->plan_counts.as<unsigned long long>() + ctx->cfg.shard_count);
    hipLaunchKernelGGL(k_segment_emit_combine, dim3(blocks_for(std::max<int64_t>(a.nchunks, 1))), dim3(kBlock), 0,
                       ctx->stream, a, ctx->work.loss_part.as<double2>(), B > 0 ? nfwd : (int64_t)0, Ud, stats);
    FM_HIP_CHECK(hipGetLastError());
    ctx->prof_end("grad", e0, ctx->stream);
    return FM_OK;
  });
}

int fm_shard_apply_device(fm_ctx* ctx, const void* req, const void* grads, int64_t n, int32_t t, double step_size,
                          double reg_param, int64_t global_rows) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0 && global_rows >= 0, "negative size");
    if (global_rows == 0) return FM_NOTHING_TO_DO;  // SGD.scala:126-128 (every rank skips)
    FM_REQUIRE(t >= 1, "iteration index t must be >= 1");
    StepParams p{};
    p.n_rows = global_rows;
    p.eta = step_size / std::sqrt((double)t);  // SGD.scala:121
    p.lam = p.eta * reg_param;                 // SGD.scala:122
    p.m = (double)global_rows;                 // global miniBatchSize
    p.scale_v = p.eta / (double)global_rows;
    p.epoch = ctx->epoch;
    p.cumE = ctx->cum_host.back();
    p.cum_next = p.cumE + p.lam;
    p.w0 = ctx->cfg.w0;
    hipEvent_t e0 = ctx->prof_begin(ctx->stream);
    if (n > 0) {
      FM_REQUIRE(req && grads, "null buffer");
      const uint32_t *ss = nullptr, *si = nullptr;
      radix_sort_pairs(ctx->work.sort, reinterpret_cast<const uint32_t*>(req), nullptr, n,
                       bits_for(std::max<int64_t>(ctx->rows - 1, 1)), ctx->stream, &ss, &si);
      const int G = lanes_per_row(ctx->kp / 4);
      const unsigned blocks = blocks_for(n * G);
      const TableView T = ctx->view();
      const float* gr = reinterpret_cast<const float*>(grads);
      switch (G) {
        case 1: hipLaunchKernelGGL(k_shard_apply<1>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, ss, si, n, gr, p); break;
        case 2: hipLaunchKernelGGL(k_shard_apply<2>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, ss, si, n, gr, p); break;
        case 4: hipLaunchKernelGGL(k_shard_apply<4>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, ss, si, n, gr, p); break;
        case 8: hipLaunchKernelGGL(k_shard_apply<8>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, ss, si, n, gr, p); break;
        default: hipLaunchKernelGGL(k_shard_apply<16>, dim3(blocks), dim3(kBlock), 0, ctx->stream, T, ss, si, n, gr, p); break;
      }
      FM_HIP_CHECK(hipGetLastError());
    }
    ctx->prof_end("apply", e0, ctx->stream);
    ctx->epoch += 1;
    ctx->cum_host.push_back(p.cum_next);
    ctx->plan_batch = nullptr;
    return FM_OK;
  });
}

int fm_shard_last_loss(fm_ctx* ctx, double* loss_sum, int64_t* n_loss_rows) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(loss_sum && n_loss_rows, "null argument");
    FM_REQUIRE(ctx->epoch >= 1, "no step executed");
    double h[3];
    FM_HIP_CHECK(hipMemcpyAsync(h, ctx->loss_hist.as<double>() + 3 * (int64_t)(ctx->epoch - 1), sizeof(h),
                                hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    *loss_sum = h[0];
    *n_loss_rows = (int64_t)h[1];
    return FM_OK;
  });
}

}  // extern "C"
