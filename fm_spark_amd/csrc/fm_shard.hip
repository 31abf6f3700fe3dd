// Row-sharded FM SGD step, owner-computes (one context per rank; the owner of feature id is
// id % R, its local slot id / R).  Every rank holds 1/R of the table and steps its own
// mini-batch.  One iteration is five phases of the C-ABI joined by three all-to-alls; the
// first two depend on the batch alone and run one iteration ahead on the side stream:
//
//   fm_shard_route          requester: per sample the owners it touches and the pair index of
//                           every (sample, owner) pair; the entries partitioned by owner (CSR
//                           order kept) as {slot} and {pair index within the owner's block, x}
//                           by one stable radix pass over owner bits above the slot   [side]
//   -- all-to-all entries -->
//   fm_shard_owner_prepare  owner: the received entries' pair table (pair = source offset + the
//                           carried local index; one pass) and their stable order by slot
//                           (source rank, then CSR order)                               [side]
//   fm_shard_owner_forward  owner: per received pair, the partial forward sums over the entries
//                           it owns: [sum v*x | sum v^2 x^2 | sum w*x], lazy L1 caught up on read
//                           (FactorizationMachinesModel.scala:173-221)                [main]
//   -- all-to-all partials <--
//   fm_shard_combine        requester: per sample, the owners' partials summed in owner order
//                           (fp64) -> vfxiSum S, yhat, loss; S | yhat | y sent back per pair
//   -- all-to-all S -->
//   fm_shard_owner_update   owner: the fused segmented gradient + update + L1 of fm_kernels.hip
//                           (SGD.scala:143-181) over the slot-sorted entries, on its own rows
//
// Semantics equal the single-table step over the ranks' batches concatenated in rank order
// (global miniBatchSize m = sum of the ranks' rows), up to fp summation order: the forward
// sums are split per owner (fp32 on the wire), the per-feature gradient sums run over the
// same entries in the same order.  Deterministic for a given R.
// Traffic per rank and step (k = 16, z = 39, R = 8): entries 12 B each (off the critical path:
// exchanged during the previous iteration), partials and S (kp + 2) * 4 B per (sample, owner)
// pair -- about 2 x 150 MB, against about 1 GB when rows and gradients of every distinct id
// travel instead.
// Wire buffers are structures of arrays over the pairs, so every k-vector is 16-B aligned and a
// 64-B row at k = 16: partials [P][kp] fp32 sum v*x then [P] fp32 {sum v^2 x^2, sum w x}; S [P][kp]
// fp32 vfxiSum then [P] fp32 {r, yhat} (r = yhat - y formed in fp64 by the requester, then rounded).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "fm_context.h"
#include "fm_device.h"

namespace fmhip {

namespace {

constexpr int kBlock = 256;
constexpr int kMaxR = 64;     // owner masks are uint64

__device__ __forceinline__ uint32_t incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// ------------------------------------------------------------------ requester: route
constexpr int kTeamR = 16;  // lanes per sample in the route kernels (coalesced entry reads)

__device__ __forceinline__ uint64_t team_or64(uint64_t m) {
  uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
#pragma unroll
  for (int o = 1; o < kTeamR; o <<= 1) {
    lo |= __shfl_xor(lo, o);
    hi |= __shfl_xor(hi, o);
  }
  return ((uint64_t)hi << 32) | lo;
}

// per sample (a team of lanes over its entries): the owners it touches (bit mask); per owner:
// entry counts.  Ids >= F (a predict batch's ids outside the model, dropped by the inner joins of
// Model.scala:103-112) belong to no owner.
__global__ __launch_bounds__(kBlock) void k_sample_mask(const int64_t* __restrict__ row_ptr,
                                                        const uint32_t* __restrict__ col, int64_t B, uint32_t R,
                                                        uint64_t F, uint64_t* __restrict__ mask,
                                                        unsigned long long* __restrict__ ecount) {
  constexpr int TPB = kBlock / kTeamR;
  __shared__ uint32_t cnt[kMaxR];
  if (threadIdx.x < kMaxR) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int tl = threadIdx.x % kTeamR;
  for (int64_t s0 = (int64_t)blockIdx.x * TPB; s0 < B; s0 += (int64_t)gridDim.x * TPB) {  // block-uniform
    const int64_t s = s0 + threadIdx.x / kTeamR;
    uint64_t m = 0;
    if (s < B) {
      for (int64_t e = row_ptr[s] + tl; e < row_ptr[s + 1]; e += kTeamR) {
        if (col[e] >= F) continue;
        const uint32_t o = col[e] % R;
        m |= 1ull << o;
        atomicAdd(&cnt[o], 1u);
      }
    }
    m = team_or64(m);
    if (s < B && tl == 0) mask[s] = m;
  }
  __syncthreads();
  if (threadIdx.x < R && cnt[threadIdx.x]) atomicAdd(&ecount[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// per entry, in CSR order: key = owner << sb | slot and the wire payload {pair index of (sample,
// owner) within the owner's block, x bits}, so one stable pass over the owner bits lays out the
// send buffers.  Ids >= F get owner R: they sort after every owner's block and are not sent.  One
// lane per entry: the exploded entry {sample, x} names its sample, so the pass streams the id and
// entry arrays without the CSR row walk (neighbouring lanes share a sample's pair indices).
__global__ __launch_bounds__(kBlock) void k_route_keys(const uint32_t* __restrict__ col, const uint2* __restrict__ ent,
                                                       int64_t N, uint32_t R, int sb, uint64_t F,
                                                       const int32_t* __restrict__ pairidx, uint32_t* __restrict__ key,
                                                       uint2* __restrict__ pay) {
  // kRkU entries per thread at once: their ids and entries, then their pair indices, each a single
  // round trip (clamped indices)
  constexpr int kRkU = 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t e0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; e0 < N; e0 += kRkU * stride) {
    uint32_t id[kRkU];
    uint2 en[kRkU];
#pragma unroll
    for (int u = 0; u < kRkU; ++u) {
      const int64_t e = e0 + u * stride;
      const int64_t ec = e < N ? e : N - 1;
      id[u] = col[ec];
      en[u] = ent[ec];
    }
    int32_t px[kRkU];
#pragma unroll
    for (int u = 0; u < kRkU; ++u) {
      const uint32_t o = id[u] < F ? id[u] % R : 0u;
      px[u] = pairidx[(int64_t)en[u].x * R + o];
    }
#pragma unroll
    for (int u = 0; u < kRkU; ++u) {
      const int64_t e = e0 + u * stride;
      if (e >= N) break;
      if (id[u] >= F) {
        key[e] = R << sb;
        pay[e] = make_uint2(0u, en[u].y);
        continue;
      }
      const uint32_t o = id[u] % R;
      key[e] = (o << sb) | (id[u] / R);
      pay[e] = make_uint2((uint32_t)px[u], en[u].y);
    }
  }
}

// The owner's received S rows, wire layout [P][kp] vectors then [P] {r, yhat} -> the single-table
// step's per-sample records [P][rec] = [S (kp) | {r, yhat} | 0 pad] (kp <= 16: 64- or 128-B
// records), so the segmented update gathers one line per entry instead of two (the S row and its
// scalars).  Streaming, float4 per lane.
__global__ __launch_bounds__(kBlock) void k_pack_srec(const float* __restrict__ vec, const float2* __restrict__ sc,
                                                      int64_t P, int kp, int rec, float* __restrict__ out) {
  const int q = rec / 4;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P * q; i += (int64_t)gridDim.x * kBlock) {
    const int64_t pr = i / q;
    const int j = (int)(i - pr * q) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < kp) {
      v = *reinterpret_cast<const float4*>(vec + pr * kp + j);
    } else if (j == kp) {
      const float2 s2 = sc[pr];
      v.x = s2.x;
      v.y = s2.y;
    }
    *reinterpret_cast<float4*>(out + pr * rec + j) = v;
  }
}

__global__ void k_key_slots(const uint32_t* __restrict__ key, int64_t n, uint32_t slot_mask,
                            uint32_t* __restrict__ slot) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    slot[i] = key[i] & slot_mask;
}

// pairs per (owner, tile of kBlock samples) -> tcnt[o][tile]
__global__ __launch_bounds__(kBlock) void k_pair_count(const uint64_t* __restrict__ mask, int64_t B, int R,
                                                       int64_t ntiles, uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t wc[kBlock / 64][kMaxR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t m = s < B ? mask[s] : 0ull;
  for (int o = 0; o < R; ++o) {
    const uint64_t b = __ballot((m >> o) & 1ull);
    if (lane == 0) wc[wave][o] = (uint32_t)__popcll(b);
  }
  __syncthreads();
  if (threadIdx.x < R) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += wc[w][threadIdx.x];
    tcnt[(int64_t)threadIdx.x * ntiles + blockIdx.x] = t;
  }
}

// one block per row: exclusive scan of rows[r][0..n) in place, row total -> tot[r]
__global__ __launch_bounds__(kBlock) void k_rows_scan(uint32_t* __restrict__ rows, int64_t n,
                                                      unsigned long long* __restrict__ tot) {
  __shared__ uint32_t ws[kBlock / 64];
  uint32_t* row = rows + (int64_t)blockIdx.x * n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t b = 0; b < n; b += kBlock) {
    const int64_t i = b + threadIdx.x;
    const uint32_t v = i < n ? row[i] : 0u;
    const uint32_t inc = incl_scan_u32(v, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      pre += w < wave ? ws[w] : 0u;
      t += ws[w];
    }
    if (i < n) row[i] = carry + pre + inc - v;
    carry += t;
    __syncthreads();
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// pair index of every (sample, owner): owner o's pairs are numbered in sample order
__global__ __launch_bounds__(kBlock) void k_pair_index(const uint64_t* __restrict__ mask, int64_t B, int R,
                                                       int64_t ntiles, const uint32_t* __restrict__ toff,
                                                       int32_t* __restrict__ pairidx) {
  __shared__ uint32_t wc[kBlock / 64][kMaxR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t m = s < B ? mask[s] : 0ull;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int o = 0; o < R; ++o) {
    const uint64_t b = __ballot((m >> o) & 1ull);
    if (lane == 0) wc[wave][o] = (uint32_t)__popcll(b);
  }
  __syncthreads();
  for (int o = 0; o < R; ++o) {
    const bool bit = (m >> o) & 1ull;
    const uint64_t b = __ballot(bit);
    uint32_t pre = toff[(int64_t)o * ntiles + blockIdx.x] + (uint32_t)__popcll(b & lt);
    for (int w = 0; w < wave; ++w) pre += wc[w][o];
    if (s < B) pairidx[s * R + o] = bit ? (int32_t)pre : -1;
  }
}

// ------------------------------------------------------------------ owner: pairs
// The received entries are source-major, each source's in its CSR order, carrying their pair's
// index within that source's block: ent2 = {pair = pbase[source] + local, x}, and the first
// entry of every pair opens it in pair_ptr (one pass, no scan).
// ent2 == nullptr (one source: its pairs start at 0, so ent2 would equal ent): the pair table only.
__global__ __launch_bounds__(kBlock) void k_pair_table(const uint2* __restrict__ ent, int64_t n,
                                                       const int64_t* __restrict__ src_off,
                                                       const int64_t* __restrict__ pbase, int R,
                                                       int64_t* __restrict__ pair_ptr, uint2* __restrict__ ent2) {
  // the source offsets and pair bases in LDS (a loop of dependent global loads per entry otherwise);
  // an entry and its predecessor loaded together (clamped index), kPtU entries per thread at once
  constexpr int kPtU = 4;
  __shared__ int64_t so[kMaxR + 1], pb[kMaxR];
  for (int t = threadIdx.x; t <= R; t += kBlock) so[t] = src_off[t];
  for (int t = threadIdx.x; t < R; t += kBlock) pb[t] = pbase[t];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += kPtU * stride) {
    uint2 e[kPtU];
    uint32_t px[kPtU];
#pragma unroll
    for (int u = 0; u < kPtU; ++u) {
      const int64_t i = i0 + u * stride;
      const int64_t ic = i < n ? i : n - 1;
      e[u] = ent[ic];
      px[u] = ent[ic > 0 ? ic - 1 : 0].x;
    }
#pragma unroll
    for (int u = 0; u < kPtU; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) break;
      int r = 0;
      while (r + 1 < R && so[r + 1] <= i) ++r;
      const uint32_t pair = (uint32_t)pb[r] + e[u].x;
      if (ent2) ent2[i] = make_uint2(pair, e[u].y);
      if (i == so[r] || px[u] != e[u].x) pair_ptr[pair] = i;
    }
  }
}

// ------------------------------------------------------------------ requester: combine
// Team of GS lanes per sample (one quad each): the owners' partials summed in owner order
// in fp64 -> S = vfxiSum, yhat = 0.5 (|S|^2 - sum v^2 x^2) + sum w x + w0
// (FactorizationMachinesModel.scala:221, :260-262), the loss partial (:230), and the S rows
// sent back to every owner holding entries of the sample.  Wire layout (structure of arrays):
// part_vec / s_vec [pair][kp], part_sc / s_sc [pair] float2 ({sum v^2 x^2, sum w x} / {yhat, y}).
// OW > 0 (R <= OW owners): the sample's pair slots live in registers and every owner's loads of a
// pass are issued before any is used (clamped owner indices; a pair the sample lacks reads poff's
// first bytes and is masked out) -- as guarded loads, one per owner, each waited out its round trip
// before the next: 2R + R round trips per sample.  OW = 0: any R up to kMaxR, owner by owner.
template <int GS, int OW>
__global__ __launch_bounds__(kBlock) void k_shard_combine(const int32_t* __restrict__ pairidx,
                                                          const int64_t* __restrict__ poff, int R, int64_t B,
                                                          const float* __restrict__ part_vec,
                                                          const float2* __restrict__ part_sc,
                                                          const double* __restrict__ label, int kp, double w0,
                                                          float* __restrict__ s_vec, float2* __restrict__ s_sc,
                                                          double2* __restrict__ loss_part) {
  constexpr int TPB = kBlock / GS;
  const int tid = threadIdx.x, g = tid % GS;
  const int nq = kp >> 2;
  double loss_acc = 0.0, nloss = 0.0;
  for (int64_t s = (int64_t)blockIdx.x * TPB + tid / GS; s < B; s += (int64_t)gridDim.x * TPB) {
    const int32_t* pi = pairidx + s * R;
    double vv = 0.0, wx = 0.0, ss = 0.0;
    bool any = false;
    if constexpr (OW > 0) {
      int32_t ix[OW];
      int64_t pj[OW];  // the sample's pair slot in owner o's block, -1: none
#pragma unroll
      for (int o = 0; o < OW; ++o) {
        const int oc = o < R ? o : R - 1;
        ix[o] = pi[oc];
        pj[o] = poff[oc];
      }
      float2 t[OW];
#pragma unroll
      for (int o = 0; o < OW; ++o) {
        pj[o] = o < R && ix[o] >= 0 ? pj[o] + ix[o] : -1;
        t[o] = *(pj[o] >= 0 ? part_sc + pj[o] : reinterpret_cast<const float2*>(poff));
      }
#pragma unroll
      for (int o = 0; o < OW; ++o) {  // owner order, as the loop below
        vv += pj[o] >= 0 ? (double)t[o].x : 0.0;
        wx += pj[o] >= 0 ? (double)t[o].y : 0.0;
        any = any || pj[o] >= 0;
      }
      for (int qc = 0; qc < nq; qc += GS) {
        const int q = qc + g;
        if (q >= nq) break;  // (q grows with qc)
        float4 tv[OW];
#pragma unroll
        for (int o = 0; o < OW; ++o)
          tv[o] = pj[o] >= 0 ? reinterpret_cast<const float4*>(part_vec + pj[o] * kp)[q]
                             : *reinterpret_cast<const float4*>(poff);
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
        for (int o = 0; o < OW; ++o) {
          const bool ok = pj[o] >= 0;
          a0 += ok ? (double)tv[o].x : 0.0; a1 += ok ? (double)tv[o].y : 0.0;
          a2 += ok ? (double)tv[o].z : 0.0; a3 += ok ? (double)tv[o].w : 0.0;
        }
        ss += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
        const float4 sq = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
#pragma unroll
        for (int o = 0; o < OW; ++o)
          if (pj[o] >= 0) reinterpret_cast<float4*>(s_vec + pj[o] * kp)[q] = sq;
      }
#pragma unroll
      for (int o = 1; o < GS; o <<= 1) ss += __shfl_xor(ss, o);
      const double yhat = 0.5 * (ss - vv) + wx + w0;
      if (g == 0) {
        const double y = label[s];
#pragma unroll
        for (int o = 0; o < OW; ++o)
          if (pj[o] >= 0) s_sc[pj[o]] = make_float2((float)(yhat - y), (float)yhat);  // {r, yhat}
        if (any) {
          const double d = yhat - y;
          loss_acc += d * d;
          nloss += 1.0;
        }
      }
      continue;
    }
    for (int o = 0; o < R; ++o) {
      const int32_t ix = pi[o];
      if (ix >= 0) {
        const float2 t = part_sc[poff[o] + ix];
        vv += (double)t.x;
        wx += (double)t.y;
        any = true;
      }
    }
    for (int qc = 0; qc < nq; qc += GS) {
      const int q = qc + g;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      if (q < nq) {
        for (int o = 0; o < R; ++o) {
          const int32_t ix = pi[o];
          if (ix >= 0) {
            const float4 t = reinterpret_cast<const float4*>(part_vec + (poff[o] + ix) * kp)[q];
            a0 += (double)t.x; a1 += (double)t.y; a2 += (double)t.z; a3 += (double)t.w;
          }
        }
        ss += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
        const float4 sq = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
        for (int o = 0; o < R; ++o) {
          const int32_t ix = pi[o];
          if (ix >= 0) reinterpret_cast<float4*>(s_vec + (poff[o] + ix) * kp)[q] = sq;
        }
      }
    }
#pragma unroll
    for (int o = 1; o < GS; o <<= 1) ss += __shfl_xor(ss, o);
    const double yhat = 0.5 * (ss - vv) + wx + w0;
    if (g == 0) {
      const double y = label[s];
      for (int o = 0; o < R; ++o) {
        const int32_t ix = pi[o];
        if (ix >= 0) s_sc[poff[o] + ix] = make_float2((float)(yhat - y), (float)yhat);  // {r, yhat}
      }
      if (any) {
        const double d = yhat - y;
        loss_acc += d * d;
        nloss += 1.0;
      }
    }
  }
  __shared__ double red[2][kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    loss_acc += __shfl_xor(loss_acc, o);
    nloss += __shfl_xor(nloss, o);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = loss_acc;
    red[1][tid >> 6] = nloss;
  }
  __syncthreads();
  if (tid == 0) {
    double l = 0.0, c = 0.0;
    for (int w = 0; w < kBlock / 64; ++w) {
      l += red[0][w];
      c += red[1][w];
    }
    loss_part[blockIdx.x] = make_double2(l, c);
  }
}

// The same sums for FactorizationMachinesModel.predict (Model.scala:90-133) over a sharded table:
// pcnt[pair] = the owner's present rows among the pair's entries (absent ids drop out, :103-112);
// a sample with none scores globalBias unclamped (na.fill, :78-86), every other
// least(greatest(yhat, minLabel), maxLabel) (:129-132).
template <int GS>
__global__ __launch_bounds__(kBlock) void k_shard_predict(const int32_t* __restrict__ pairidx,
                                                          const int64_t* __restrict__ poff, int R, int64_t B,
                                                          const float* __restrict__ part_vec,
                                                          const float2* __restrict__ part_sc,
                                                          const uint32_t* __restrict__ pcnt, int kp, double w0,
                                                          double lo, double hi, double* __restrict__ pred) {
  constexpr int TPB = kBlock / GS;
  const int tid = threadIdx.x, g = tid % GS;
  const int nq = kp >> 2;
  for (int64_t s = (int64_t)blockIdx.x * TPB + tid / GS; s < B; s += (int64_t)gridDim.x * TPB) {
    const int32_t* pi = pairidx + s * R;
    double vv = 0.0, wx = 0.0, ss = 0.0;
    uint32_t cnt = 0;
    for (int o = 0; o < R; ++o) {
      const int32_t ix = pi[o];
      if (ix >= 0) {
        const float2 t = part_sc[poff[o] + ix];
        vv += (double)t.x;
        wx += (double)t.y;
        cnt += pcnt[poff[o] + ix];
      }
    }
    for (int qc = 0; qc < nq; qc += GS) {
      const int q = qc + g;
      if (q >= nq) continue;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      for (int o = 0; o < R; ++o) {
        const int32_t ix = pi[o];
        if (ix >= 0) {
          const float4 t = reinterpret_cast<const float4*>(part_vec + (poff[o] + ix) * kp)[q];
          a0 += (double)t.x; a1 += (double)t.y; a2 += (double)t.z; a3 += (double)t.w;
        }
      }
      ss += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
    }
#pragma unroll
    for (int o = 1; o < GS; o <<= 1) ss += __shfl_xor(ss, o);
    const double yhat = 0.5 * (ss - vv) + wx + w0;
    if (g == 0) pred[s] = cnt == 0 ? w0 : fmin(fmax(yhat, lo), hi);
  }
}

inline unsigned blocks_for(int64_t threads, int64_t cap = 256 * 16) {
  int64_t b = (threads + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

inline int team_for(int nq) {
  int G = 1;
  while (G < nq && G < 16) G <<= 1;
  return G;
}

// owner blocks of the partial / S rows: poff[o] = pairs sent to owners before o
__global__ void k_owner_offsets(const unsigned long long* __restrict__ pairs, int R, int64_t* __restrict__ poff) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int64_t acc = 0;
    for (int o = 0; o < R; ++o) {
      poff[o] = acc;
      acc += (int64_t)pairs[o];
    }
    poff[R] = acc;
  }
}

}  // namespace

// The owner partial pass of fm_shard_owner_forward; present_out (optional, [P] uint32): the pair's
// present rows (sharded predict).
void shard_owner_partials(fm_ctx* ctx, fm_batch* b, void* partials_out, uint32_t* present_out, int chunk,
                          int chunks);

}  // namespace fmhip

using namespace fmhip;

namespace {

// Owner-side step parameters (SGD.scala:121-124 with the global miniBatchSize).
StepParams shard_params(fm_ctx* ctx, int32_t t, double step_size, double reg_param, int64_t global_rows) {
  StepParams p{};
  p.n_rows = global_rows;
  p.eta = step_size / std::sqrt((double)t);  // SGD.scala:121
  p.lam = p.eta * reg_param;                 // SGD.scala:122
  p.m = (double)global_rows;
  p.scale_v = p.eta / (double)global_rows;
  p.epoch = ctx->epoch;
  p.cumE = ctx->cum_host.back();
  p.cum_next = p.cumE + p.lam;
  p.w0 = ctx->cfg.w0;
  return p;
}

// The batch's sharded state, created on first use with its events already "done".
ShardBatchState& shard_state(fm_ctx* ctx, fm_batch* b) {
  FM_REQUIRE(b != nullptr && b->owner == ctx, "batch belongs to another context");
  FM_REQUIRE(!ctx->group, "a multi-GPU context runs its sharded phases itself (fm_step / fm_step_batch)");
  FM_REQUIRE(ctx->cfg.shard_count >= 1, "bad context");
  if (!b->sh) {
    std::unique_ptr<ShardBatchState> s(new ShardBatchState());
    FM_HIP_CHECK(hipEventCreateWithFlags(&s->ready_fwd, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventCreateWithFlags(&s->ready_upd, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventCreateWithFlags(&s->last_use, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventRecord(s->ready_fwd, ctx->side));
    FM_HIP_CHECK(hipEventRecord(s->ready_upd, ctx->side));
    FM_HIP_CHECK(hipEventRecord(s->last_use, ctx->stream));
    b->sh = std::move(s);
  }
  return *b->sh;
}

}  // namespace

extern "C" {

int fm_shard_route(fm_ctx* ctx, fm_batch* b, void* send_slot, void* send_ent, int64_t* counts) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(counts != nullptr, "bad arguments");
    shard_route_launch(ctx, b, send_slot, send_ent, ctx->side);
    const int R = ctx->cfg.shard_count;
    ctx->side_pinned.ensure(sizeof(unsigned long long) * 2 * R);
    FM_HIP_CHECK(hipMemcpyAsync(ctx->side_pinned.p, ctx->sh_tot.p, sizeof(unsigned long long) * 2 * R,
                                hipMemcpyDeviceToHost, ctx->side));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->side));  // the side stream only: the main stream keeps running
    shard_route_finish(ctx, b, reinterpret_cast<const unsigned long long*>(ctx->side_pinned.p), counts);
    return FM_OK;
  });
}

}  // extern "C"

namespace fmhip {

// Phase 1 enqueued on the side stream, its counts left on the device in ctx->sh_tot ([R] pairs,
// then [R] entries per owner, uint64): a multi-GPU context gathers every rank's counts on the
// device and reads them back once for the whole job (fm_group.hip prefetch).
void shard_route_launch(fm_ctx* ctx, fm_batch* b, void* send_slot, void* send_ent, hipStream_t st) {
  {
    ShardBatchState& S = shard_state(ctx, b);
    const int R = ctx->cfg.shard_count;
    FM_REQUIRE(R <= kMaxR, "the owner-computes sharded step supports at most 64 ranks");
    const int64_t B = b->dev.n_rows, N = b->dev.nnz;
    FM_REQUIRE(N == 0 || (send_slot && send_ent), "null send buffer");
    if (!st) st = ctx->side;
    // the batch's previous iteration may still read its requester state on the main stream; a batch
    // refilled by fm_batch_from_rows is routed once its gather is done
    FM_HIP_CHECK(hipStreamWaitEvent(st, S.last_use, 0));
    wait_built(b, st);
    hipEvent_t e0 = ctx->prof_begin(st);
    const int64_t ntiles = std::max<int64_t>((B + kBlock - 1) / kBlock, 1);
    ctx->sh_okey.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
    ctx->sh_mask.ensure(sizeof(uint64_t) * std::max<int64_t>(B, 1));
    ctx->sh_tcnt.ensure(sizeof(uint32_t) * R * ntiles);
    ctx->sh_tot.ensure(sizeof(unsigned long long) * 2 * R);
    S.pairidx.ensure(sizeof(int32_t) * std::max<int64_t>(B, 1) * R);
    S.poff.ensure(sizeof(int64_t) * (R + 1));
    unsigned long long* tot = ctx->sh_tot.as<unsigned long long>();  // [R] pairs, [R] entries
    FM_HIP_CHECK(hipMemsetAsync(tot, 0, sizeof(unsigned long long) * 2 * R, st));
    const uint64_t F = (uint64_t)ctx->cfg.num_features;
    const bool drop = b->max_id >= (int64_t)F;  // a predict batch with ids outside the model
    if (B > 0) {
      hipLaunchKernelGGL(k_sample_mask, dim3(blocks_for(B * kTeamR)), dim3(kBlock), 0, st, b->dev.row_ptr.as<int64_t>(),
                         b->dev.col.as<uint32_t>(), B, (uint32_t)R, F, ctx->sh_mask.as<uint64_t>(), tot + R);
      hipLaunchKernelGGL(k_pair_count, dim3((unsigned)ntiles), dim3(kBlock), 0, st, ctx->sh_mask.as<uint64_t>(), B,
                         R, ntiles, ctx->sh_tcnt.as<uint32_t>());
      hipLaunchKernelGGL(k_rows_scan, dim3((unsigned)R), dim3(kBlock), 0, st, ctx->sh_tcnt.as<uint32_t>(), ntiles,
                         tot);
      hipLaunchKernelGGL(k_pair_index, dim3((unsigned)ntiles), dim3(kBlock), 0, st, ctx->sh_mask.as<uint64_t>(), B,
                         R, ntiles, ctx->sh_tcnt.as<uint32_t>(), S.pairidx.as<int32_t>());
    }
    hipLaunchKernelGGL(k_owner_offsets, dim3(1), dim3(64), 0, st, tot, R, S.poff.as<int64_t>());
    if (N > 0) {
      // wire keys owner << sb | slot with payload {pair index within the owner's block, x}; one
      // stable pass over the owner bits partitions them (CSR order kept inside each owner).  sb
      // must hold the largest slot of ANY owner (owner 0 has the most rows), the same on every rank
      const int sb = bits_for(std::max<int64_t>((ctx->cfg.num_features - 1) / R, 1));
      const int ob = bits_for(drop ? R : R - 1);
      FM_REQUIRE(sb + ob <= 32, "route key does not fit 32 bits");
      if (R == 1 && !drop) {
        // one owner: CSR order is already the owner order and the key is the slot -- the keys and
        // payloads go straight to the send buffers, no partition pass
        hipLaunchKernelGGL(k_route_keys, dim3(blocks_for(N)), dim3(kBlock), 0, st, b->dev.col.as<uint32_t>(),
                           b->dev.ent.as<uint2>(), N, (uint32_t)R, sb, F, S.pairidx.as<int32_t>(),
                           reinterpret_cast<uint32_t*>(send_slot), reinterpret_cast<uint2*>(send_ent));
      } else {
        ctx->sh_pay.ensure(sizeof(uint2) * std::max<int64_t>(N, 4) + 16);
        ctx->sh_skey.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
        hipLaunchKernelGGL(k_route_keys, dim3(blocks_for(N)), dim3(kBlock), 0, st, b->dev.col.as<uint32_t>(),
                           b->dev.ent.as<uint2>(), N, (uint32_t)R, sb, F, S.pairidx.as<int32_t>(),
                           ctx->sh_okey.as<uint32_t>(), ctx->sh_pay.as<uint2>());
        radix_sort_pairs64_bits(ctx->route_sort, ctx->sh_okey.as<uint32_t>(), ctx->sh_pay.as<uint2>(), N, sb, sb + ob, st,
                                ctx->sh_skey.as<uint32_t>(), reinterpret_cast<uint2*>(send_ent));
        hipLaunchKernelGGL(k_key_slots, dim3(blocks_for(N)), dim3(kBlock), 0, st, ctx->sh_skey.as<uint32_t>(), N,
                           (uint32_t)((sb >= 32) ? 0xFFFFFFFFu : ((1u << sb) - 1u)), reinterpret_cast<uint32_t*>(send_slot));
      }
    }
    FM_HIP_CHECK(hipGetLastError());
    ctx->prof_end("route", e0, st);
    S.route_nnz = -1;  // until shard_route_finish has the counts
  }
}

// The host's copy of the route counts hc ([R] pairs, [R] entries) -> counts[0..R) entries and
// counts[R..2R) pairs per owner, and the batch's requester state.
void shard_route_finish(fm_ctx* ctx, fm_batch* b, const unsigned long long* hc, int64_t* counts) {
  {
    ShardBatchState& S = shard_state(ctx, b);
    const int R = ctx->cfg.shard_count;
    const int64_t N = b->dev.nnz;
    const bool drop = b->max_id >= (int64_t)ctx->cfg.num_features;
    S.pairs_out.assign(R, 0);
    int64_t ne = 0;
    for (int o = 0; o < R; ++o) {
      counts[o] = (int64_t)hc[R + o];      // entries to owner o
      counts[R + o] = (int64_t)hc[o];      // (sample, owner) pairs to owner o
      S.pairs_out[o] = (int64_t)hc[o];
      ne += (int64_t)hc[R + o];
    }
    FM_REQUIRE(drop ? ne <= N : ne == N, "route: inconsistent entry count");
    S.route_nnz = N;
    S.combined = false;
  }
}

}  // namespace fmhip

extern "C" {

int fm_shard_owner_prepare(fm_ctx* ctx, fm_batch* b, const void* recv_slot, const void* recv_ent, int64_t n,
                           const int64_t* src_entries, const int64_t* src_pairs) {
  return guarded(ctx, [&]() -> int {
    ShardBatchState& S = shard_state(ctx, b);
    const int R = ctx->cfg.shard_count;
    FM_REQUIRE(n >= 0 && src_entries && src_pairs, "bad arguments");
    std::vector<int64_t> off(2 * (R + 1), 0);  // [R+1] source entry offsets, [R+1] source pair offsets
    int64_t P = 0;
    for (int r = 0; r < R; ++r) {
      FM_REQUIRE(src_entries[r] >= 0 && src_pairs[r] >= 0 && src_pairs[r] <= src_entries[r], "bad source counts");
      FM_REQUIRE(src_entries[r] == 0 || src_pairs[r] >= 1, "bad source counts");
      off[r + 1] = off[r] + src_entries[r];
      off[R + 1 + r + 1] = off[R + 1 + r] + src_pairs[r];
      P += src_pairs[r];
    }
    FM_REQUIRE(off[R] == n, "source entry counts do not add up to n");
    FM_REQUIRE(n < (int64_t(1) << 32) - 1 && P < (int64_t(1) << 32) - 1, "too many received entries");
    FM_REQUIRE(n == 0 || (recv_slot && recv_ent), "null buffer");
    hipStream_t st = ctx->side;
    FM_HIP_CHECK(hipStreamWaitEvent(st, S.last_use, 0));
    // the staging of this batch's previous preparation has been consumed once its pair table was
    FM_HIP_CHECK(hipEventSynchronize(S.ready_fwd));
    hipEvent_t e0 = ctx->prof_begin(st);
    S.src_off.ensure(sizeof(int64_t) * 2 * (R + 1));
    S.pair_ptr.ensure(sizeof(int64_t) * (P + 1));
    S.pin_off.ensure(sizeof(int64_t) * 2 * (R + 1));
    std::memcpy(S.pin_off.p, off.data(), sizeof(int64_t) * 2 * (R + 1));
    FM_HIP_CHECK(hipMemcpyAsync(S.src_off.p, S.pin_off.p, sizeof(int64_t) * 2 * (R + 1), hipMemcpyHostToDevice, st));
    int64_t* pair_ptr = S.pair_ptr.as<int64_t>();
    // the pair table closes with n (pair_ptr[P])
    FM_HIP_CHECK(hipMemcpyAsync(pair_ptr + P, S.src_off.as<int64_t>() + R, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
    // the slot sort's payload: {pair index at this owner, x}; one source numbers its pairs from 0,
    // so the received entries already are that (no copy)
    const uint2* ent2 = reinterpret_cast<const uint2*>(recv_ent);
    if (n > 0) {
      if (R > 1) {
        ctx->sh_ent2.ensure(sizeof(uint2) * n);
        ent2 = ctx->sh_ent2.as<uint2>();
      }
      hipLaunchKernelGGL(k_pair_table, dim3(blocks_for(n)), dim3(kBlock), 0, st, reinterpret_cast<const uint2*>(recv_ent),
                         n, S.src_off.as<int64_t>(), S.src_off.as<int64_t>() + (R + 1), R, pair_ptr,
                         R > 1 ? ctx->sh_ent2.as<uint2>() : nullptr);
      FM_HIP_CHECK(hipGetLastError());
    }
    FM_HIP_CHECK(hipEventRecord(S.ready_fwd, st));
    if (n > 0) {
      // the update's grouping: received entries sorted by slot (stable: source rank, then CSR order)
      S.skeys.ensure(sizeof(uint32_t) * n);
      S.sents.ensure(sizeof(uint2) * n);
      const uint32_t* sk = nullptr;
      const uint2* sv = nullptr;
      const uint32_t* keys = reinterpret_cast<const uint32_t*>(recv_slot);
      const int kb = bits_for(std::max<int64_t>(ctx->rows - 1, 1));
      radix_sort_pairs64(ctx->side_sort, keys, ent2, n, kb, st, &sk, &sv, S.skeys.as<uint32_t>(), S.sents.as<uint2>());
    }
    FM_HIP_CHECK(hipEventRecord(S.ready_upd, st));
    ctx->prof_end("owner_prepare", e0, st);
    S.recv_slot = reinterpret_cast<const uint32_t*>(recv_slot);
    S.recv_ent = reinterpret_cast<const uint2*>(recv_ent);
    S.n = n;
    S.P = P;
    S.prepared = true;
    return FM_OK;
  });
}

int fm_shard_owner_forward(fm_ctx* ctx, fm_batch* b, void* partials_out) {
  return guarded(ctx, [&]() -> int {
    shard_owner_partials(ctx, b, partials_out, nullptr);
    return FM_OK;
  });
}

}  // extern "C"

namespace fmhip {

void shard_owner_partials(fm_ctx* ctx, fm_batch* b, void* partials_out, uint32_t* present_out, int chunk,
                          int chunks) {
  ShardBatchState& S = shard_state(ctx, b);
  FM_REQUIRE(S.prepared, "fm_shard_owner_prepare must run on this batch first");
  FM_REQUIRE(S.P == 0 || partials_out, "null buffer");
  const int R = ctx->cfg.shard_count;
  FM_REQUIRE(chunks >= 1 && chunk >= 0 && chunk < chunks && (chunks == 1 || R <= kMaxChunkSources),
             "bad owner-forward chunk");
  hipStream_t st = ctx->stream;
  FM_HIP_CHECK(hipStreamWaitEvent(st, S.ready_fwd, 0));
  if (chunk == 0) S.fwd_e0 = ctx->prof_begin(st);  // the profile spans every chunk
  if (S.P > 0) {
    // partial forward over the pairs, rows of the local table (lazy L1 caught up on read)
    BatchDev view;
    view.n_rows = S.P;
    view.nnz = S.n;
    view.row_ptr.p = S.pair_ptr.p;
    view.col.p = const_cast<uint32_t*>(S.recv_slot);
    view.ent.p = const_cast<uint2*>(S.recv_ent);
    StepParams p{};
    p.cumE = ctx->cum_host.back();
    int64_t nblk = 0;
    FwdOut xo{};  // the partial pass (partial_out given); only the present counts and the chunk are read
    xo.pcount = present_out;
    if (chunks > 1) {
      xo.ch_off = S.src_off.as<int64_t>() + (R + 1);  // the sources' pair offsets (owner_prepare)
      xo.ch_R = R;
      xo.ch_c = chunk;
      xo.ch_C = chunks;
    }
    launch_forward(ctx->view(), view, ctx->work, p, st, &nblk, reinterpret_cast<float*>(partials_out), &xo);
    view.row_ptr.p = view.col.p = view.ent.p = nullptr;  // borrowed
    FM_HIP_CHECK(hipGetLastError());
  }
  if (chunk + 1 == chunks) {
    ctx->prof_end("owner_forward", S.fwd_e0, st);
    S.fwd_e0 = nullptr;
  }
}

void shard_combine_predict(fm_ctx* ctx, fm_batch* b, const void* partials_in, const uint32_t* present_in,
                           double lo, double hi, double* pred_dev) {
  ShardBatchState& S = shard_state(ctx, b);
  FM_REQUIRE(S.route_nnz == b->dev.nnz && (int)S.pairs_out.size() == ctx->cfg.shard_count,
             "fm_shard_route must run on this batch first");
  const int R = ctx->cfg.shard_count;
  const int64_t B = b->dev.n_rows;
  if (B == 0) return;
  int64_t Ps = 0;
  for (int o = 0; o < R; ++o) Ps += S.pairs_out[o];
  FM_REQUIRE(Ps == 0 || (partials_in && present_in), "null buffer");
  const int kp = ctx->kp;
  const int GS = team_for(kp / 4);
  int64_t blocks = std::max<int64_t>((B + kBlock / GS - 1) / (kBlock / GS), 1);
  if (blocks > 256 * 8) blocks = 256 * 8;
  const float* pv = reinterpret_cast<const float*>(partials_in);
  const float2* ps = reinterpret_cast<const float2*>(pv ? pv + Ps * kp : nullptr);
  const int32_t* pi = S.pairidx.as<int32_t>();
  const int64_t* poff = S.poff.as<int64_t>();
  const double w0 = ctx->cfg.w0;
  hipStream_t st = ctx->stream;
  const dim3 grid((unsigned)blocks), blk(kBlock);
  switch (GS) {
    case 1: hipLaunchKernelGGL(k_shard_predict<1>, grid, blk, 0, st, pi, poff, R, B, pv, ps, present_in, kp, w0, lo, hi, pred_dev); break;
    case 2: hipLaunchKernelGGL(k_shard_predict<2>, grid, blk, 0, st, pi, poff, R, B, pv, ps, present_in, kp, w0, lo, hi, pred_dev); break;
    case 4: hipLaunchKernelGGL(k_shard_predict<4>, grid, blk, 0, st, pi, poff, R, B, pv, ps, present_in, kp, w0, lo, hi, pred_dev); break;
    case 8: hipLaunchKernelGGL(k_shard_predict<8>, grid, blk, 0, st, pi, poff, R, B, pv, ps, present_in, kp, w0, lo, hi, pred_dev); break;
    default: hipLaunchKernelGGL(k_shard_predict<16>, grid, blk, 0, st, pi, poff, R, B, pv, ps, present_in, kp, w0, lo, hi, pred_dev); break;
  }
  FM_HIP_CHECK(hipGetLastError());
}

}  // namespace fmhip

extern "C" {

int fm_shard_combine(fm_ctx* ctx, fm_batch* b, const void* partials_in, void* s_send) {
  return guarded(ctx, [&]() -> int {
    ShardBatchState& S = shard_state(ctx, b);
    FM_REQUIRE(S.route_nnz == b->dev.nnz && (int)S.pairs_out.size() == ctx->cfg.shard_count,
               "fm_shard_route must run on this batch first");
    const int R = ctx->cfg.shard_count;
    const int64_t B = b->dev.n_rows;
    int64_t Ps = 0;
    for (int o = 0; o < R; ++o) Ps += S.pairs_out[o];
    FM_REQUIRE(Ps == 0 || (partials_in && s_send), "null buffer");
    hipStream_t st = ctx->stream;
    hipEvent_t e0 = ctx->prof_begin(st);
    const int nq = ctx->kp / 4;
    const int GS = team_for(nq);
    const int64_t tpb = kBlock / GS;
    int64_t blocks = std::max<int64_t>((B + tpb - 1) / tpb, 1);
    if (blocks > 256 * 8) blocks = 256 * 8;
    ctx->work.loss_part.ensure(sizeof(double) * 2 * 256 * 8);  // reserve_work's size: no reallocation later
    const int32_t* pi = S.pairidx.as<int32_t>();
    const int64_t* poff = S.poff.as<int64_t>();
    const int kp = ctx->kp;
    const float* pin = reinterpret_cast<const float*>(partials_in);
    const float2* psc = reinterpret_cast<const float2*>(pin ? pin + Ps * kp : nullptr);
    float* so = reinterpret_cast<float*>(s_send);
    float2* ssc = reinterpret_cast<float2*>(so ? so + Ps * kp : nullptr);
    const double* lab = b->dev.label.as<double>();
    double2* lp = ctx->work.loss_part.as<double2>();
    const double w0 = ctx->cfg.w0;
    const dim3 grid((unsigned)blocks), blk(kBlock);
    if (R <= 8) {
      switch (GS) {
        case 1: hipLaunchKernelGGL((k_shard_combine<1, 8>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 2: hipLaunchKernelGGL((k_shard_combine<2, 8>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 4: hipLaunchKernelGGL((k_shard_combine<4, 8>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 8: hipLaunchKernelGGL((k_shard_combine<8, 8>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        default: hipLaunchKernelGGL((k_shard_combine<16, 8>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
      }
    } else {
      switch (GS) {
        case 1: hipLaunchKernelGGL((k_shard_combine<1, 0>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 2: hipLaunchKernelGGL((k_shard_combine<2, 0>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 4: hipLaunchKernelGGL((k_shard_combine<4, 0>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        case 8: hipLaunchKernelGGL((k_shard_combine<8, 0>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
        default: hipLaunchKernelGGL((k_shard_combine<16, 0>), grid, blk, 0, st, pi, poff, R, B, pin, psc, lab, kp, w0, so, ssc, lp); break;
      }
    }
    FM_HIP_CHECK(hipGetLastError());
    ctx->prof_end("combine", e0, st);
    S.loss_blocks = blocks;
    S.combined = true;
    return FM_OK;
  });
}

int fm_shard_owner_update(fm_ctx* ctx, fm_batch* b, const void* s_recv, int32_t t, double step_size,
                          double reg_param, int64_t global_rows) {
  return guarded(ctx, [&]() -> int {
    ShardBatchState& S = shard_state(ctx, b);
    FM_REQUIRE(global_rows >= 0, "negative global_rows");
    if (global_rows == 0) return FM_NOTHING_TO_DO;  // SGD.scala:126-128 (every rank skips)
    FM_REQUIRE(t >= 1, "iteration index t must be >= 1");
    FM_REQUIRE(std::isfinite(step_size) && std::isfinite(reg_param), "non-finite step size / regParam");
    FM_REQUIRE(S.prepared && S.combined, "owner_prepare, owner_forward and combine must run on this batch first");
    const int64_t n = S.n;
    FM_REQUIRE(S.P == 0 || s_recv != nullptr, "null buffer");
    hipStream_t st = ctx->stream;
    StepParams p = shard_params(ctx, t, step_size, reg_param, global_rows);
    ctx->ensure_hist(ctx->epoch + 1);
    double* stats = ctx->loss_hist.as<double>() + 3 * (int64_t)ctx->epoch;
    FM_HIP_CHECK(hipStreamWaitEvent(st, S.ready_upd, 0));
    hipEvent_t e0 = ctx->prof_begin(st);
    const float* Srow = reinterpret_cast<const float*>(s_recv);  // [P][kp] S, then [P] {r, yhat}
    const int kp = ctx->kp;
    SegSource src{Srow, kp, reinterpret_cast<const float2*>(Srow ? Srow + S.P * kp : nullptr), 1};
    if (s_rec_yl(kp) && S.P > 0) {
      // one record per pair (S and {r, yhat} in one line), as the single-table step's
      const int rec = s_rec_floats(kp);
      ctx->work.S.ensure(sizeof(float) * (size_t)S.P * rec);
      const int64_t nq = S.P * (rec / 4);
      hipLaunchKernelGGL(k_pack_srec, dim3(blocks_for(nq)), dim3(kBlock), 0, st, Srow, src.yl, S.P, kp, rec,
                         ctx->work.S.as<float>());
      FM_HIP_CHECK(hipGetLastError());
      src = SegSource{ctx->work.S.as<float>(), rec, reinterpret_cast<const float2*>(ctx->work.S.as<float>() + kp), rec / 2};
    }
    launch_segment_update(ctx->view(), n, src, ctx->work, p, S.skeys.as<uint32_t>(), S.sents.as<uint2>(),
                          S.loss_blocks, stats, st);
    ctx->prof_end("owner_update", e0, st);
    FM_HIP_CHECK(hipEventRecord(S.last_use, st));
    // the iteration's last main-stream read of this rank's batch (its combine read the labels before
    // this): a refill of the batch (fm_batch_from_rows, copy stream) waits for it
    if (b->last_use) FM_HIP_CHECK(hipEventRecord(b->last_use, st));
    ctx->epoch += 1;
    ctx->cum_host.push_back(p.cum_next);
    S.prepared = false;
    S.combined = false;
    S.recv_slot = nullptr;
    S.recv_ent = nullptr;
    return FM_OK;
  });
}

}  // extern "C"
