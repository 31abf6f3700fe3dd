// FM SGD step kernels for gfx950 (MI355X).
//
// One iteration of FactorizationMachinesSGD.runMiniBatchSGD's fold body
// (FactorizationMachinesSGD.scala:116-211) is, on the device:
//
//   k_forward          sample-major.  A team of TEAM lanes owns one sample; GS lanes hold one
//                      k-wide V row as float4 quads (coalesced 16 B per lane), so a pass covers
//                      TEAM/GS of the sample's entries.  Pending L1 is applied on the fly
//                      (lazy soft-threshold, see below).  Computes vfxiSum (S), the linear and
//                      v^2 x^2 terms with fp64 accumulation, yhat and the loss partial
//                      (FactorizationMachinesModel.scala:173-233).
//   radix sort         (fm_sort.hip) entries by feature slot -> CSC order, stable.
//   k_segment_update   feature-major.  One wave per 64 sorted entries, one lane per entry:
//                      per-entry gradient (SGD.scala:145-146, keeping the reference's
//                      x*yhat - y w-gradient), fixed-order segmented scan across lanes, and
//                      the tail lane of every complete run applies the fused update + L1
//                      (SGD.scala:150-181) to its row.  Runs that cross a 64-entry chunk write
//                      fp64 partials instead.
//   k_segment_combine  sums the partials of crossing runs in chunk order and applies the same
//                      update; block 0 also closes the step (loss sum, epoch bookkeeping).
//
// Lazy L1.  The reference soft-thresholds EVERY model row every iteration (outer joins,
// SGD.scala:157-181).  S_b(S_a(z)) = S_{a+b}(z) for a, b >= 0, so each row keeps the epoch t
// through which it is current and cum[] holds the running sum of lambda over executed steps;
// a row read at epoch E is first brought current by S_{cum[E]-cum[t]}.  Export flushes.
#include "fm_internal.h"

namespace fmhip {

namespace {

constexpr int kBlock = 256;

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

// Row of `slot` brought current to epoch E (cumE = cum[E]).  Absent rows read as zero.
__device__ __forceinline__ void load_row_quad(const TableView& T, uint32_t slot, int q, bool qok,
                                              double cumE, float& w, float4& v, bool& present) {
  const WT wt = T.wt[slot];
  v = qok ? *reinterpret_cast<const float4*>(T.V + (int64_t)slot * T.kp + q * 4)
          : make_float4(0.f, 0.f, 0.f, 0.f);
  present = wt.t >= 0;
  w = wt.w;
  if (!present) {
    w = 0.f;
    v = make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    const double a = cumE - T.cum[wt.t];
    if (a > 0.0) {
      w = shrink_f(w, a);
      v = shrink4(v, a);
    }
  }
}

// ------------------------------------------------------------------------ forward
template <int GS, int TEAM>
__global__ __launch_bounds__(kBlock) void k_forward(TableView T, const int64_t* __restrict__ row_ptr,
                                                    const uint32_t* __restrict__ col,
                                                    const float* __restrict__ val,
                                                    const float* __restrict__ label, int64_t B,
                                                    double w0, int32_t epoch, float* __restrict__ S_out,
                                                    float2* __restrict__ yl_out, int2* __restrict__ rec_out,
                                                    double2* __restrict__ loss_part) {
  constexpr int RPP = TEAM / GS;  // rows (entries) per pass
  constexpr int TPB = kBlock / TEAM;
  const int tid = threadIdx.x;
  const int tl = tid % TEAM;
  const int g = tl % GS;
  const int rs = tl / GS;
  const int kp = T.kp;
  const bool qok = g * 4 < kp;
  const double cumE = T.cum[epoch];
  double loss_acc = 0.0, nloss = 0.0;

  for (int64_t s = (int64_t)blockIdx.x * TPB + tid / TEAM; s < B; s += (int64_t)gridDim.x * TPB) {
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, vv = 0.0, wx = 0.0;
    int64_t e = e0 + rs;
    // 2-deep unroll: issue both entries' gathers before consuming them
    for (; e + RPP < e1; e += 2 * RPP) {
      const uint32_t id0 = col[e], id1 = col[e + RPP];
      const float x0 = val[e], x1 = val[e + RPP];
      float w_0, w_1;
      float4 v0, v1;
      bool p0, p1;
      load_row_quad(T, id0, g, qok, cumE, w_0, v0, p0);
      load_row_quad(T, id1, g, qok, cumE, w_1, v1, p1);
      {
        const double x = x0;
        a0 += (double)v0.x * x; a1 += (double)v0.y * x; a2 += (double)v0.z * x; a3 += (double)v0.w * x;
        const double v2 = (double)v0.x * v0.x + (double)v0.y * v0.y + (double)v0.z * v0.z + (double)v0.w * v0.w;
        vv += v2 * x * x;
        if (g == 0) wx += (double)w_0 * x;
      }
      {
        const double x = x1;
        a0 += (double)v1.x * x; a1 += (double)v1.y * x; a2 += (double)v1.z * x; a3 += (double)v1.w * x;
        const double v2 = (double)v1.x * v1.x + (double)v1.y * v1.y + (double)v1.z * v1.z + (double)v1.w * v1.w;
        vv += v2 * x * x;
        if (g == 0) wx += (double)w_1 * x;
      }
      if (g == 0) {
        rec_out[e] = make_int2((int)s, __float_as_int(x0));
        rec_out[e + RPP] = make_int2((int)s, __float_as_int(x1));
      }
    }
    for (; e < e1; e += RPP) {
      const uint32_t id0 = col[e];
      const float x0 = val[e];
      float w_0;
      float4 v0;
      bool p0;
      load_row_quad(T, id0, g, qok, cumE, w_0, v0, p0);
      const double x = x0;
      a0 += (double)v0.x * x; a1 += (double)v0.y * x; a2 += (double)v0.z * x; a3 += (double)v0.w * x;
      const double v2 = (double)v0.x * v0.x + (double)v0.y * v0.y + (double)v0.z * v0.z + (double)v0.w * v0.w;
      vv += v2 * x * x;
      if (g == 0) {
        wx += (double)w_0 * x;
        rec_out[e] = make_int2((int)s, __float_as_int(x0));
      }
    }
    // sum the row slots (lanes with equal g), then the whole team for the scalars
#pragma unroll
    for (int o = GS; o < TEAM; o <<= 1) {
      a0 += __shfl_xor(a0, o); a1 += __shfl_xor(a1, o);
      a2 += __shfl_xor(a2, o); a3 += __shfl_xor(a3, o);
    }
#pragma unroll
    for (int o = 1; o < TEAM; o <<= 1) {
      vv += __shfl_xor(vv, o);
      wx += __shfl_xor(wx, o);
    }
    double ss = qok ? a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3 : 0.0;
#pragma unroll
    for (int o = 1; o < GS; o <<= 1) ss += __shfl_xor(ss, o);
    // sumVx + wixiSum + w0 (Model.scala:221, :260-262)
    const double yhat = 0.5 * (ss - vv) + wx + w0;
    if (rs == 0 && qok)
      *reinterpret_cast<float4*>(S_out + s * kp + g * 4) = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
    if (tl == 0) {
      const float y = label[s];
      yl_out[s] = make_float2((float)yhat, y);
      if (e1 > e0) {
        const double d = yhat - (double)y;
        loss_acc += d * d;  // pow(pred - label, 2.0), Model.scala:230
        nloss += 1.0;
      }
    }
  }
  // deterministic block reduction of the loss partials
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

// -------------------------------------------------------------- segmented update
struct SegArgs {
  TableView T;
  const uint32_t* skeys;
  const uint32_t* svals;
  int64_t N;
  const int2* rec;
  const float* S;
  const float2* yl;
  double* part;  // [nchunks][2][kp + 1]
  int64_t nchunks;
  StepParams p;
  unsigned long long* n_unique;
};

__device__ __forceinline__ double seg_scan(double v, int lane, int start_lane) {
  // inclusive segmented scan over lanes [start_lane, lane]; fixed (tree) order
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o);
    if (lane - o >= start_lane) v += t;
  }
  return v;
}

// Row update of SGD.scala:150-181 for one factor quad, fp64:
//   vec' = S_lambda(vec - sum * (eta / m))
__device__ __forceinline__ float upd_v(float v, double g, const StepParams& p) {
  return (float)shrink_d((double)v - g * p.scale_v, p.lam);
}

template <int Q>
__global__ __launch_bounds__(kBlock) void k_segment_update(SegArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t chunk = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  if (chunk >= a.nchunks) return;  // wave-uniform
  const TableView& T = a.T;
  const int kp = T.kp, nq = kp >> 2;
  const int64_t p0 = chunk * 64;
  const int64_t pp = p0 + lane;
  const bool valid = pp < a.N;
  const uint32_t kNone = 0xFFFFFFFFu;
  const uint32_t key = valid ? a.skeys[pp] : kNone;
  const uint32_t e = valid ? a.svals[pp] : 0u;
  uint32_t prev_key = __shfl_up(key, 1);
  uint32_t next_key = __shfl_down(key, 1);
  if (lane == 0) prev_key = p0 > 0 ? a.skeys[p0 - 1] : kNone;
  if (lane == 63) next_key = (p0 + 64 < a.N) ? a.skeys[p0 + 64] : kNone;
  if (pp == a.N - 1) next_key = kNone;
  const bool seg_start = valid && key != prev_key;  // a run of this key starts here
  const bool seg_end = valid && key != next_key;     // ... ends here
  const bool piece_head = valid && (lane == 0 || seg_start);
  const bool piece_tail = valid && (lane == 63 || seg_end);
  const uint64_t heads = __ballot(piece_head);
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  const int start_lane = 63 - __clzll(heads & upto);
  const uint64_t starts = __ballot(seg_start);
  if (lane == 0 && starts) atomicAdd(a.n_unique, (unsigned long long)__popcll(starts));
  // the piece is a whole run iff its head lane starts the run and its tail lane ends it
  const bool head_is_start = (starts >> start_lane) & 1ull;
  const bool complete = head_is_start && seg_end;
  // partial slot: 0 = the chunk's first piece continuing from the previous chunk (also used
  // when that piece spans the whole chunk), 1 = the last piece continuing into the next chunk
  const int slot = (start_lane == 0 && !head_is_start) ? 0 : 1;
  double* prow = a.part + ((chunk * 2 + slot) * (int64_t)(kp + 1));

  // per-entry inputs: (s, x) from the forward's record, (yhat, y) of its sample
  int2 rc = valid ? a.rec[e] : make_int2(0, 0);
  const int s = rc.x;
  const double x = valid ? (double)__int_as_float(rc.y) : 0.0;
  const float2 yl = valid ? a.yl[s] : make_float2(0.f, 0.f);
  const double yhat = yl.x, y = yl.y;
  const double r = yhat - y;
  const double cumE = T.cum[a.p.epoch];

  // ---- linear term: g_w = deltaWi * pred - label (SGD.scala:145)
  double gw = valid ? x * yhat - y : 0.0;
  gw = seg_scan(gw, lane, start_lane);
  WT wt = valid ? T.wt[key] : WT{0.f, -1};
  if (piece_tail) {
    if (complete) {
      float w = wt.w;
      if (wt.t < 0) {
        w = 0.f;
      } else {
        const double ac = cumE - T.cum[wt.t];
        if (ac > 0.0) w = shrink_f(w, ac);
      }
      // strength - (sum/m)*eta, then S_lambda (SGD.scala:150, :171, :179)
      const double wn = shrink_d((double)w - (gw / a.p.m) * a.p.eta, a.p.lam);
      WT o;
      o.w = (float)wn;
      o.t = a.p.epoch + 1;
      T.wt[key] = o;
    } else {
      prow[0] = gw;
    }
  }
  // ---- interaction term: g_V = (vfxiSum*x - (v*x)*x) * (pred - label) (Model.scala:201-204,
  //      SGD.scala:146), in chunks of Q quads
  for (int qc = 0; qc < nq; qc += Q) {
    double c[4 * Q];
    float4 vq[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int q = qc + j;
      if (valid && q < nq) {
        const float4 sq = *reinterpret_cast<const float4*>(a.S + (int64_t)s * kp + q * 4);
        float w_unused;
        bool pres;
        load_row_quad(T, key, q, true, cumE, w_unused, vq[j], pres);
        c[4 * j + 0] = ((double)sq.x * x - ((double)vq[j].x * x) * x) * r;
        c[4 * j + 1] = ((double)sq.y * x - ((double)vq[j].y * x) * x) * r;
        c[4 * j + 2] = ((double)sq.z * x - ((double)vq[j].z * x) * x) * r;
        c[4 * j + 3] = ((double)sq.w * x - ((double)vq[j].w * x) * x) * r;
      } else {
        vq[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        c[4 * j + 0] = c[4 * j + 1] = c[4 * j + 2] = c[4 * j + 3] = 0.0;
      }
    }
#pragma unroll
    for (int i = 0; i < 4 * Q; ++i) c[i] = seg_scan(c[i], lane, start_lane);
    if (piece_tail) {
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        const int q = qc + j;
        if (q >= nq) continue;
        if (complete) {
          float4 o;
          o.x = upd_v(vq[j].x, c[4 * j + 0], a.p);
          o.y = upd_v(vq[j].y, c[4 * j + 1], a.p);
          o.z = upd_v(vq[j].z, c[4 * j + 2], a.p);
          o.w = upd_v(vq[j].w, c[4 * j + 3], a.p);
          *reinterpret_cast<float4*>(T.V + (int64_t)key * kp + q * 4) = o;
        } else {
          prow[1 + 4 * q + 0] = c[4 * j + 0];
          prow[1 + 4 * q + 1] = c[4 * j + 1];
          prow[1 + 4 * q + 2] = c[4 * j + 2];
          prow[1 + 4 * q + 3] = c[4 * j + 3];
        }
      }
    }
  }
}

// Runs that cross chunk boundaries: the chunk holding the run's first entry owns it and
// adds the following chunks' head partials in chunk order.  Block 0 also closes the step.
__global__ __launch_bounds__(kBlock) void k_segment_combine(SegArgs a, const double2* __restrict__ loss_part,
                                                            int64_t n_loss_blocks,
                                                            double* __restrict__ cum_w,
                                                            double* __restrict__ stats_out) {
  const int kp = a.T.kp;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double l = 0.0, c = 0.0;
    for (int64_t i = 0; i < n_loss_blocks; ++i) {
      l += loss_part[i].x;
      c += loss_part[i].y;
    }
    stats_out[0] = l;
    stats_out[1] = c;
    stats_out[2] = (double)(*a.n_unique);
    cum_w[a.p.epoch + 1] = a.p.cum_next;
  }
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (chunk >= a.nchunks) return;
  const int64_t p0 = chunk * 64;
  const int64_t p1 = p0 + 64 < a.N ? p0 + 64 : a.N;
  if (p1 >= a.N) return;                            // nothing continues past the last chunk
  const uint32_t key = a.skeys[p1 - 1];
  if (a.skeys[p1] != key) return;                   // last run ends inside this chunk
  // does the last run start inside this chunk?  (otherwise an earlier chunk owns it)
  if (a.skeys[p0] == key && p0 > 0 && a.skeys[p0 - 1] == key) return;
  const TableView& T = a.T;
  const double cumE = T.cum[a.p.epoch];
  const double* tail = a.part + (chunk * 2 + 1) * (int64_t)(kp + 1);
  // the owner chunk's piece was written to slot 1, unless it is also the chunk's first piece
  // that continues from before (excluded above) -> always slot 1 here.
  double gw = tail[0];
  int64_t c2 = chunk + 1;
  while (c2 < a.nchunks && a.skeys[c2 * 64] == key) {
    gw += a.part[(c2 * 2 + 0) * (int64_t)(kp + 1)];
    ++c2;
  }
  WT wt = T.wt[key];
  const bool present = wt.t >= 0;
  const double ac = present ? cumE - T.cum[wt.t] : 0.0;
  float w = present ? wt.w : 0.f;
  if (ac > 0.0) w = shrink_f(w, ac);
  WT o;
  o.w = (float)shrink_d((double)w - (gw / a.p.m) * a.p.eta, a.p.lam);
  o.t = a.p.epoch + 1;
  for (int f = 0; f < kp; ++f) {
    double g = tail[1 + f];
    for (int64_t c3 = chunk + 1; c3 < c2; ++c3) g += a.part[(c3 * 2 + 0) * (int64_t)(kp + 1) + 1 + f];
    float v = present ? T.V[(int64_t)key * kp + f] : 0.f;
    if (ac > 0.0) v = shrink_f(v, ac);
    T.V[(int64_t)key * kp + f] = upd_v(v, g, a.p);
  }
  T.wt[key] = o;
}

// ---------------------------------------------------------------- table utilities
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// N(0, sd^2) draw keyed by (seed, feature id, factor f; f = -1 for w).  Box-Muller in fp64.
__device__ __forceinline__ float gauss_draw(uint64_t seed, int64_t id, int f, double sd) {
  const uint64_t c = ((uint64_t)id << 10) ^ (uint64_t)(f + 1);
  const uint64_t h1 = splitmix64(seed ^ splitmix64(c));
  const uint64_t h2 = splitmix64(h1 ^ 0x632BE59BD9B4E019ull);
  const double u1 = (double)((h1 >> 11) + 1) * 0x1.0p-53;
  const double u2 = (double)(h2 >> 11) * 0x1.0p-53;
  const double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  return (float)(g * sd);
}

__global__ void k_init_random(TableView T, const int32_t* __restrict__ ids, int64_t n, int64_t id_begin,
                              uint64_t seed, double sd, int32_t epoch) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids ? (int64_t)ids[i] : id_begin + i;
    if (id % T.shard_count != T.shard_index) continue;
    const int64_t slot = id / T.shard_count;
    if (slot >= T.rows) continue;
    WT o;
    o.w = gauss_draw(seed, id, -1, sd);
    o.t = epoch;
    for (int f = 0; f < T.kp; ++f) T.V[slot * T.kp + f] = f < T.k ? gauss_draw(seed, id, f, sd) : 0.f;
    T.wt[slot] = o;
  }
}

__global__ void k_load_rows(TableView T, const int32_t* __restrict__ ids, int64_t n, const double* __restrict__ w,
                            const double* __restrict__ V, int32_t epoch) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids[i];
    if (id % T.shard_count != T.shard_index) continue;
    const int64_t slot = id / T.shard_count;
    if (slot >= T.rows) continue;
    WT o;
    o.w = (float)w[i];
    o.t = epoch;
    for (int f = 0; f < T.kp; ++f) T.V[slot * T.kp + f] = f < T.k ? (float)V[i * T.k + f] : 0.f;
    T.wt[slot] = o;
  }
}

__global__ void k_table_reset(TableView T) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x) {
    WT o;
    o.w = 0.f;
    o.t = -1;
    T.wt[i] = o;
  }
}

__global__ void k_flush(TableView T, int32_t epoch) {
  const double cumE = T.cum[epoch];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x) {
    WT wt = T.wt[i];
    if (wt.t < 0 || wt.t == epoch) continue;
    const double a = cumE - T.cum[wt.t];
    if (a > 0.0) {
      wt.w = shrink_f(wt.w, a);
      for (int f = 0; f < T.kp; ++f) T.V[i * T.kp + f] = shrink_f(T.V[i * T.kp + f], a);
    }
    wt.t = epoch;
    T.wt[i] = wt;
  }
}

__global__ void k_count_present(TableView T, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x)
    c += T.wt[i].t >= 0 ? 1ull : 0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// FactorizationMachinesModel.predict/transform (Model.scala:69-133), one thread per sample.
// Global ids arrive in b.col; ids >= num_features or absent from the model are dropped.
__global__ void k_predict(TableView T, const int64_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
                          const float* __restrict__ val, int64_t B, int64_t num_features, int32_t epoch,
                          double w0, double lo, double hi, double* __restrict__ pred) {
  const double cumE = T.cum[epoch];
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B; s += (int64_t)gridDim.x * blockDim.x) {
    double acc[64];
    for (int f = 0; f < 64; ++f) acc[f] = 0.0;
    double wx = 0.0, vv = 0.0;
    int n = 0;
    for (int64_t e = row_ptr[s]; e < row_ptr[s + 1]; ++e) {
      const int64_t id = col[e];
      if (id >= num_features) continue;
      const WT wt = T.wt[id];
      if (wt.t < 0) continue;
      const double a = cumE - T.cum[wt.t];
      const double x = val[e];
      const float w = a > 0.0 ? shrink_f(wt.w, a) : wt.w;
      wx += (double)w * x;
      double v2 = 0.0;
      for (int f = 0; f < T.k; ++f) {
        float v = T.V[id * T.kp + f];
        if (a > 0.0) v = shrink_f(v, a);
        acc[f & 63] += (double)v * x;  // k <= 64 on this path (checked on the host)
        v2 += (double)v * v;
      }
      vv += v2 * x * x;
      ++n;
    }
    if (n == 0) {
      pred[s] = w0;  // na.fill(globalBias), Model.scala:86 (unclamped)
    } else {
      double ss = 0.0;
      for (int f = 0; f < T.k; ++f) ss += acc[f] * acc[f];
      const double yhat = 0.5 * (ss - vv) + wx + w0;
      pred[s] = fmin(fmax(yhat, lo), hi);  // least(greatest(pred, min), max), :131
    }
  }
}

// calcLossGrad per-entry outputs (Model.scala:135-234), one thread per sample.
__global__ void k_loss_grad(TableView T, const int64_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
                            const float* __restrict__ val, const float* __restrict__ label, int64_t B,
                            int32_t epoch, double w0, double* pred, double* loss, double* dw, double* dv,
                            int32_t* absent) {
  const double cumE = T.cum[epoch];
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B; s += (int64_t)gridDim.x * blockDim.x) {
    double acc[64];
    for (int f = 0; f < 64; ++f) acc[f] = 0.0;
    double wx = 0.0, vv = 0.0;
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t id = col[e];
      const WT wt = T.wt[id];
      if (wt.t < 0) {
        *absent = 1;
        continue;
      }
      const double a = cumE - T.cum[wt.t];
      const double x = val[e];
      const float w = a > 0.0 ? shrink_f(wt.w, a) : wt.w;
      wx += (double)w * x;
      double v2 = 0.0;
      for (int f = 0; f < T.k; ++f) {
        float v = T.V[id * T.kp + f];
        if (a > 0.0) v = shrink_f(v, a);
        acc[f & 63] += (double)v * x;
        v2 += (double)v * v;
      }
      vv += v2 * x * x;
    }
    double ss = 0.0;
    for (int f = 0; f < T.k; ++f) ss += acc[f] * acc[f];
    const double yhat = 0.5 * (ss - vv) + wx + w0;
    const double d = yhat - (double)label[s];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t id = col[e];
      const WT wt = T.wt[id];
      const double x = val[e];
      if (pred) pred[e] = yhat;
      if (loss) loss[e] = d * d;
      if (dw) dw[e] = x;
      if (dv) {
        const double a = wt.t >= 0 ? cumE - T.cum[wt.t] : 0.0;
        for (int f = 0; f < T.k; ++f) {
          float v = wt.t >= 0 ? T.V[id * T.kp + f] : 0.f;
          if (a > 0.0) v = shrink_f(v, a);
          dv[e * T.k + f] = acc[f & 63] * x - ((double)v * x) * x;
        }
      }
    }
  }
}

// groupBy(key).agg(VectorSum(vec)) on sorted keys: each run summed sequentially in input
// order (the stable sort keeps it), FactorizationMachines.scala:56-67.
__global__ void k_segment_sum(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals, int64_t n,
                              const double* __restrict__ vecs, int32_t k, const uint32_t* __restrict__ run_index,
                              int32_t* __restrict__ out_keys, double* __restrict__ out_sums) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (i > 0 && skeys[i - 1] == skeys[i]) continue;
    const uint32_t r = run_index[i];
    out_keys[r] = (int32_t)skeys[i];
    for (int f = 0; f < k; ++f) {
      double acc = 0.0;
      for (int64_t j = i; j < n && skeys[j] == skeys[i]; ++j) acc += vecs[(int64_t)svals[j] * k + f];
      out_sums[(int64_t)r * k + f] = acc;
    }
  }
}

__global__ void k_run_index(const uint32_t* __restrict__ skeys, int64_t n, uint32_t* __restrict__ run_index,
                            int64_t* __restrict__ n_out) {
  // single block: exclusive scan of run-start flags
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t b = 0; b < n; b += kBlock) {
    const int64_t i = b + threadIdx.x;
    const uint32_t f = (i < n && (i == 0 || skeys[i - 1] != skeys[i])) ? 1u : 0u;
    uint32_t v = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      wpre += w < wave ? wsum[w] : 0u;
      tot += wsum[w];
    }
    if (i < n) run_index[i] = carry + wpre + v - f;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_out = carry;
}

inline unsigned grid_for(int64_t n, int block, int64_t cap = 256 * 16) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

template <int GS, int TEAM>
void launch_fwd_t(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                  int64_t* nblk) {
  constexpr int TPB = kBlock / TEAM;
  int64_t blocks = (b.n_rows + TPB - 1) / TPB;
  if (blocks > 256 * 8) blocks = 256 * 8;
  if (blocks < 1) blocks = 1;
  *nblk = blocks;
  w.loss_part.ensure(sizeof(double2) * blocks);
  hipLaunchKernelGGL((k_forward<GS, TEAM>), dim3((unsigned)blocks), dim3(kBlock), 0, st, T,
                     b.row_ptr.as<int64_t>(), b.col.as<uint32_t>(), b.val.as<float>(), b.label.as<float>(),
                     b.n_rows, p.w0, p.epoch, w.S.as<float>(), w.yl.as<float2>(), w.rec.as<int2>(),
                     w.loss_part.as<double2>());
}

}  // namespace

void launch_forward(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                    int64_t* n_fwd_blocks) {
  const int nq = T.kp / 4;
  if (nq <= 1) launch_fwd_t<1, 16>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 2) launch_fwd_t<2, 16>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 4) launch_fwd_t<4, 16>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 8) launch_fwd_t<8, 16>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 16) launch_fwd_t<16, 16>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 32) launch_fwd_t<32, 32>(T, b, w, p, st, n_fwd_blocks);
  else if (nq <= 64) launch_fwd_t<64, 64>(T, b, w, p, st, n_fwd_blocks);
  else FM_REQUIRE(false, "dimFactorization > 256 is not supported");
  FM_HIP_CHECK(hipGetLastError());
}

void launch_segment_update(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint32_t* svals, int64_t n_fwd_blocks,
                           double* cum_w, double* stats_out, hipStream_t st) {
  const int64_t N = b.nnz;
  const int64_t nchunks = (N + 63) / 64;
  w.part.ensure(sizeof(double) * (size_t)(nchunks > 0 ? nchunks : 1) * 2 * (T.kp + 1));
  w.stats.ensure(sizeof(unsigned long long));
  unsigned long long* n_unique = w.stats.as<unsigned long long>();
  FM_HIP_CHECK(hipMemsetAsync(n_unique, 0, sizeof(unsigned long long), st));
  SegArgs a;
  a.T = T;
  a.skeys = skeys;
  a.svals = svals;
  a.N = N;
  a.rec = w.rec.as<int2>();
  a.S = w.S.as<float>();
  a.yl = w.yl.as<float2>();
  a.part = w.part.as<double>();
  a.nchunks = nchunks;
  a.p = p;
  a.n_unique = n_unique;
  if (nchunks > 0) {
    const unsigned blocks = (unsigned)((nchunks * 64 + kBlock - 1) / kBlock);
    const int nq = T.kp / 4;
    if (nq <= 1) hipLaunchKernelGGL(k_segment_update<1>, dim3(blocks), dim3(kBlock), 0, st, a);
    else if (nq <= 2) hipLaunchKernelGGL(k_segment_update<2>, dim3(blocks), dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(k_segment_update<4>, dim3(blocks), dim3(kBlock), 0, st, a);
    FM_HIP_CHECK(hipGetLastError());
  }
  const unsigned cblocks = (unsigned)((nchunks + kBlock - 1) / kBlock) > 0 ? (unsigned)((nchunks + kBlock - 1) / kBlock) : 1u;
  hipLaunchKernelGGL(k_segment_combine, dim3(cblocks), dim3(kBlock), 0, st, a,
                     w.loss_part.as<double2>(), n_fwd_blocks, cum_w, stats_out);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_init_random(const TableView& T, const int32_t* ids, int64_t n, int64_t id_begin, uint64_t seed,
                        double sd, int32_t epoch, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_init_random, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, id_begin, seed, sd,
                     epoch);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_load_rows(const TableView& T, const int32_t* ids, int64_t n, const double* w, const double* V,
                      int32_t epoch, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_load_rows, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, w, V, epoch);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_table_reset(const TableView& T, hipStream_t st) {
  if (T.rows <= 0) return;
  FM_HIP_CHECK(hipMemsetAsync(T.V, 0, sizeof(float) * (size_t)T.rows * T.kp, st));
  hipLaunchKernelGGL(k_table_reset, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_flush(const TableView& T, int32_t epoch, hipStream_t st) {
  if (T.rows <= 0) return;
  hipLaunchKernelGGL(k_flush, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T, epoch);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_count_present(const TableView& T, int64_t* out, hipStream_t st) {
  FM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(int64_t), st));
  if (T.rows <= 0) return;
  hipLaunchKernelGGL(k_count_present, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T,
                     reinterpret_cast<unsigned long long*>(out));
  FM_HIP_CHECK(hipGetLastError());
}

void launch_predict(const TableView& T, const BatchDev& b, int32_t epoch, int64_t num_features, double w0,
                    double lo, double hi, double* pred, hipStream_t st) {
  FM_REQUIRE(T.k <= 64, "fm_predict supports dimFactorization <= 64");
  FM_REQUIRE(T.shard_count == 1, "fm_predict needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  hipLaunchKernelGGL(k_predict, dim3(grid_for(b.n_rows, kBlock)), dim3(kBlock), 0, st, T, b.row_ptr.as<int64_t>(),
                     b.col.as<uint32_t>(), b.val.as<float>(), b.n_rows, num_features, epoch, w0, lo, hi, pred);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_loss_grad(const TableView& T, const BatchDev& b, int32_t epoch, double w0, double* pred, double* loss,
                      double* dw, double* dv, int32_t* absent_flag, hipStream_t st) {
  FM_REQUIRE(T.k <= 64, "fm_loss_grad supports dimFactorization <= 64");
  FM_REQUIRE(T.shard_count == 1, "fm_loss_grad needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  hipLaunchKernelGGL(k_loss_grad, dim3(grid_for(b.n_rows, kBlock)), dim3(kBlock), 0, st, T,
                     b.row_ptr.as<int64_t>(), b.col.as<uint32_t>(), b.val.as<float>(), b.label.as<float>(),
                     b.n_rows, epoch, w0, pred, loss, dw, dv, absent_flag);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_segment_sum(const uint32_t* skeys, const uint32_t* svals, int64_t n, const double* vecs, int32_t k,
                        uint32_t* run_index, int32_t* out_keys, double* out_sums, int64_t* n_out_dev,
                        hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_run_index, dim3(1), dim3(kBlock), 0, st, skeys, n, run_index, n_out_dev);
  hipLaunchKernelGGL(k_segment_sum, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, skeys, svals, n, vecs, k,
                     run_index, out_keys, out_sums);
  FM_HIP_CHECK(hipGetLastError());
}

}  // namespace fmhip
