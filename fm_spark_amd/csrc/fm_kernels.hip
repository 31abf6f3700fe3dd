// FM SGD step kernels for gfx950 (MI355X).
//
// One iteration of FactorizationMachinesSGD.runMiniBatchSGD's fold body
// (FactorizationMachinesSGD.scala:116-211) is, on the device:
//
//   k_forward          sample-major.  A team of TEAM lanes owns one sample; GS lanes hold one
//                      k-wide V row as float4 quads (coalesced 16 B per lane), so a pass covers
//                      TEAM/GS of the sample's entries; four passes are issued before any is
//                      consumed.  Pending L1 is applied on the fly (lazy soft-threshold, below).
//                      fp64 accumulation of vfxiSum (S), the linear and v^2 x^2 terms, yhat and
//                      the loss partial (FactorizationMachinesModel.scala:173-233).
//   radix sort         (fm_sort.hip) entries by feature slot -> CSC order, stable; runs on a
//                      second stream concurrently with k_forward (it only reads the batch).
//   k_segment_update   feature-major.  One wave per 64 sorted entries, one lane per entry:
//                      per-entry gradient (SGD.scala:145-146, keeping the reference's
//                      x*yhat - y w-gradient), fixed-order segmented scan across lanes, and
//                      the tail lane of every complete run applies the fused update + L1
//                      (SGD.scala:150-181) to its row.  Runs that cross a 64-entry chunk write
//                      fp64 partials instead.
//   k_segment_combine  one wave per crossing run sums its partials in chunk order (lanes over
//                      the k+1 columns) and applies the same update; block 0 closes the step
//                      (loss sum and distinct-id count, fixed-order reductions).
//
// Lazy L1.  The reference soft-thresholds EVERY model row every iteration (outer joins,
// SGD.scala:157-181).  S_b(S_a(z)) = S_{a+b}(z) for a, b >= 0, so each row header keeps the
// cumulative shrink `cum` it has received; a row read when the running total is cumE is first
// brought current by S_{cumE - cum}.  Export flushes every row.
#include <algorithm>
#include <cstdlib>

#include "fm_device.h"


namespace fmhip {

namespace {

constexpr int kBlock = 256;
constexpr int kWaveEnt = 256;  // sorted entries per update wave
constexpr int kUpdD = 2;   // entries whose rows a lane group loads per step
// (two entries ahead at k = 5..8 or 13..16 measured slower at c2 / c5 / c3: profiles/r04_o)
constexpr int kUpdD4 = 1;  // k = 13..16 (4 lanes per entry, paired row stores): one entry ahead keeps the
                           // kernel within the 5-wave register budget
constexpr int kUpdD2 = 1;  // k = 5..8 (2 lanes per entry, paired row stores)

// The row header and one V quad brought current (absent rows read as zero).
__device__ __forceinline__ void current_row(const RowHdr& h, float4& v, float& w, double cumE) {
  if (h.t < 0) {
    w = 0.f;
    v = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  w = h.w;
  const double a = cumE - h.cum;
  if (a > 0.0) {
    w = shrink_f(w, a);
    v = shrink4(v, a);
  }
}

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

// ------------------------------------------------------------------------ forward
// MODE kTrain: the step's forward (S, {yhat, y}, loss partials).
// MODE kPartial: the sharded owner's pass (fm_shard.hip).  "Samples" are (source rank, sample)
// pairs of the entries this owner received; the output per pair is the partial vector
// sum v*x (kp fp32, S_out) and the scalars {sum v^2 x^2, sum w*x} (yl_out) instead of S / yhat / loss.
// MODE kPredict: FactorizationMachinesModel.predict (Model.scala:90-133): ids outside the table
// or absent from the model are dropped (the inner joins, :103-112), a row left without a learned
// feature scores globalBias unclamped (na.fill, :86), every other row
// least(greatest(yhat, minLabel), maxLabel) (:129-132), fp64 into pred_out.
// MODE kLossGrad: calcLossGrad's per-entry columns (Model.scala:225-233): the sample's yhat, its
// squared error, deltaWi = x and deltaVi = vfxiSum * x - (v * x) * x, fp64 from the team's fp64
// sums (a second walk over the sample's entries re-reads their rows); absent ids set the flag.
// MODE kTrainFused: kTrain, and every row whose feature has exactly one entry in the batch (a
// singleton: 92 % of a c3 batch's distinct rows) is updated here, by the sample that holds that
// entry, instead of by the segmented update (see "Singleton rows" below).
constexpr int kTrain = 0, kPartial = 1, kPredict = 2, kLossGrad = 3, kTrainFused = 4;
constexpr int kFuseNS = 5;    // kTrainFused: singleton rows per lane group and sample that wait in LDS
constexpr int kPartialU = 4;  // sharded partial pass: passes (entries per lane) whose rows are in flight together
// The step's forward (and predict / loss-grad): 32 lanes per sample, 2 passes in flight -- the
// same 16 rows in flight per sample at k = 16 as 16 lanes x 4 passes, with fewer registers per
// lane (measured 1.196 against 1.213 ms per c3 step, 5 runs each on two boxes)
constexpr int kFwdTeam = 32, kFwdU = 2;
// k <= 8 (one or two lanes per row): 3 passes in flight, 96 rows per team-sample round -- c2 0.171 /
// 0.173 against 0.175 / 0.174 ms per step (median 0.162 against 0.165), at c5 (k = 16) slower
// (profiles/r04_o)
constexpr int kFwdUNarrow = 3;
// forward blocks at most (grid-stride over samples beyond): 8192 (four samples per team at c3, one at
// c2 / c5) against 2048 in round 5, c3 0.859-0.863 against 0.867-0.869 ms, c2 0.161-0.163 against
// 0.163-0.168, c5 0.178-0.181 against 0.182-0.185 (profiles/r05_ab, r05_ac; 1024 and 32768 slower)
constexpr int kFwdGrid = 8192;
// the fused forward (kTrainFused): 5 passes in flight (40 rows per sample at k = 16, so a 39-entry
// c3 sample takes one round instead of two): round 5 at 4 waves per SIMD, c3 0.869-0.872 against
// 0.878-0.883 ms for 3 passes, 4 passes slower (profiles/r05_x); round 3 had taken 3 (-2 to -4 %
// against 2, 4 slower under the 5-wave cap: profiles/r03_v7/ab)
constexpr int kFuseU = 5;

// Singleton rows.  fm_batch_prepare sorts the batch (side stream); at the start of the step the
// split (k_split_*, main stream) keeps the runs of two or more entries (the only ones that need a
// per-feature reduction) and marks every such row in the row header's t field, the word that
// otherwise only says present (t >= 0) or absent (t = -1):
//   present, multi at epoch E : t = kTagPresent + (E & kTagMask)   (>= 2^30; normal t < 2^30)
//   absent,  multi at epoch E : t = -2 - (E & kTagMask)            (<= -2: still "absent")
// so every reader that asks t >= 0 is unchanged, and the fused forward, which loads the header of
// every entry's row anyway, knows which rows it may update in place: nobody else reads them in
// this step.  The segmented update then walks the multi runs only and rewrites their headers
// (t = E + 1), clearing the tags.
constexpr int32_t kTagPresent = 1 << 30;
constexpr int32_t kTagMask = (1 << 29) - 1;
__device__ __forceinline__ int32_t multi_tag(int32_t epoch, bool present) {
  return present ? kTagPresent + (epoch & kTagMask) : -2 - (epoch & kTagMask);
}
__device__ __forceinline__ bool is_multi(int32_t t, int32_t epoch) {
  const int32_t e = epoch & kTagMask;
  return t >= kTagPresent ? t - kTagPresent == e : (t <= -2 && -2 - t == e);
}

// The fused forward at 4 waves per SIMD (107 VGPRs, no spill).  Round 3 measured 5 waves (96
// VGPRs, a few spilled) faster: c3 step 0.98 against 1.03 ms (profiles/r03_v9/ab, r03_v10/ab);
// with the small kernels' latency chains cut (round 5) the spills cost more than the fifth wave
// buys: 0.881-0.882 against 0.892-0.894 ms, five alternating reps (profiles/r05_w2).  6 waves (80
// VGPRs, more spills) measured 1.066 in round 3.  The other modes keep the compiler's choice.
template <int MODE, int GS>
constexpr int fwd_min_waves() { return MODE == kTrainFused && GS == 4 ? 4 : 1; }  // k = 9..16 (smaller
// k: the stash's LDS holds the block count below 4 waves anyway)
template <int GS, int TEAM, int MODE, int U>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(fwd_min_waves<MODE, GS>())))
void k_forward(TableView T, const int64_t* __restrict__ row_ptr,
                                                    const uint32_t* __restrict__ col,
                                                    const uint2* __restrict__ ent, const float* __restrict__ xs,
                                                    const double* __restrict__ label, int64_t B,
                                                    double w0, double cumE, float* __restrict__ S_out,
                                                    float2* __restrict__ yl_out, int64_t sstr, int64_t ystr,
                                                    double2* __restrict__ loss_part,
                                                    FwdOut xo) {
  constexpr bool PARTIAL = MODE == kPartial;
  constexpr int RPP = TEAM / GS;  // entries per pass
  constexpr int TPB = kBlock / TEAM;
  const int tid = threadIdx.x;
  const int tl = tid % TEAM;
  const int g = tl % GS;
  const int rs = tl / GS;
  const int kp = T.kp;
  const bool qok = g * 4 < kp;
  double loss_acc = 0.0, nloss = 0.0;
  // calcLossGrad's draw for an entry whose id the model lacks (columns 4g .. 4g + 3 of k; f = -1: w)
  auto fill_row = [&](int64_t e, float4& v, float& w) {
    const int c = 4 * g, k = T.k;
    v = make_float4(c + 0 < k ? gauss_draw(xo.fill_seed, e, c + 0, xo.fill_sd) : 0.f,
                    c + 1 < k ? gauss_draw(xo.fill_seed, e, c + 1, xo.fill_sd) : 0.f,
                    c + 2 < k ? gauss_draw(xo.fill_seed, e, c + 2, xo.fill_sd) : 0.f,
                    c + 3 < k ? gauss_draw(xo.fill_seed, e, c + 3, xo.fill_sd) : 0.f);
    w = gauss_draw(xo.fill_seed, e, -1, xo.fill_sd);
  };
  // kPartial over one chunk of the pairs: the chunk's pairs numbered source by source
  __shared__ int64_t ch_base[PARTIAL ? kMaxChunkSources + 1 : 1], ch_start[PARTIAL ? kMaxChunkSources : 1];
  const bool chunked = PARTIAL && xo.ch_C > 1;
  int64_t Bl = B;
  if (chunked) {
    if (tid == 0) {
      int64_t acc = 0;
      for (int r = 0; r < xo.ch_R; ++r) {
        const int64_t p0 = xo.ch_off[r], P = xo.ch_off[r + 1] - p0;
        const int64_t lo = P * xo.ch_c / xo.ch_C, hi = P * (xo.ch_c + 1) / xo.ch_C;
        ch_start[r] = p0 + lo;
        ch_base[r] = acc;
        acc += hi - lo;
      }
      ch_base[xo.ch_R] = acc;
    }
    __syncthreads();
    Bl = ch_base[xo.ch_R];
  }

  // kTrainFused (kp <= 16): each lane group keeps, in LDS, the singleton rows among the entries it
  // gathers (raw V quads + header with x + id; slot rs + j RPP for its j-th singleton, at most NS
  // per sample) -- no global re-read -- and after the sample's reduction rewrites them updated in
  // place.  Their stores go out during the next sample, once its first ids are in and before its
  // first row gathers, so no gather is queued behind them; the last sample's at the end.  Every
  // slot is read and written by the lanes of the group that gathered it: no barrier.
  constexpr bool STASH = MODE == kTrainFused;
  static_assert(!STASH || (GS <= 4 && TEAM >= 16), "the fused forward serves kp <= 16");
  constexpr int NS = STASH ? kFuseNS : 1;  // singleton rows a lane group keeps per sample
  constexpr int MZ = STASH ? NS * RPP : 1;
  __shared__ float4 st_v[STASH ? TPB : 1][MZ][STASH ? GS : 1];
  __shared__ float4 st_h[STASH ? TPB : 1][MZ];
  __shared__ uint32_t st_id[STASH ? TPB : 1][MZ];
  const int team = tid / TEAM;
  int nst = 0;          // singletons of the current sample met by this lane group
  int pend = 0;         // updated rows of the previous sample waiting in slots rs + j RPP, j < pend
  const int span = 4 + ((16 - ((kp + 4) & 15)) & 15);  // header + zero pad of its 64-B granule
  // pp = the neighbour group's pend, exchanged while the whole team is active (flush() itself runs
  // from two call sites: a group without an entry in the sample flushes before the entry loop, one
  // with entries inside it, so the two groups of a pair may flush at different points; each then
  // writes its own rows' V and the neighbour's headers from the count taken here, and neither
  // group's slots change before both have flushed -- a group stashes only after its own flush, and
  // only when it has entries)
  auto flush = [&](int pp) {
    if constexpr (GS >= 2) {
      // paired: each updated record leaves in ONE store instruction of 2 GS lanes -- the group
      // writes its row's V, the neighbour group (rs ^ 1) that row's header granule (span <= 4 GS)
      // -- first the even groups' rows, then the odd groups' (a record written by two half-record
      // instructions costs more: DESIGN.md §5, paired row stores)
      const bool even = (rs & 1) == 0;
      const int n = pend > pp ? pend : pp;
      for (int j = 0; j < n; ++j) {
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const bool writer = even == (pass == 0);  // this lane writes V of its own group's row
          const int slot = (writer ? rs : rs ^ 1) + j * RPP;
          const bool live = j < (writer ? pend : pp);
          const uint32_t sid = live ? st_id[team][slot] : 0u;
          float* rec = T.v(sid);
          const float4 val = writer ? st_v[team][slot][g] : (g == 0 ? st_h[team][slot] : make_float4(0.f, 0.f, 0.f, 0.f));
          if (live && (writer ? qok : 4 * g < span)) st_row4(writer ? rec + 4 * g : rec + kp + 4 * g, val);
        }
      }
    } else {
      for (int j = 0; j < pend; ++j) {
        const int i = rs + j * RPP;
        float* rec = T.v(st_id[team][i]);
        if (qok) st_row4(rec + 4 * g, st_v[team][i][g]);
        for (int c = 4 * g; c < span; c += 4 * GS) st_row4(rec + kp + c, c == 0 ? st_h[team][i] : make_float4(0.f, 0.f, 0.f, 0.f));
      }
    }
    pend = 0;
  };

  for (int64_t sl = (int64_t)blockIdx.x * TPB + tid / TEAM; sl < Bl; sl += (int64_t)gridDim.x * TPB) {
    int64_t s = sl;
    if (chunked) {
      int r = 0;
      while (sl >= ch_base[r + 1]) ++r;
      s = ch_start[r] + (sl - ch_base[r]);
    }
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    // the fused update needs the label in every lane after the reduction: its load is issued now,
    // with the sample's first loads, not behind the reduction
    const double ys = MODE == kTrainFused ? label[s] : 0.0;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, vv = 0.0, wx = 0.0;
    uint32_t npres = 0;  // kPredict: learned entries of the sample (this lane's share)
    // the neighbour group's count of rows waiting from the previous sample, taken here, where every
    // lane of the team is active (a shuffle from a lane outside the exec mask reads garbage)
    const int pp_s = STASH && GS >= 2 ? __shfl_xor(pend, GS) : 0;
    if (STASH) {
      nst = 0;
      if (e0 + rs >= e1) flush(pp_s);  // no entry of this sample for the lane group: nothing to wait behind
    }
    for (int64_t eb = e0 + rs; eb < e1; eb += U * RPP) {
      uint32_t id[U];
      float x[U];
      bool ok[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int64_t e = eb + j * RPP;
        ok[j] = e < e1;
        if constexpr (MODE == kTrainFused) {
          // (the fused forward issues these guarded loads together already; under its register
          // budget the unguarded form below came out c3 within the noise, slower: profiles/r05_q)
          id[j] = ok[j] ? col[e] : 0u;
          x[j] = ok[j] ? xs[e] : 0.f;
        } else {
          // loaded from a clamped index, unguarded (eb < e1 here): every id and x of the round in
          // flight at once (a guarded load, or one behind the predict's id test, waits out its round
          // trip first -- the partial pass's were issued in three groups: R = 8 owner forward 0.356
          // -> 0.277 ms, profiles/r05_q)
          const int64_t ec = ok[j] ? e : e1 - 1;
          const uint32_t idl = col[ec];
          // the batch's x stream (4 B per entry); the partial pass's entries carry x themselves
          const float xl = PARTIAL ? __uint_as_float(ent[ec].y) : xs[ec];
          id[j] = ok[j] ? idl : 0u;
          if (MODE == kPredict) ok[j] = ok[j] && id[j] < (uint64_t)T.rows;
          x[j] = ok[j] ? xl : 0.f;
        }
      }
      if (STASH && eb == e0 + rs) flush(pp_s);  // the previous sample's rows: ids in, gathers not yet issued
      RowHdr h[U];
      float4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        // loss-grad with the fill takes ids beyond the table (the left outer join): absent rows
        if (ok[j] && (MODE != kLossGrad || id[j] < (uint64_t)T.rows)) {
          h[j] = *T.hdr(id[j]);
          v[j] = qok ? reinterpret_cast<const float4*>(T.v(id[j]))[g] : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          h[j] = RowHdr{0.f, -1, 0.0};
          v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        // a singleton row (untagged), updated by this sample after its reduction; the group's
        // lanes see the same entry, so nst stays uniform across them
        if (STASH && ok[j] && !is_multi(h[j].t, xo.sp.epoch)) {
          if (nst < NS) {
            const int i = rs + nst * RPP;
            st_v[team][i][g] = v[j];
            if (g == 0) {  // the header with the entry's x in place of t (the update rewrites t)
              RowHdr hx = h[j];
              hx.t = __float_as_int(x[j]);
              st_h[team][i] = *reinterpret_cast<const float4*>(&hx);
              st_id[team][i] = id[j];
            }
          }
          ++nst;
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        float w;
        if ((MODE == kPredict || PARTIAL) && g == 0 && h[j].t >= 0) ++npres;
        current_row(h[j], v[j], w, cumE);
        if (MODE == kLossGrad && xo.fill_sd > 0.0 && ok[j] && h[j].t < 0) fill_row(eb + j * RPP, v[j], w);
        const double xd = x[j];
        // vfxi = v * x (Model.scala:179), VectorSum over the sample (:191)
        a0 += (double)v[j].x * xd; a1 += (double)v[j].y * xd;
        a2 += (double)v[j].z * xd; a3 += (double)v[j].w * xd;
        // vi2xi2 = (sum_f v_f^2) * x * x (Model.scala:256-258), this lane's factors
        const double v2 = (double)v[j].x * v[j].x + (double)v[j].y * v[j].y + (double)v[j].z * v[j].z +
                          (double)v[j].w * v[j].w;
        vv += v2 * xd * xd;
        if (g == 0) wx += (double)w * xd;  // wixi (Model.scala:178)
      }
    }
    // sum the entry slots (lanes with equal g), then the whole team for the scalars
#pragma unroll
    for (int o = GS; o < TEAM; o <<= 1) {
      a0 += __shfl_xor(a0, o); a1 += __shfl_xor(a1, o);
      a2 += __shfl_xor(a2, o); a3 += __shfl_xor(a3, o);
    }
#pragma unroll
    for (int o = 1; o < TEAM; o <<= 1) {
      vv += __shfl_xor(vv, o);
      wx += __shfl_xor(wx, o);
      if (MODE == kPredict || PARTIAL) npres += __shfl_xor(npres, o);
    }
    if (PARTIAL) {  // vectors [pair][kp] in S_out, scalars {sum v^2 x^2, sum w x} in yl_out
      if (rs == 0 && qok)
        *reinterpret_cast<float4*>(S_out + s * sstr + g * 4) = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
      if (tl == 0) {
        yl_out[s * ystr] = make_float2((float)vv, (float)wx);
        if (xo.pcount) xo.pcount[s] = npres;
      }
      continue;
    }
    double ss = qok ? a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3 : 0.0;
#pragma unroll
    for (int o = 1; o < GS; o <<= 1) ss += __shfl_xor(ss, o);
    // sumVx + wixiSum + w0 (Model.scala:221, :260-262)
    const double yhat = 0.5 * (ss - vv) + wx + w0;
    if (MODE == kPredict) {
      if (tl == 0) xo.pred[s] = npres == 0 ? w0 : fmin(fmax(yhat, xo.lo), xo.hi);
      continue;
    }
    if (MODE == kLossGrad) {
      const double d = yhat - label[s];
      const int k = T.k;
      for (int64_t e = e0 + rs; e < e1; e += RPP) {
        const uint32_t id = col[e];
        const double xd = (double)xs[e];
        const bool inr = id < (uint64_t)T.rows;
        const RowHdr h = inr ? *T.hdr(id) : RowHdr{0.f, -1, 0.0};
        float4 v = qok && inr ? reinterpret_cast<const float4*>(T.v(id))[g] : make_float4(0.f, 0.f, 0.f, 0.f);
        float w;
        current_row(h, v, w, cumE);
        if (xo.fill_sd > 0.0 && h.t < 0) fill_row(e, v, w);
        if (g == 0) {
          if (h.t < 0) *xo.absent = 1;
          xo.pred[e] = yhat;    // prediction (Model.scala:221)
          xo.loss[e] = d * d;   // pow(pred - label, 2.0) (:230)
          xo.dw[e] = xd;        // deltaWi (:200)
        }
        double* out = xo.dv + e * k;  // deltaVi (:201-204), columns 4g .. 4g + 3 of k
        const int c = 4 * g;
        if (c + 0 < k) out[c + 0] = a0 * xd - ((double)v.x * xd) * xd;
        if (c + 1 < k) out[c + 1] = a1 * xd - ((double)v.y * xd) * xd;
        if (c + 2 < k) out[c + 2] = a2 * xd - ((double)v.z * xd) * xd;
        if (c + 3 < k) out[c + 3] = a3 * xd - ((double)v.w * xd) * xd;
      }
      continue;
    }
    if (rs == 0 && qok)
      *reinterpret_cast<float4*>(S_out + s * sstr + g * 4) = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
    if (MODE == kTrainFused) {
      // The rows whose only entry in this batch belongs to this sample: their update (SGD.scala:
      // 145-181 over a run of one entry) is applied here, from the values the update kernel would
      // read back -- S, r and yhat rounded to fp32 as stored, x from the batch -- with its
      // arithmetic, so the table is bit for bit the unfused step's.  The row was read a moment ago
      // (an L2 hit); the update kernel skips these runs (no row read, no S gather there).
      const float r32 = (float)(yhat - ys), yh32 = (float)yhat;
      const double rj = (double)r32, yh = (double)yh32;
      const float4 Sq = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
      const StepParams& sp = xo.sp;
      const float lamf = (float)sp.lam;
      if (STASH) {
        // the stashed rows (the group's first NS singletons), updated in place in LDS
        const int zc = nst < NS ? nst : NS;
        for (int jj = 0; jj < zc; ++jj) {
          const int i = rs + jj * RPP;
          const float4 hq = st_h[team][i];
          const RowHdr h = *reinterpret_cast<const RowHdr*>(&hq);
          const double xd = (double)__int_as_float(h.t);  // the stash keeps x in the t word
          const float acf = (float)(sp.cumE - h.cum);  // pending L1 of the row
          const double t = xd * rj, b = (xd * xd) * rj;
          const double gwe = (xd - 1.0) * yh + rj;  // x yhat - y (SGD.scala:145)
          if (qok) {
            const float4 v = shrink4f(st_v[team][i][g], acf);
            const double g0 = fma((double)Sq.x, t, 0.0) - (double)v.x * b, g1 = fma((double)Sq.y, t, 0.0) - (double)v.y * b;
            const double g2 = fma((double)Sq.z, t, 0.0) - (double)v.z * b, g3 = fma((double)Sq.w, t, 0.0) - (double)v.w * b;
            const float4 u = make_float4((float)fma(g0, -sp.scale_v, (double)v.x), (float)fma(g1, -sp.scale_v, (double)v.y),
                                         (float)fma(g2, -sp.scale_v, (double)v.z), (float)fma(g3, -sp.scale_v, (double)v.w));
            st_v[team][i][g] = shrink4f(u, lamf);
          }
          if (g == 0) {
            RowHdr o;
            o.w = upd_w(shrink1f(h.w, acf), 0.0 + gwe, sp);  // SGD.scala:150, :171
            o.t = sp.epoch + 1;
            o.cum = sp.cum_next;
            st_h[team][i] = *reinterpret_cast<const float4*>(&o);
          }
        }
        pend = zc;
      }
      // singletons beyond the group's NS (long samples): the group walks its entries again, and
      // rows past the first NS singletons are read again (nobody else reads or writes a singleton
      // row in this step) and updated straight away
      int seen = 0;
      for (int64_t e = e0 + rs; STASH && nst > NS && e < e1; e += RPP) {
        const uint32_t id = col[e];
        const RowHdr h = *T.hdr(id);
        if (is_multi(h.t, sp.epoch)) continue;
        if (++seen <= NS) continue;  // stashed
        const float4 vq = qok ? reinterpret_cast<const float4*>(T.v(id))[g] : make_float4(0.f, 0.f, 0.f, 0.f);
        const double xd = (double)xs[e];
        const float acf = (float)(sp.cumE - h.cum);  // pending L1 of the row
        float* rec = T.v(id);
        const double t = xd * rj, b = (xd * xd) * rj;
        const double gwe = (xd - 1.0) * yh + rj;  // x yhat - y (SGD.scala:145)
        if (qok) {
          const float4 v = shrink4f(vq, acf);
          const double g0 = fma((double)Sq.x, t, 0.0) - (double)v.x * b, g1 = fma((double)Sq.y, t, 0.0) - (double)v.y * b;
          const double g2 = fma((double)Sq.z, t, 0.0) - (double)v.z * b, g3 = fma((double)Sq.w, t, 0.0) - (double)v.w * b;
          const float4 u = make_float4((float)fma(g0, -sp.scale_v, (double)v.x), (float)fma(g1, -sp.scale_v, (double)v.y),
                                       (float)fma(g2, -sp.scale_v, (double)v.z), (float)fma(g3, -sp.scale_v, (double)v.w));
          st_row4(rec + 4 * g, shrink4f(u, lamf));
        }
        for (int i = 4 * g; i < span; i += 4 * GS) {  // the header and the zero pad of its granule
          float4 hq = make_float4(0.f, 0.f, 0.f, 0.f);
          if (i == 0) {
            RowHdr o;
            o.w = upd_w(shrink1f(h.w, acf), 0.0 + gwe, sp);  // SGD.scala:150, :171
            o.t = sp.epoch + 1;
            o.cum = sp.cum_next;
            hq = *reinterpret_cast<const float4*>(&o);
          }
          st_row4(rec + kp + i, hq);
        }
      }
    }
    if (tl == 0) {
      const double y = label[s];
      // r = pred - label in fp64 (SGD.scala:146), rounded once: relative error 2^-24 of r itself
      yl_out[s * ystr] = make_float2((float)(yhat - y), (float)yhat);
      if (e1 > e0) {
        const double d = yhat - y;
        loss_acc += d * d;  // pow(pred - label, 2.0), Model.scala:230
        nloss += 1.0;
      }
    }
  }
  if (STASH) flush(GS >= 2 ? __shfl_xor(pend, GS) : 0);  // the last sample's rows (the whole wave active)
  if (MODE != kTrain && MODE != kTrainFused) return;
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
  const uint32_t* skeys;  // sorted feature slots
  const uint2* sents;     // their entries {sample, x bits}, same order
  int64_t N;
  const float* S;    // per-sample rows of s_stride floats (vfxiSum first)
  const float2* yl;  // {r = yhat - y, yhat} of sample s at yl[s * yl_stride]
  int64_t s_stride;
  int64_t yl_stride;
  double* part;      // [nranges][2][kp + 2] = [sum g_w | sum S*x*r (kp) | sum x*x*r]
  int64_t nranges;   // ranges of L sorted entries (one update wave each)
  int64_t L;         // entries per range (kWaveEnt)
  StepParams p;
  uint32_t* ucnt;  // [update blocks]
  float* emit;     // replicated mode: per-slot gradient sums [rows][kp + 4] instead of the update
  // non-null: the entry count is n_dev[0] <= N (a prepared batch's multi runs, counted on the
  // device by k_split_*), and n_dev[1] distinct singleton rows were updated by the forward
  const int64_t* n_dev;
};

constexpr uint32_t kFValid = 1u, kFEnd = 2u, kFStart = 4u;


// Lane-group geometry: Q lanes per entry, NF float4 column quads per lane (columns
// 4 (q + Q n) .. + 3), NG = 64 / Q groups per wave, RL = 256 / NG entries per group.
template <int Q, int NF>
struct UpdGeom {
  static constexpr int NG = 64 / Q;
  static constexpr int RL = kWaveEnt / NG;
  static constexpr int KP = 4 * Q * NF;   // widest kp served
  static constexpr int PIECE = KP + 2;    // doubles per piece: [g_w | columns | b]
  static constexpr int IMG_N = RL * NG;   // image slots: RL rows of NG, column g XOR-swizzled by the
                                          // row against bank conflicts (no pad column: at k = 32 the
                                          // pad cost the fourth block per CU)
  static __device__ __forceinline__ int at(int row, int g) { return row * NG + (g ^ (row & (NG - 1))); }
  // image entry: {slot, flags} | sample | x (16 B)
  static constexpr int IMG = IMG_N * 16;
  // the groups' head pieces go to their own region after the image as they close (one slot per
  // group) instead of living in registers until phase 3
  static constexpr int HEADS = NG * PIECE * 8;
  static constexpr int BYTES = IMG + HEADS;
};

// The interaction gradient of one entry (Model.scala:201-204, SGD.scala:146) is
//   g_V[f] = (S[s][f] * x - (v[f] * x) * x) * r,   r = yhat - y,
// so a feature's run sums to   A[f] - v[f] * b,   A[f] = sum_e S[s_e][f] * (x_e r_e),
// b = sum_e x_e^2 r_e: neither sum needs the row, which is read once per run, with its header,
// when the run closes.  g_w = x * yhat - y per entry (SGD.scala:145).
//
// One wave per 256 sorted entries.
//  Phase 1, one lane per entry: run structure (ballots), staged in the wave's LDS image with the
//    entry's sample and x (16 B per entry, step-major so that a step's entries are contiguous).
//  Phase 2, NG lane groups of Q lanes (float4 column quads per lane): group g walks its RL
//    consecutive entries in order, accumulating A, b and g_w in fp64 from the S rows and {r, yhat}
//    of D entries loaded ahead (one record per sample in the single-table step, FM_S_REC; with
//    the V row + header of those that close a run): t = x r, x^2 r and x yhat - y per entry.  A run that
//    begins and closes inside the group's entries is applied in place (update + L1,
//    SGD.scala:150-181, or its gradient emitted in replicated mode).
//  Phase 3: the pieces cut by group boundaries meet in LDS: the group holding a run's start
//    extends its open piece through the following groups' head pieces and applies the run when
//    it closes inside the wave; the wave's first piece (run begun in an earlier wave) and a run
//    still open at the wave's end leave fp64 partials (slot 0 / slot 1), summed in wave order by
//    k_segment_combine.  Every sum runs in a fixed order: the step is bitwise reproducible.
// k <= 64 (NF = 1): waves per SIMD the register allocation must allow (4 blocks/CU); without it the
// compiler took 130 VGPRs at k = 16 (3 waves/SIMD): update -8.6 %, step -1.7 % (A/B 3 x 40 steps)
// (round 3: 5 waves, 96 VGPRs with 32 B/lane spilled at k = 16, measured 0.981-0.984 against
// 0.986-0.990 ms at c3 and 0.192-0.193 against 0.194-0.195 at c5: within the noise, not taken)
constexpr int kUpdMinW = 4;
template <int Q, int NF, int D0>
__global__ __launch_bounds__(kBlock, NF == 1 ? kUpdMinW : 1) void k_segment_update(SegArgs a) {
  using Geo = UpdGeom<Q, NF>;
  constexpr int NG = Geo::NG, RL = Geo::RL, PIECE = Geo::PIECE, NP = kWaveEnt / 64, C = 4 * NF;
  constexpr int D = D0 < RL ? D0 : RL;  // entries loaded ahead (divides RL)
  __shared__ __align__(16) unsigned char smem_all[kBlock / 64][Geo::BYTES];
  __shared__ int pflag_all[kBlock / 64][2 * NG];
  __shared__ uint32_t wcnt[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned char* smem = smem_all[wave];
  constexpr int IN = Geo::IMG_N;
  uint2* img_k = reinterpret_cast<uint2*>(smem);            // {slot, flags}
  int* img_s = reinterpret_cast<int*>(smem + IN * 8);       // sample
  float* img_x = reinterpret_cast<float*>(smem + IN * 12);  // x
  int* pflag = pflag_all[wave];
  const TableView& T = a.T;
  const int kp = T.kp;
  const uint32_t kNone = 0xFFFFFFFFu;
  auto li = [](int e) { return Geo::at(e % RL, e / RL); };
  const int64_t N = a.n_dev ? a.n_dev[0] : a.N;
  // logical blocks of 4 waves x 256 entries (one per block of the grid; blocks beyond a device count exit)
  const int64_t nlblk = (N + (int64_t)kWaveEnt * (kBlock / 64) - 1) / ((int64_t)kWaveEnt * (kBlock / 64));
  for (int64_t lblk = blockIdx.x; lblk < nlblk; lblk += gridDim.x) {
  const int64_t wid = lblk * (kBlock / 64) + wave;
  const int64_t base = wid * kWaveEnt;
  uint32_t ucount = 0;

  if (base < N) {  // wave-uniform
    // ---------------- phase 1: one lane per entry
    uint32_t key[NP];
    uint2 en[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int64_t p = base + i * 64 + lane;
      const bool v = p < N;
      key[i] = v ? a.skeys[p] : kNone;
      en[i] = v ? a.sents[p] : make_uint2(0u, 0u);
    }
    const uint32_t before = base > 0 ? a.skeys[base - 1] : kNone;
    const uint32_t after = base + kWaveEnt < N ? a.skeys[base + kWaveEnt] : kNone;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const uint32_t up = __shfl_up(key[i], 1);
      const uint32_t dn = __shfl_down(key[i], 1);
      const uint32_t pl = i > 0 ? __shfl(key[i > 0 ? i - 1 : 0], 63) : before;
      const uint32_t nf = i + 1 < NP ? __shfl(key[i + 1 < NP ? i + 1 : i], 0) : after;
      const uint32_t prev = lane == 0 ? pl : up;
      const uint32_t next = lane == 63 ? nf : dn;
      const bool valid = key[i] != kNone;
      const bool st = valid && key[i] != prev;
      const bool end = valid && key[i] != next;
      ucount += (uint32_t)__popcll(__ballot(st));
      const int l = li(i * 64 + lane);
      img_k[l] = make_uint2(key[i], (valid ? kFValid : 0u) | (end ? kFEnd : 0u) | (st ? kFStart : 0u));
      img_s[l] = (int)en[i].x;
      img_x[l] = __uint_as_float(en[i].y);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---------------- phase 2: group g, lane q of the group
    const int g = lane / Q, q = lane % Q;
    // D entries loaded ahead (one buffer: the next step's loads are issued after a step is consumed)
    float4 Sp0[D][NF], Vp0[D][NF], Hp0[D];
    float2 Yp0[D];  // the samples' {r, yhat}
    auto prefetch = [&](int b0, float4 (&Sp)[D][NF], float4 (&Vp)[D][NF], float4 (&Hp)[D], float2 (&Yp)[D]) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int l = Geo::at(b0 + u, g);  // li(g * RL + b0 + u)
        const uint2 kf = img_k[l];
        const int s = img_s[l];
        const bool valid = (kf.y & kFValid) != 0, end = (kf.y & kFEnd) != 0;
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          const int c = 4 * (q + Q * n);
          const bool cv = valid && c < kp;
          Sp[u][n] = cv ? *reinterpret_cast<const float4*>(a.S + (int64_t)s * a.s_stride + c)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
          Vp[u][n] = (valid && c < kp && end) ? *reinterpret_cast<const float4*>(T.v(kf.x) + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        Hp[u] = (valid && end) ? *reinterpret_cast<const float4*>(T.hdr(kf.x)) : make_float4(0.f, __int_as_float(-1), 0.f, 0.f);
        Yp[u] = valid ? a.yl[(int64_t)s * a.yl_stride] : make_float2(0.f, 0.f);
      }
    };
    prefetch(0, Sp0, Vp0, Hp0, Yp0);

    // Paired row stores (kp = 4Q, Q = 2 or 4: records of V (16Q B) + a header granule of the same
    // size, i.e. k = 5..8 in 64 B and k = 13..16 in 128 B): the new row of a run closed in phase 2
    // is kept in registers and written at the end of the entry step by 2Q lanes, the group's Q (V)
    // and its neighbour group's Q (header + zero pad), so every row leaves in ONE store
    // instruction covering its whole record instead of two half-record ones.
    constexpr bool kPairCfg = (Q == 2 || Q == 4) && NF == 1;
    const bool paired = kPairCfg && kp == 4 * Q && !a.emit;  // wave-uniform
    float4 pend_v = make_float4(0.f, 0.f, 0.f, 0.f);
    float pend_w = 0.f;             // the row's new w (its header is {w, epoch + 1, cum_next})
    uint32_t pend_slot = kNone;     // kNone: nothing pending

    // apply (or emit) a closed run: the row brought current (absent rows are all zero with
    // cum = 0, so they need no case of their own), then SGD.scala:150-181
    auto close_run = [&](uint32_t slot, const float4 (&vq)[NF], float4 hq, const double (&A)[C], double b, double gw,
                         bool defer) {
      const RowHdr h = *reinterpret_cast<const RowHdr*>(&hq);
      const float acf = (float)(a.p.cumE - h.cum);  // pending L1 of the row
      const float lamf = (float)a.p.lam;
      float* rec = T.v(slot);
      if (kPairCfg && defer) {  // this lane's V quad and (lane q = 0) the header, written by flush_pair
        const float4 v = shrink4f(vq[0], acf);
        const double g0 = A[0] - (double)v.x * b, g1 = A[1] - (double)v.y * b;
        const double g2 = A[2] - (double)v.z * b, g3 = A[3] - (double)v.w * b;
        const float4 u = make_float4((float)fma(g0, -a.p.scale_v, (double)v.x), (float)fma(g1, -a.p.scale_v, (double)v.y),
                                     (float)fma(g2, -a.p.scale_v, (double)v.z), (float)fma(g3, -a.p.scale_v, (double)v.w));
        pend_v = shrink4f(u, lamf);
        pend_w = upd_w(shrink1f(h.w, acf), gw, a.p);  // SGD.scala:150, :171
        pend_slot = slot;
        return;
      }
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int c = 4 * (q + Q * n);
        if (c >= kp) continue;
        const float4 v = shrink4f(vq[n], acf);
        const double g0 = A[4 * n + 0] - (double)v.x * b, g1 = A[4 * n + 1] - (double)v.y * b;
        const double g2 = A[4 * n + 2] - (double)v.z * b, g3 = A[4 * n + 3] - (double)v.w * b;
        if (a.emit) {
          *reinterpret_cast<float4*>(a.emit + (int64_t)slot * (kp + 4) + c) =
              make_float4((float)g0, (float)g1, (float)g2, (float)g3);
        } else {
          // vec' = S_lambda(vec - sum * (eta / m))  (SGD.scala:153, :179)
          const float4 u = make_float4((float)fma(g0, -a.p.scale_v, (double)v.x), (float)fma(g1, -a.p.scale_v, (double)v.y),
                                       (float)fma(g2, -a.p.scale_v, (double)v.z), (float)fma(g3, -a.p.scale_v, (double)v.w));
          st_row4(rec + c, shrink4f(u, lamf));
        }
      }
      if (a.emit) {
        if (q == 0) *reinterpret_cast<float2*>(a.emit + (int64_t)slot * (kp + 4) + kp) = make_float2((float)gw, 1.f);
        return;
      }
      // the header and the zero pad of its 64-B granule: the granule is written whole
      const int span = 4 + ((16 - ((kp + 4) & 15)) & 15);
      for (int i = 4 * q; i < span; i += 4 * Q) {
        float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i == 0) {
          RowHdr o;
          o.w = upd_w(shrink1f(h.w, acf), gw, a.p);  // SGD.scala:150, :171
          o.t = a.p.epoch + 1;
          o.cum = a.p.cum_next;
          hv = *reinterpret_cast<const float4*>(&o);
        }
        st_row4(rec + kp + i, hv);
      }
    };
    // the rows closed in this entry step (all lanes, converged): even groups' rows, then odd
    // groups'; the partner group (lane ^ Q) writes the header granule of the row
    const int pair_span = 4 + ((16 - ((kp + 4) & 15)) & 15);
    auto flush_pair = [&]() {
      // ds_swizzle bit mode within 32 lanes: and 0x1F, or 0, xor Q -> lane ^ Q
      auto swz = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (Q << 10)); };
      const uint32_t p_slot = swz(pend_slot);
      const float p_w = __uint_as_float(swz(__float_as_uint(pend_w)));
      float4 p_h = make_float4(0.f, 0.f, 0.f, 0.f);  // the partner row's header granule: lane q = 0 the header
      if (q == 0) {
        RowHdr o;
        o.w = p_w;
        o.t = a.p.epoch + 1;
        o.cum = a.p.cum_next;
        p_h = *reinterpret_cast<const float4*>(&o);
      }
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const bool writer = (g & 1) == pass;
        const uint32_t slot = writer ? pend_slot : p_slot;
        // the header granule is 4 + pad floats: 4Q of them at kp = 4Q <= 16
        if (slot != kNone && (writer || 4 * q < pair_span)) st_row4(T.v(slot) + (writer ? 4 * q : kp + 4 * q), writer ? pend_v : p_h);
      }
      pend_slot = kNone;
    };

    double* heads = reinterpret_cast<double*>(smem + Geo::IMG);  // [NG][PIECE]
    auto put_head = [&](const double (&A)[C], double b, double gw) {
      double* ph = heads + g * PIECE;
#pragma unroll
      for (int n = 0; n < NF; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) ph[1 + 4 * (q + Q * n) + j] = A[4 * n + j];
      if (q == 0) {
        ph[0] = gw;
        ph[PIECE - 1] = b;
      }
    };
    double acc[C];
#pragma unroll
    for (int j = 0; j < C; ++j) acc[j] = 0.0;
    double accb = 0.0, accw = 0.0;
    int hst = 0;  // the group's head piece: 0 none, 1 open through the group's end, 2 closed
    bool started = false, open = false;
    uint32_t lastkey = kNone;
    auto consume = [&](int b0, const float4 (&Sp)[D][NF], const float4 (&Vp)[D][NF], const float4 (&Hp)[D],
                       const float2 (&Yp)[D]) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int l = Geo::at(b0 + u, g);
        const uint2 kf = img_k[l];
        if (kf.y & kFValid) {
        // t = x r, x^2 r and g_w = deltaWi * pred - label = x yhat - (yhat - r) (SGD.scala:145)
        const double xd = (double)img_x[l], rj = (double)Yp[u].x, yh = (double)Yp[u].y;
        const double t = xd * rj;
        const double2 tb = make_double2(t, (xd * xd) * rj);
        const double gwe = (xd - 1.0) * yh + rj;
        if (kf.y & kFStart) started = true;
        open = true;
        lastkey = kf.x;
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          acc[4 * n + 0] = fma((double)Sp[u][n].x, t, acc[4 * n + 0]);
          acc[4 * n + 1] = fma((double)Sp[u][n].y, t, acc[4 * n + 1]);
          acc[4 * n + 2] = fma((double)Sp[u][n].z, t, acc[4 * n + 2]);
          acc[4 * n + 3] = fma((double)Sp[u][n].w, t, acc[4 * n + 3]);
        }
        accb += tb.y;
        accw += gwe;
        if (kf.y & kFEnd) {
          if (started) {
            close_run(kf.x, Vp[u], Hp[u], acc, accb, accw, paired);
          } else {  // the head piece closes
            put_head(acc, accb, accw);
            hst = 2;
          }
#pragma unroll
          for (int j = 0; j < C; ++j) acc[j] = 0.0;
          accb = 0.0;
          accw = 0.0;
          started = false;
          open = false;
        }
        }
        // converged: every lane of the wave (with one entry per step, after the next step's
        // loads: see the loop below)
        if (kPairCfg && paired && D > 1) flush_pair();
      }
    };
#pragma unroll 1
    for (int b0 = D; b0 <= RL; b0 += D) {  // the first step's loads are in flight already
      consume(b0 - D, Sp0, Vp0, Hp0, Yp0);
      if (b0 < RL) prefetch(b0, Sp0, Vp0, Hp0, Yp0);
      // the closed rows' stores after the next step's loads: issued before them, the loads had to
      // wait for the stores to complete (their destination registers held the stores' data)
      if (kPairCfg && paired && D == 1) flush_pair();
    }
    const bool tail = open && started;  // the open piece began in this group
    if (open && !started) {             // the head piece runs through the group's end
      put_head(acc, accb, accw);
      hst = 1;
    }

    // ---------------- phase 3: pieces cut by group boundaries (the image is dead now)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double* pc = heads;  // head piece of group g at pc + g * PIECE, written in phase 2
    if (q == 0) pflag[2 * g] = hst;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // extend a piece through the head pieces of groups g2 = from, from + 1, ...; true when it closes
    auto extend = [&](double (&A)[C], double& b, double& gw, int from) -> bool {
      for (int g2 = from; g2 < NG; ++g2) {
        const int f2 = pflag[2 * g2];
        if (f2 == 0) return false;  // unreachable: an open piece always continues into a head piece
        const double* ph = pc + g2 * PIECE;
#pragma unroll
        for (int n = 0; n < NF; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) A[4 * n + j] += ph[1 + 4 * (q + Q * n) + j];
        gw += ph[0];
        b += ph[PIECE - 1];
        if (f2 == 2) return true;
      }
      return false;
    };
    const int W = kp + 2;
    auto write_part = [&](int slot, const double (&A)[C], double b, double gw) {
      double* pr = a.part + (wid * 2 + slot) * (int64_t)W;
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int c = 4 * (q + Q * n);
        if (c < kp) {
          pr[1 + c + 0] = A[4 * n + 0];
          pr[1 + c + 1] = A[4 * n + 1];
          pr[1 + c + 2] = A[4 * n + 2];
          pr[1 + c + 3] = A[4 * n + 3];
        }
      }
      if (q == 0) {
        pr[0] = gw;
        pr[kp + 1] = b;
      }
    };
    if (g == 0 && hst) {  // the wave's first piece: its run began in an earlier wave
      double hacc[C], hb = pc[PIECE - 1], hw = pc[0];
#pragma unroll
      for (int n = 0; n < NF; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) hacc[4 * n + j] = pc[1 + 4 * (q + Q * n) + j];
      if (hst == 1) extend(hacc, hb, hw, 1);
      write_part(0, hacc, hb, hw);
    }
    if (tail) {
      if (extend(acc, accb, accw, g + 1)) {
        float4 vq[NF];
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          const int c = 4 * (q + Q * n);
          vq[n] = c < kp ? *reinterpret_cast<const float4*>(T.v(lastkey) + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const float4 hq = *reinterpret_cast<const float4*>(T.hdr(lastkey));
        close_run(lastkey, vq, hq, acc, accb, accw, false);
      } else {
        write_part(1, acc, accb, accw);  // still open at the wave's end
      }
    }
  }
  if (lane == 0) wcnt[wave] = ucount;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += wcnt[w];
    a.ucnt[lblk] = t;
  }
  __syncthreads();  // the image and the counts are reused by the next logical block
  }
}

// Runs that cross range boundaries: the range holding the run's first entry owns it and sums
// the following ranges' head partials in range order (a lane alone when the run ends in the
// next range, one wave per run with lanes over the factor columns otherwise), then applies the
// same update as k_segment_update:  g_V[f] = sum S*x*r [f] - v[f] * sum x*x*r.  Block 0 also
// closes the step with fixed-order reductions.
// The row of `key` brought current, then columns [c_lo, c_hi) step c_step of the run's update
// (sums[j] = sum S*x*r of column c_lo + j * c_step), then its header.
struct RowCur {
  bool present;
  double ac;
  float w;
};
__device__ __forceinline__ RowCur row_current(const SegArgs& a, uint32_t key) {
  const RowHdr h = *a.T.hdr(key);
  RowCur r;
  r.present = h.t >= 0;
  r.ac = r.present ? a.p.cumE - h.cum : 0.0;
  r.w = r.present ? h.w : 0.f;
  if (r.ac > 0.0) r.w = shrink_f(r.w, r.ac);
  return r;
}
// column c of the run's update from the row's stored value vraw (read whatever the row's presence)
__device__ __forceinline__ void close_col(const SegArgs& a, uint32_t key, const RowCur& rc, int c, float vraw, double b,
                                          double sum) {
  float v = rc.present ? vraw : 0.f;
  if (rc.ac > 0.0) v = shrink_f(v, rc.ac);
  const double gv = sum - (double)v * b;
  if (a.emit) a.emit[(int64_t)key * (a.T.kp + 4) + c] = (float)gv;
  else a.T.v(key)[c] = upd_v(v, gv, a.p);
}
__device__ __forceinline__ void close_cols(const SegArgs& a, uint32_t key, const RowCur& rc, int c_lo, int c_hi,
                                           int c_step, double b, const double* sums) {
  const float* vrow = a.T.v(key);
  for (int c = c_lo, j = 0; c < c_hi; c += c_step, ++j) close_col(a, key, rc, c, vrow[c], b, sums[j]);
}
__device__ __forceinline__ void close_hdr(const SegArgs& a, uint32_t key, const RowCur& rc, double gw) {
  const int kp = a.T.kp;
  if (a.emit) {
    *reinterpret_cast<float2*>(a.emit + (int64_t)key * (kp + 4) + kp) = make_float2((float)gw, 1.f);
  } else {
    RowHdr o;
    o.w = upd_w(rc.w, gw, a.p);
    o.t = a.p.epoch + 1;
    o.cum = a.p.cum_next;
    store_hdr(a.T, key, o);
  }
}

constexpr int kStatLd = 8;     // block 0's stats loads in flight per thread
constexpr int kCombCols = 10;  // long-run columns a lane sums at once (even; W = kp + 2: k = 8 in one pass)
__global__ __launch_bounds__(kBlock) void k_segment_combine(SegArgs a, const double2* __restrict__ loss_part,
                                                            int64_t n_loss_blocks, int64_t n_ucnt,
                                                            double* __restrict__ stats_out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kp = a.T.kp;
  const int64_t W = kp + 2;
  const int64_t N = a.n_dev ? a.n_dev[0] : a.N;
  const int64_t nranges = (N + a.L - 1) / a.L;
  __shared__ double run_sum[kBlock / 64][258];  // one long run's summed piece per wave (kp <= 256)
  if (blockIdx.x == 0) {
    __shared__ double rl[kBlock], rc[kBlock], ru[kBlock];
    double l = 0.0, c = 0.0, u = 0.0;
    // each thread's partials in index order as ever, their loads issued kStatLd at a time from
    // clamped addresses (a plain loop waits one memory round trip per element: this block closed
    // the kernel 20-30 us after the others)
    for (int64_t i0 = tid; i0 < n_loss_blocks; i0 += kStatLd * kBlock) {
      double2 v[kStatLd];
#pragma unroll
      for (int j = 0; j < kStatLd; ++j) {
        const int64_t i = i0 + j * kBlock;
        v[j] = loss_part[i < n_loss_blocks ? i : n_loss_blocks - 1];
      }
#pragma unroll
      for (int j = 0; j < kStatLd; ++j) {
        const bool in = i0 + j * kBlock < n_loss_blocks;
        l += in ? v[j].x : 0.0;
        c += in ? v[j].y : 0.0;
      }
    }
    // update blocks that held entries (a device count leaves the grid's tail without any)
    const int64_t per_blk = (int64_t)kWaveEnt * (kBlock / 64);
    const int64_t nu = a.n_dev ? min(n_ucnt, (N + per_blk - 1) / per_blk) : n_ucnt;
    for (int64_t i0 = tid; i0 < nu; i0 += kStatLd * kBlock) {
      uint32_t v[kStatLd];
#pragma unroll
      for (int j = 0; j < kStatLd; ++j) {
        const int64_t i = i0 + j * kBlock;
        v[j] = a.ucnt[i < nu ? i : nu - 1];
      }
#pragma unroll
      for (int j = 0; j < kStatLd; ++j) u += i0 + j * kBlock < nu ? (double)v[j] : 0.0;
    }
    if (a.n_dev && tid == 0) u += (double)a.n_dev[1];  // the singleton rows the forward updated
    rl[tid] = l;
    rc[tid] = c;
    ru[tid] = u;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
      if (tid < o) {
        rl[tid] += rl[tid + o];
        rc[tid] += rc[tid + o];
        ru[tid] += ru[tid + o];
      }
      __syncthreads();
    }
    if (tid == 0) {
      stats_out[0] = rl[0];
      stats_out[1] = rc[0];
      stats_out[2] = ru[0];
    }
  }
  // 16 lanes per range (lane f: factor columns f, f + 16, ...)
  const int64_t chunk = ((int64_t)blockIdx.x * kBlock + tid) / 16;  // range index
  const int f = tid & 15;
  const int64_t L = a.L;
  bool owner = false, two = false;
  uint32_t key = 0;
  if (chunk < nranges) {
    const int64_t p0 = chunk * L;
    const int64_t p1 = p0 + L < N ? p0 + L : N;
    if (p1 < N) {
      // every key the two tests need, loaded together (clamped addresses: no load waits behind
      // another's comparison)
      const int64_t p2 = (chunk + 2) * L;
      const uint32_t kl = a.skeys[p1 - 1], kn = a.skeys[p1], kf = a.skeys[p0];
      const uint32_t kb = a.skeys[p0 > 0 ? p0 - 1 : 0], k2 = a.skeys[p2 < N ? p2 : N - 1];
      key = kl;
      // the range's last run continues into the next range and starts inside this range
      owner = kn == kl && !(kf == kl && p0 > 0 && kb == kl);
      // common case: the run ends inside the next range -> its two partials
      two = owner && !(p2 < N && k2 == kl);
    }
  }
  if (owner && two) {
    const double* pt = a.part + (chunk * 2 + 1) * W;
    const double* ph = a.part + ((chunk + 1) * 2) * W;
    // the two pieces' scalars and first column, the row's header and V column: one round trip
    const int cf = f < kp ? f : kp - 1;
    const double bt = pt[kp + 1], bh = ph[kp + 1], wt = pt[0], wh = ph[0];
    const double st = pt[1 + cf], sh = ph[1 + cf];
    const float vf = a.T.v(key)[cf];
    const RowCur rc = row_current(a, key);
    const double b = bt + bh;
    if (f < kp) close_col(a, key, rc, f, vf, b, st + sh);
    for (int c = f + 16; c < kp; c += 16) {
      const double sm = pt[1 + c] + ph[1 + c];
      close_cols(a, key, rc, c, c + 1, 1, b, &sm);
    }
    if (f == 0) close_hdr(a, key, rc, wt + wh);
  }
  // long runs (hot features): one wave per run, lanes over the factor columns, range order
  uint64_t owners = __ballot(owner && !two && f == 0);
  while (owners) {
    const int l = __ffsll((unsigned long long)owners) - 1;
    owners &= owners - 1;
    const int64_t c0 = __shfl(chunk, l);
    const uint32_t k0 = __shfl(key, l);
    // end of the run: first range after c0 whose first key differs
    int64_t cend = c0 + 1;
    for (;;) {
      const int64_t c = cend + lane;
      const bool cont = c < nranges && a.skeys[c * L] == k0;
      const uint64_t m = __ballot(cont);
      if (m == ~0ull) {
        cend += 64;
        continue;
      }
      cend += __ffsll((unsigned long long)~m) - 1;
      break;
    }
    // the run's pieces = the owner range's tail + the head pieces of ranges c0+1 .. cend-1, each a
    // row of W = kp + 2 doubles [g_w | sum S*x*r (kp) | sum x*x*r].  Lane l sums the pieces of
    // ranges c0+1+l, +64, ... kCombCols columns at a time (a piece's columns are contiguous, loaded
    // unconditionally from clamped addresses: one round trip per 64 ranges), then a fixed xor tree
    // over the 64 lanes, then the tail: a fixed order, so the step stays bitwise reproducible.
    for (int col0 = 0; col0 < (int)W; col0 += kCombCols) {
      double s[kCombCols];
#pragma unroll
      for (int j = 0; j < kCombCols; ++j) s[j] = 0.0;
      for (int64_t c = c0 + 1 + lane; c < cend; c += 64) {
        const double* pr = a.part + (c * 2) * W;
#pragma unroll
        for (int j = 0; j < kCombCols / 2; ++j) {
          const int cc = col0 + 2 * j;
          const double2 v = *reinterpret_cast<const double2*>(pr + (cc < (int)W ? cc : (int)W - 2));
          s[2 * j] += cc < (int)W ? v.x : 0.0;
          s[2 * j + 1] += cc < (int)W ? v.y : 0.0;
        }
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < kCombCols; ++j) s[j] += __shfl_xor(s[j], o);
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < kCombCols; ++j)
          if (col0 + j < (int)W) run_sum[wave][col0 + j] = s[j];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int col = lane; col < (int)W; col += 64) run_sum[wave][col] = a.part[(c0 * 2 + 1) * W + col] + run_sum[wave][col];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double gw = run_sum[wave][0], b = run_sum[wave][kp + 1];
    double sums[4];  // kp <= 256: columns lane, lane + 64, ...
    int j = 0;
    for (int col = lane; col < kp; col += 64, ++j) sums[j] = run_sum[wave][1 + col];
    const RowCur rc = row_current(a, k0);
    close_cols(a, k0, rc, lane, kp, 64, b, sums);
    if (lane == 0) close_hdr(a, k0, rc, gw);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // run_sum is rewritten by the wave's next long run
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ------------------------------------------------------------- replicated apply
// Every rank holds the whole table; the gradient sums of all ranks were all-reduced into
// grad[rows][kp + 4] = [sum g_V | sum g_w | touched | 0].  G lanes per row: the update + L1
// of SGD.scala:150-181 on touched rows (untouched rows take their L1 lazily, as always).
template <int G>
__global__ __launch_bounds__(kBlock) void k_repl_apply(TableView T, const float* __restrict__ grad, StepParams p,
                                                       uint32_t* __restrict__ blk_touched) {
  const int g = threadIdx.x % G;
  const int kp = T.kp, nq = kp >> 2, W = kp + 4;
  uint32_t touched = 0;
  for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / G; i < T.rows;
       i += (int64_t)gridDim.x * kBlock / G) {
    const float* gr = grad + i * W;
    const float2 wt = *reinterpret_cast<const float2*>(gr + kp);
    if (wt.y == 0.f) continue;
    touched += g == 0 ? 1u : 0u;
    const RowHdr h = *T.hdr(i);
    const bool present = h.t >= 0;
    const double ac = present ? p.cumE - h.cum : 0.0;
    float4* rec = reinterpret_cast<float4*>(T.v(i));
    for (int q = g; q < nq; q += G) {
      float4 v = present ? rec[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (ac > 0.0) v = shrink4(v, ac);
      const float4 d = reinterpret_cast<const float4*>(gr)[q];
      rec[q] = make_float4(upd_v(v.x, d.x, p), upd_v(v.y, d.y, p), upd_v(v.z, d.z, p), upd_v(v.w, d.w, p));
    }
    if (g == 0) {
      float w = present ? h.w : 0.f;
      if (ac > 0.0) w = shrink_f(w, ac);
      RowHdr o;
      o.w = upd_w(w, (double)wt.x, p);
      o.t = p.epoch + 1;
      o.cum = p.cum_next;
      store_hdr(T, i, o);
    }
  }
  // the block's count (one word per block: a same-address atomic per wave serialises ~16K waves)
  __shared__ uint32_t wt[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) touched += __shfl_xor(touched, o);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = touched;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += wt[w];
    blk_touched[blockIdx.x] = t;
  }
}

// the blocks' counts summed into one fp64 stats slot (one block, fixed order)
__global__ __launch_bounds__(kBlock) void k_sum_counts(const uint32_t* __restrict__ c, int64_t n, double* __restrict__ out) {
  __shared__ uint64_t ws[kBlock / 64];
  uint64_t t = 0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) t += c[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0;
    for (int w = 0; w < kBlock / 64; ++w) a += ws[w];
    *out = (double)a;
  }
}

// ---------------------------------------------------------------- table utilities
// ids != nullptr: the listed ids (those this shard owns); else every id in [id_begin, id_begin + n)
// that this shard owns, walked slot by slot (i = the i-th owned id of the range)
__global__ void k_init_random(TableView T, const int32_t* __restrict__ ids, int64_t n, int64_t id_begin,
                              uint64_t seed, double sd, int32_t epoch, double cumE) {
  const int64_t R = T.shard_count;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t id;
    if (ids) {
      id = (int64_t)ids[i];
      if (id % R != T.shard_index) continue;
    } else {
      const int64_t first = id_begin + ((T.shard_index - id_begin % R) % R + R) % R;  // first owned id >= id_begin
      id = first + i * R;
    }
    const int64_t slot = id / R;
    if (slot >= T.rows) continue;
    RowHdr o;
    o.w = gauss_draw(seed, id, -1, sd);
    o.t = epoch;
    o.cum = cumE;
    for (int f = 0; f < T.kp; ++f) T.v(slot)[f] = f < T.k ? gauss_draw(seed, id, f, sd) : 0.f;
    store_hdr(T, slot, o);
  }
}

// createInitialModel (SGD.scala:218-252) from the data itself: every id of the batch's entries
// that this context owns and that is absent gets the seeded draw of k_init_random.  The draw is a
// function of (seed, id, factor) only, so no distinct pass is needed: entries of one id that race
// write identical bytes, and rows already present are kept.
__global__ void k_init_entries(TableView T, const uint32_t* __restrict__ col, int64_t n, uint64_t seed, double sd,
                               int32_t epoch, double cumE) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = (int64_t)col[i];
    if (id % T.shard_count != T.shard_index) continue;
    const int64_t slot = id / T.shard_count;
    if (slot >= T.rows || T.hdr(slot)->t >= 0) continue;
    for (int f = 0; f < T.kp; ++f) T.v(slot)[f] = f < T.k ? gauss_draw(seed, id, f, sd) : 0.f;
    RowHdr o;
    o.w = gauss_draw(seed, id, -1, sd);
    o.t = epoch;
    o.cum = cumE;
    store_hdr(T, slot, o);
  }
}

__global__ void k_load_rows(TableView T, const int32_t* __restrict__ ids, int64_t n, const double* __restrict__ w,
                            const double* __restrict__ V, int32_t epoch, double cumE) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids[i];
    if (id % T.shard_count != T.shard_index) continue;
    const int64_t slot = id / T.shard_count;
    if (slot >= T.rows) continue;
    RowHdr o;
    o.w = (float)w[i];
    o.t = epoch;
    o.cum = cumE;
    for (int f = 0; f < T.kp; ++f) T.v(slot)[f] = f < T.k ? (float)V[i * T.k + f] : 0.f;
    store_hdr(T, slot, o);
  }
}

// Rows by feature id (owned by this shard), brought current (pending L1 applied) without writing
// the table: the model Datasets queried by id (Strength / FactorizedInteraction, Model.scala:281,289)
__global__ void k_gather_rows(TableView T, const int32_t* __restrict__ ids, int64_t n, double cumE,
                              double* __restrict__ w_out, double* __restrict__ V_out, int8_t* __restrict__ present) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = (int64_t)ids[i] / T.shard_count;
    const RowHdr h = *T.hdr(slot);
    const bool pr = h.t >= 0;
    const double a = pr ? cumE - h.cum : 0.0;
    present[i] = pr ? 1 : 0;
    w_out[i] = pr ? (double)(a > 0.0 ? shrink_f(h.w, a) : h.w) : 0.0;
    const float* v = T.v(slot);
    for (int f = 0; f < T.k; ++f) V_out[i * T.k + f] = pr ? (double)(a > 0.0 ? shrink_f(v[f], a) : v[f]) : 0.0;
  }
}

__global__ void k_table_reset(TableView T) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x)
    store_hdr(T, i, RowHdr{0.f, -1, 0.0});
}

__global__ void k_flush(TableView T, int32_t epoch, double cumE) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x) {
    RowHdr h = (*T.hdr(i));
    if (h.t < 0) continue;
    const double a = cumE - h.cum;
    if (a > 0.0) {
      h.w = shrink_f(h.w, a);
      for (int f = 0; f < T.kp; ++f) T.v(i)[f] = shrink_f(T.v(i)[f], a);
    }
    h.t = epoch;
    h.cum = cumE;
    store_hdr(T, i, h);
  }
}

__global__ void k_count_present(TableView T, unsigned long long* out) {
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T.rows; i += (int64_t)gridDim.x * blockDim.x)
    c += (*T.hdr(i)).t >= 0 ? 1ull : 0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
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

template <int GS, int TEAM, int U>
void launch_fwd_t(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                  int64_t* nblk, float* partial_out, const FwdOut* xo) {
  constexpr int TPB = kBlock / TEAM;
  int64_t blocks = (b.n_rows + TPB - 1) / TPB;
  if (blocks > kFwdGrid) blocks = kFwdGrid;
  if (blocks < 1) blocks = 1;
  *nblk = blocks;
  const dim3 grid((unsigned)blocks), blk(kBlock);
  const FwdOut none{};
  if (partial_out) {  // [n_rows][kp] fp32 vectors, then [n_rows] float2 scalars (xo: the present counts)
    hipLaunchKernelGGL((k_forward<GS, TEAM, kPartial, U>), grid, blk, 0, st, T, b.row_ptr.as<int64_t>(),
                       b.col.as<uint32_t>(), b.ent.as<uint2>(), nullptr, nullptr, b.n_rows, p.w0, p.cumE, partial_out,
                       reinterpret_cast<float2*>(partial_out + b.n_rows * T.kp), (int64_t)T.kp, (int64_t)1, nullptr,
                       xo ? *xo : none);
    return;
  }
  if (xo && xo->mode == kPredict) {
    hipLaunchKernelGGL((k_forward<GS, TEAM, kPredict, U>), grid, blk, 0, st, T, b.row_ptr.as<int64_t>(),
                       b.col.as<uint32_t>(), b.ent.as<uint2>(), b.xs.as<float>(), nullptr, b.n_rows, p.w0, p.cumE, nullptr, nullptr,
                       (int64_t)T.kp, (int64_t)1, nullptr, *xo);
    return;
  }
  if (xo && xo->mode == kLossGrad) {
    hipLaunchKernelGGL((k_forward<GS, TEAM, kLossGrad, U>), grid, blk, 0, st, T, b.row_ptr.as<int64_t>(),
                       b.col.as<uint32_t>(), b.ent.as<uint2>(), b.xs.as<float>(), b.label.as<double>(), b.n_rows, p.w0, p.cumE, nullptr,
                       nullptr, (int64_t)T.kp, (int64_t)1, nullptr, *xo);
    return;
  }
  w.loss_part.ensure(sizeof(double2) * blocks);
  FwdOut tr = xo ? *xo : none;  // train mode: xo->fused = the singleton rows' updates in the forward
  auto kern = k_forward<GS, TEAM, kTrain, U>;
  if constexpr (GS <= 4 && TEAM >= 16) {
    if (tr.fused) {
      tr.sp = p;
      kern = k_forward<GS, TEAM, kTrainFused, kFuseU>;
    }
  } else {
    FM_REQUIRE(!tr.fused, "the fused forward serves kp <= 16");
  }
  hipLaunchKernelGGL(kern, grid, blk, 0, st, T, b.row_ptr.as<int64_t>(),
                     b.col.as<uint32_t>(), b.ent.as<uint2>(), b.xs.as<float>(), b.label.as<double>(), b.n_rows, p.w0, p.cumE,
                     w.S.as<float>(), s_rec_yl(T.kp) ? reinterpret_cast<float2*>(w.S.as<float>() + T.kp) : w.yl.as<float2>(),
                     (int64_t)s_rec_floats(T.kp), s_rec_yl(T.kp) ? (int64_t)s_rec_floats(T.kp) / 2 : (int64_t)1,
                     w.loss_part.as<double2>(), tr);
}

}  // namespace

// The sharded owner's partial pass sees short segments (about z / R entries per pair): its team
// is sized so one round of U = 4 passes covers a segment, instead of 16 lanes per segment.
template <int GS>
void launch_partial_t(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                      int64_t* nblk, float* partial_out, const FwdOut* xo) {
  const double avg = b.n_rows > 0 ? (double)b.nnz / (double)b.n_rows : 0.0;
  if (GS <= 16 && avg <= 4.0) launch_fwd_t<GS, GS, kPartialU>(T, b, w, p, st, nblk, partial_out, xo);
  else if (GS <= 16 && avg <= 8.0) launch_fwd_t<GS, (2 * GS > 16 ? 16 : 2 * GS), kPartialU>(T, b, w, p, st, nblk, partial_out, xo);
  else launch_fwd_t<GS, (GS > 16 ? GS : 16), kPartialU>(T, b, w, p, st, nblk, partial_out, xo);
}

void launch_forward(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                    int64_t* nblk, float* partial_out, const FwdOut* pred) {
  const int nq = T.kp / 4;
  if (partial_out) {
    if (nq <= 1) launch_partial_t<1>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 2) launch_partial_t<2>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 4) launch_partial_t<4>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 8) launch_partial_t<8>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 16) launch_partial_t<16>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 32) launch_fwd_t<32, 32, kPartialU>(T, b, w, p, st, nblk, partial_out, pred);
    else if (nq <= 64) launch_fwd_t<64, 64, kPartialU>(T, b, w, p, st, nblk, partial_out, pred);
    else FM_REQUIRE(false, "dimFactorization > 256 is not supported");
    FM_HIP_CHECK(hipGetLastError());
    return;
  }
  constexpr int TM = kFwdTeam, TU = kFwdU;
  if (nq <= 1) launch_fwd_t<1, TM, kFwdUNarrow>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 2) launch_fwd_t<2, TM, kFwdUNarrow>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 4) launch_fwd_t<4, (TM < 4 ? 4 : TM), TU>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 8) launch_fwd_t<8, (TM < 8 ? 8 : TM), TU>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 16) launch_fwd_t<16, (TM < 16 ? 16 : TM), TU>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 32) launch_fwd_t<32, 32, kPartialU>(T, b, w, p, st, nblk, partial_out, pred);
  else if (nq <= 64) launch_fwd_t<64, 64, kPartialU>(T, b, w, p, st, nblk, partial_out, pred);
  else FM_REQUIRE(false, "dimFactorization > 256 is not supported");
  FM_HIP_CHECK(hipGetLastError());
}

void launch_segment_update(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_fwd_blocks,
                           double* stats_out, hipStream_t st, float* emit, const int64_t* n_dev) {
  SegSource src{w.S.as<float>(), s_rec_floats(T.kp),
                 s_rec_yl(T.kp) ? reinterpret_cast<const float2*>(w.S.as<float>() + T.kp) : w.yl.as<float2>(),
                 s_rec_yl(T.kp) ? s_rec_floats(T.kp) / 2 : 1};
  src.n_dev = n_dev;
  launch_segment_update(T, b.nnz, src, w, p, skeys, sents, n_fwd_blocks, stats_out, st, emit);
}

void launch_segment_update(const TableView& T, int64_t N, const SegSource& src, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_fwd_blocks, double* stats_out,
                           hipStream_t st, float* emit) {
  const int64_t L = kWaveEnt;
  const int64_t nranges = (N + L - 1) / L;
  w.part.ensure(sizeof(double) * (size_t)(nranges > 0 ? nranges : 1) * 2 * (T.kp + 2));
  const int64_t per_block = (int64_t)kWaveEnt * (kBlock / 64);
  const int64_t ublocks = (N + per_block - 1) / per_block;
  w.ucnt.ensure(sizeof(uint32_t) * (size_t)(ublocks > 0 ? ublocks : 1));
  SegArgs a;
  a.T = T;
  a.skeys = skeys;
  a.sents = sents;
  a.N = N;
  a.S = src.S;
  a.yl = src.yl;
  a.s_stride = src.s_stride;
  a.yl_stride = src.yl_stride;
  a.part = w.part.as<double>();
  a.nranges = nranges;
  a.L = L;
  a.p = p;
  a.ucnt = w.ucnt.as<uint32_t>();
  a.emit = emit;
  a.n_dev = src.n_dev;
  if (ublocks > 0) {
    const dim3 grid((unsigned)ublocks), blk(kBlock);
    const int nq = T.kp / 4;  // column quads
    if (nq <= 1) hipLaunchKernelGGL((k_segment_update<1, 1, kUpdD>), grid, blk, 0, st, a);
    else if (nq <= 2) hipLaunchKernelGGL((k_segment_update<2, 1, kUpdD2>), grid, blk, 0, st, a);
    else if (nq <= 4) hipLaunchKernelGGL((k_segment_update<4, 1, kUpdD4>), grid, blk, 0, st, a);
    else if (nq <= 8) hipLaunchKernelGGL((k_segment_update<8, 1, kUpdD>), grid, blk, 0, st, a);
    else if (nq <= 16) hipLaunchKernelGGL((k_segment_update<16, 1, kUpdD>), grid, blk, 0, st, a);
    else if (nq <= 32) hipLaunchKernelGGL((k_segment_update<16, 2, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((k_segment_update<16, 4, 1>), grid, blk, 0, st, a);
    FM_HIP_CHECK(hipGetLastError());
  }
  int64_t cblocks = (nranges * 16 + kBlock - 1) / kBlock;
  if (cblocks < 1) cblocks = 1;
  hipLaunchKernelGGL(k_segment_combine, dim3((unsigned)cblocks), dim3(kBlock), 0, st, a,
                     w.loss_part.as<double2>(), n_fwd_blocks, ublocks, stats_out);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_init_random(const TableView& T, const int32_t* ids, int64_t n, int64_t id_begin, uint64_t seed,
                        double sd, int32_t epoch, double cumE, hipStream_t st) {
  if (n <= 0) return;
  if (!ids) {  // a range: only the ids this shard owns
    const int64_t R = T.shard_count, end = id_begin + n;
    const int64_t first = id_begin + ((T.shard_index - id_begin % R) % R + R) % R;
    n = first < end ? (end - first + R - 1) / R : 0;
    if (n <= 0) return;
  }
  hipLaunchKernelGGL(k_init_random, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, id_begin, seed, sd,
                     epoch, cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_init_entries(const TableView& T, const uint32_t* col, int64_t n, uint64_t seed, double sd, int32_t epoch,
                         double cumE, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_init_entries, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, col, n, seed, sd, epoch,
                     cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_load_rows(const TableView& T, const int32_t* ids, int64_t n, const double* w, const double* V,
                      int32_t epoch, double cumE, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_load_rows, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, w, V, epoch, cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_gather_rows(const TableView& T, const int32_t* ids, int64_t n, double cumE, double* w, double* V,
                        int8_t* present, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_rows, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, cumE, w, V, present);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_table_reset(const TableView& T, hipStream_t st) {
  if (T.rows <= 0) return;
  FM_HIP_CHECK(hipMemsetAsync(T.rec, 0, sizeof(float) * (size_t)T.rows * T.stride, st));
  hipLaunchKernelGGL(k_table_reset, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_repl_apply(const TableView& T, const float* grad, const StepParams& p, uint32_t* blk_touched,
                       double* n_touched, hipStream_t st) {
  if (T.rows <= 0) {
    FM_HIP_CHECK(hipMemsetAsync(n_touched, 0, sizeof(double), st));
    return;
  }
  const int nq = T.kp / 4;
  const int G = nq <= 1 ? 1 : nq <= 2 ? 2 : nq <= 4 ? 4 : nq <= 8 ? 8 : 16;
  const unsigned grid = grid_for(T.rows * G, kBlock);  // <= kReplApplyBlocks
  switch (G) {
    case 1: hipLaunchKernelGGL(k_repl_apply<1>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, blk_touched); break;
    case 2: hipLaunchKernelGGL(k_repl_apply<2>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, blk_touched); break;
    case 4: hipLaunchKernelGGL(k_repl_apply<4>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, blk_touched); break;
    case 8: hipLaunchKernelGGL(k_repl_apply<8>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, blk_touched); break;
    default: hipLaunchKernelGGL(k_repl_apply<16>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, blk_touched); break;
  }
  hipLaunchKernelGGL(k_sum_counts, dim3(1), dim3(kBlock), 0, st, blk_touched, (int64_t)grid, n_touched);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_flush(const TableView& T, int32_t epoch, double cumE, hipStream_t st) {
  if (T.rows <= 0) return;
  hipLaunchKernelGGL(k_flush, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T, epoch, cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_count_present(const TableView& T, int64_t* out, hipStream_t st) {
  FM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(int64_t), st));
  if (T.rows <= 0) return;
  hipLaunchKernelGGL(k_count_present, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T,
                     reinterpret_cast<unsigned long long*>(out));
  FM_HIP_CHECK(hipGetLastError());
}

void launch_predict(const TableView& T, const BatchDev& b, double cumE, double w0, double lo, double hi,
                    double* pred, hipStream_t st) {
  FM_REQUIRE(T.shard_count == 1, "fm_predict needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  StepParams p{};
  p.cumE = cumE;
  p.w0 = w0;
  FwdOut xo{};
  xo.mode = kPredict;
  xo.lo = lo;
  xo.hi = hi;
  xo.pred = pred;
  StepWork unused;
  int64_t nblk = 0;
  launch_forward(T, b, unused, p, st, &nblk, nullptr, &xo);
}

void launch_loss_grad(const TableView& T, const BatchDev& b, double cumE, double w0, double* pred, double* loss,
                      double* dw, double* dv, int32_t* absent_flag, hipStream_t st, double fill_sd, uint64_t fill_seed) {
  FM_REQUIRE(T.shard_count == 1, "fm_loss_grad needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  StepParams p{};
  p.cumE = cumE;
  p.w0 = w0;
  FwdOut xo{};
  xo.mode = kLossGrad;
  xo.pred = pred;
  xo.loss = loss;
  xo.dw = dw;
  xo.dv = dv;
  xo.absent = absent_flag;
  xo.fill_sd = fill_sd;
  xo.fill_seed = fill_seed;
  StepWork unused;
  int64_t nblk = 0;
  launch_forward(T, b, unused, p, st, &nblk, nullptr, &xo);
}

// One team of 16 lanes per sample: its entries get {sample, x}, x = 1 unless the id's bit 31 says
// the value follows in the row's run of compact values (xoff); col (bit 31 cleared), label and
// row_ptr are copied alongside (grid-stride, the same pass).
__global__ __launch_bounds__(kBlock) void k_explode(const int64_t* __restrict__ rp_in, const double* __restrict__ lab_in,
                                                   const int32_t* __restrict__ xoff, const uint32_t* __restrict__ col_in,
                                                   const float* __restrict__ x_in, int64_t B, int64_t* __restrict__ rp,
                                                   double* __restrict__ lab, uint32_t* __restrict__ col,
                                                   uint2* __restrict__ ent, float* __restrict__ xs) {
  constexpr int T = 16;
  const int tl = threadIdx.x % T;
  const int lane = threadIdx.x & 63;
  const uint64_t team_bits = 0xFFFFull << (lane & ~(T - 1));
  const uint64_t below = team_bits & ((1ull << lane) - 1ull);
  const int64_t gtid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * kBlock;
  for (int64_t i = gtid; i <= B; i += nthreads) rp[i] = rp_in[i];
  for (int64_t i = gtid; i < B; i += nthreads) lab[i] = lab_in[i];
  for (int64_t s = gtid / T; s < B; s += nthreads / T) {
    const int64_t e0 = rp_in[s], e1 = rp_in[s + 1];
    int64_t xo = xoff[s];
    for (int64_t eb = rp_in[s]; eb < e1; eb += T) {  // the team's lanes take the same trips
      const int64_t e = eb + tl;
      const uint32_t c = e < e1 ? col_in[e] : 0u;
      const bool valued = (c >> 31) != 0u;
      const uint64_t m = __ballot(valued);
      const float x = valued ? x_in[xo + __popcll(m & below)] : 1.0f;
      xo += __popcll(m & team_bits);
      if (e < e1) {
        col[e] = c & 0x7FFFFFFFu;
        ent[e] = make_uint2((uint32_t)s, __float_as_uint(x));
        xs[e] = x;
      }
    }
  }
}

// fm_batch_from_rows: output row s is row rows[s] of a resident dataset (the randomSplit split of
// the cached dfData, FactorizationMachinesSGD.scala:93, 111-112).  One team of 16 lanes per output
// row copies the source row's ids and fp32 x (8 B per entry, contiguous) and writes the exploded
// {s, x} entries; row_ptr (computed by the host from the dataset's row_ptr) and the labels are
// written alongside (grid-stride, the same pass).
__global__ __launch_bounds__(kBlock) void k_select_rows(const int64_t* __restrict__ src_rp, const uint32_t* __restrict__ src_col,
                                                       const float* __restrict__ src_xs, const double* __restrict__ src_lab,
                                                       const int64_t* __restrict__ rows, const int64_t* __restrict__ rp_in,
                                                       int64_t B, int64_t* __restrict__ rp, double* __restrict__ lab,
                                                       uint32_t* __restrict__ col, uint2* __restrict__ ent,
                                                       float* __restrict__ xs) {
  constexpr int T = 16;
  const int tl = threadIdx.x % T;
  const int64_t gtid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * kBlock;
  for (int64_t i = gtid; i <= B; i += nthreads) rp[i] = rp_in[i];
  for (int64_t i = gtid; i < B; i += nthreads) lab[i] = src_lab[rows[i]];
  for (int64_t s = gtid / T; s < B; s += nthreads / T) {
    const int64_t e0 = rp_in[s], e1 = rp_in[s + 1];
    const int64_t d = src_rp[rows[s]] - e0;  // source entry of output entry e: e + d
    for (int64_t e = e0 + tl; e < e1; e += T) {
      const uint32_t c = src_col[e + d];
      const float x = src_xs[e + d];
      col[e] = c;
      xs[e] = x;
      ent[e] = make_uint2((uint32_t)s, __float_as_uint(x));
    }
  }
}

// fm_batch_create_splits: a dataset laid out split after split (split_rows [n_splits + 1] row offsets,
// the randomSplit splits of the cached dfData in iteration order, FactorizationMachinesSGD.scala:93,
// 111-112).  Each split's rows get their own row_ptr, rebased to the split's first entry, at
// split_rp[split_rows[s] + s ..= split_rows[s + 1] + s] (zeroed beforehand, so an empty split's one
// slot is 0), and each entry's sample index becomes relative to its split's first row: a split is
// then a mini-batch in place (fm_batch_split_view), with no gather.  One team of 16 lanes per row.
__global__ __launch_bounds__(kBlock) void k_split_rebase(const int64_t* __restrict__ rp, const int64_t* __restrict__ split_rows,
                                                        int32_t n_splits, int64_t B, uint2* __restrict__ ent,
                                                        int64_t* __restrict__ split_rp) {
  constexpr int T = 16;
  const int tl = threadIdx.x % T;
  const int64_t gtid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * kBlock;
  for (int64_t s = gtid / T; s < B; s += nthreads / T) {
    int lo = 0, hi = n_splits;  // the split holding row s: split_rows[lo] <= s < split_rows[lo + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) / 2;
      if (split_rows[mid] <= s) lo = mid;
      else hi = mid;
    }
    const int64_t r0 = split_rows[lo], eb = rp[r0];
    const int64_t e0 = rp[s], e1 = rp[s + 1];
    if (tl == 0) {
      split_rp[s + lo] = e0 - eb;
      if (s + 1 == split_rows[lo + 1]) split_rp[s + 1 + lo] = e1 - eb;
    }
    for (int64_t e = e0 + tl; e < e1; e += T) ent[e].x = (uint32_t)(s - r0);
  }
}

// ------------------------------------------------------- singleton split (fm_batch_prepare)
// The sorted view of a batch -> the entries of its runs of two or more (stable: the order the
// segmented update needs) and the number of singleton runs.  One wave per chunk of 1024 sorted
// entries: count, one-block scan of the chunk counts, then each wave writes its multi entries at
// its offset in order (ballot ranks).  Integer work only: deterministic.  Each pass loads a wave's
// whole chunk at once (16 independent loads, not a round trip per row): in round 4 that made both
// passes twice as fast and the step slower, their bursts landing on the side stream's sort
// (profiles/r04_z, r04_za); once the sort's own latency chains were cut (round 5), the step is
// faster with it ("Latency chains").
constexpr int kSplitChunk = 1024;

// A wave's whole chunk of the sorted keys, loaded at once: row r's key per lane (clamped addresses,
// every load issued before any is used) and the keys just before and after the chunk; then per row
// whether the entry belongs to a run of two or more (multi) and whether it opens its run.
constexpr int kSplitRows = kSplitChunk / 64;
constexpr uint32_t kSplitNone = 0xFFFFFFFFu;
struct SplitChunk {
  uint32_t key[kSplitRows];
  uint32_t multi = 0, first = 0;  // bit r: row r's entry is multi / opens its run
};
__device__ __forceinline__ void split_chunk(const uint32_t* __restrict__ skeys, int64_t N, int64_t c, int lane,
                                            SplitChunk& sc) {
  const int64_t base = c * kSplitChunk;
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) {
    const int64_t p = base + r * 64 + lane;
    sc.key[r] = skeys[p < N ? p : N - 1];
  }
  // the keys just before and after the chunk, in one more load per lane (lane 0: before, the
  // others: after), unconditional so that it is issued with the rows' and not sunk into a branch
  const int64_t eb = lane == 0 ? (base > 0 ? base - 1 : 0) : (base + kSplitChunk < N ? base + kSplitChunk : N - 1);
  const uint32_t edge = skeys[eb];
  const uint32_t before = base > 0 ? __shfl(edge, 0) : kSplitNone;
  const uint32_t after = base + kSplitChunk < N ? __shfl(edge, 1) : kSplitNone;
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) {
    const int64_t p = base + r * 64 + lane;
    const uint32_t up = __shfl_up(sc.key[r], 1), dn = __shfl_down(sc.key[r], 1);
    const uint32_t pl = r > 0 ? __shfl(sc.key[r > 0 ? r - 1 : 0], 63) : before;
    const uint32_t nf = r + 1 < kSplitRows ? __shfl(sc.key[r + 1 < kSplitRows ? r + 1 : r], 0) : after;
    const uint32_t prev = lane == 0 ? pl : up;
    const uint32_t next = p + 1 >= N ? kSplitNone : (lane == 63 ? nf : dn);
    const bool valid = p < N;
    sc.multi |= (uint32_t)(valid && (prev == sc.key[r] || next == sc.key[r])) << r;
    sc.first |= (uint32_t)(valid && prev != sc.key[r]) << r;
  }
}

// (the split at the step's start, main stream) the first entry of every multi run also writes the
// epoch's multi tag into its row's header: the headers' t words are read for all rows of the chunk
// before any tag is written
__global__ __launch_bounds__(kBlock) void k_split_count(const uint32_t* __restrict__ skeys, int64_t N,
                                                        uint2* __restrict__ cnt, int64_t nchunks, TableView T,
                                                        int32_t epoch) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;  // wave-uniform
  SplitChunk sc;
  split_chunk(skeys, N, c, lane, sc);
  const uint32_t tag = sc.multi & sc.first;
  // every lane loads a t word per row, unconditionally (a guarded load waits out its round trip
  // before the next is issued): the run's row where it tags one, else row 0's (one shared line)
  int32_t tv[kSplitRows];
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) tv[r] = T.hdr((tag >> r) & 1u ? sc.key[r] : 0u)->t;
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r)
    if ((tag >> r) & 1u) T.hdr(sc.key[r])->t = multi_tag(epoch, tv[r] >= 0);
  uint32_t nm = 0, ns = 0;
  const int64_t base = c * kSplitChunk;
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) {
    const bool valid = base + r * 64 + lane < N;
    const bool m = (sc.multi >> r) & 1u;
    nm += (uint32_t)__popcll(__ballot(m));
    ns += (uint32_t)__popcll(__ballot(valid && !m));
  }
  if (lane == 0) cnt[c] = make_uint2(nm, ns);
}

// one block: exclusive scan of the chunks' multi counts -> off[c]; totals -> n_out[0] (multi
// entries), n_out[1] (singleton runs).  It sits on the step's critical path (main stream, before
// the forward), so each thread loads its kSplitPer consecutive chunk counts of a round at once
// (from clamped addresses: as guarded loads they compiled to one round trip each):
// one memory round trip per 12K chunks (a 12.6M-entry batch: all of a c3 batch).  1024 threads x 12
// counts since round 5 (c3 0.852-0.856 against 0.856-0.862 ms for 256 x 48, four alternating reps,
// profiles/r05_aj); in round 3, with its loads still chained, 256 threads had been the faster block
// (profiles/r03_v13/ab).  Scanning in the count pass's last block instead (a device-scope counter, a
// release fence per block) cost 1.355 against 0.973 ms: each fence writes back the XCD's L2
// (profiles/r04_v); no scan at all, each scatter block summing the count pass's block totals before
// it, 1.025 against 0.976 ms (profiles/r04_w)
constexpr int kSplitPer = 12;
constexpr int kSplitScanNT = 1024;
__global__ __launch_bounds__(kSplitScanNT) void k_split_scan(const uint2* __restrict__ cnt, int64_t nchunks,
                                                             int64_t* __restrict__ off, int64_t* __restrict__ n_out) {
  constexpr int NW = kSplitScanNT / 64;
  __shared__ int64_t wsum[NW], ssum[NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t carry = 0, singles = 0;
  for (int64_t b = 0; b < nchunks; b += kSplitScanNT * kSplitPer) {
    const int64_t i0 = b + (int64_t)threadIdx.x * kSplitPer;
    uint2 v[kSplitPer];
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j) v[j] = cnt[i0 + j < nchunks ? i0 + j : nchunks - 1];  // clamped: one round trip
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j)
      if (i0 + j >= nchunks) v[j] = make_uint2(0u, 0u);
    int64_t t = 0, sg = 0;
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j) {
      t += v[j].x;
      sg += v[j].y;
    }
    int64_t incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sg += __shfl_xor(sg, o);
    if (lane == 63) wsum[wave] = incl;
    if (lane == 0) ssum[wave] = sg;
    __syncthreads();
    int64_t wpre = 0, tot = 0, stot = 0;
    for (int w = 0; w < NW; ++w) {
      wpre += w < wave ? wsum[w] : 0;
      tot += wsum[w];
      stot += ssum[w];
    }
    int64_t run = carry + wpre + incl - t;
#pragma unroll
    for (int j = 0; j < kSplitPer; ++j) {
      if (i0 + j < nchunks) off[i0 + j] = run;
      run += v[j].x;
    }
    carry += tot;
    singles += stot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    n_out[0] = carry;
    n_out[1] = singles;
  }
}

__global__ __launch_bounds__(kBlock) void k_split_scatter(const uint32_t* __restrict__ skeys,
                                                          const uint2* __restrict__ sents, int64_t N,
                                                          const int64_t* __restrict__ off, int64_t nchunks,
                                                          uint32_t* __restrict__ mkeys, uint2* __restrict__ ments) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;  // wave-uniform
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t base = c * kSplitChunk;
  // the chunk's payloads with its keys, all loads in one round trip (the payload rows are read
  // whole: a row of multi entries touches the same lines)
  uint2 en[kSplitRows];
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) {
    const int64_t p = base + r * 64 + lane;
    en[r] = sents[p < N ? p : N - 1];
  }
  int64_t o = off[c];
  SplitChunk sc;
  split_chunk(skeys, N, c, lane, sc);
#pragma unroll
  for (int r = 0; r < kSplitRows; ++r) {
    const bool m = (sc.multi >> r) & 1u;
    const uint64_t bm = __ballot(m);
    if (m) {
      const int64_t d = o + __popcll(bm & lt);
      mkeys[d] = sc.key[r];
      ments[d] = en[r];
    }
    o += __popcll(bm);
  }
}

void launch_split(const uint32_t* skeys, const uint2* sents, int64_t N, SplitWork& sw, uint32_t* mkeys, uint2* ments,
                  int64_t* n_out, hipStream_t st, const TableView& tag_T, int32_t epoch) {
  const int64_t nchunks = (N + kSplitChunk - 1) / kSplitChunk;
  sw.cnt.ensure_slack(sizeof(uint2) * (size_t)std::max<int64_t>(nchunks, 1));
  sw.off.ensure_slack(sizeof(int64_t) * (size_t)std::max<int64_t>(nchunks, 1));
  if (N <= 0) {
    FM_HIP_CHECK(hipMemsetAsync(n_out, 0, 2 * sizeof(int64_t), st));
    return;
  }
  const unsigned blocks = (unsigned)((nchunks + kBlock / 64 - 1) / (kBlock / 64));
  hipLaunchKernelGGL(k_split_count, dim3(blocks), dim3(kBlock), 0, st, skeys, N, sw.cnt.as<uint2>(), nchunks, tag_T,
                     epoch);
  hipLaunchKernelGGL(k_split_scan, dim3(1), dim3(kSplitScanNT), 0, st, sw.cnt.as<uint2>(), nchunks, sw.off.as<int64_t>(), n_out);
  hipLaunchKernelGGL(k_split_scatter, dim3(blocks), dim3(kBlock), 0, st, skeys, sents, N, sw.off.as<int64_t>(), nchunks,
                     mkeys, ments);
  FM_HIP_CHECK(hipGetLastError());
}


void launch_explode(const int64_t* row_ptr_in, const double* label_in, const int32_t* xoff, const uint32_t* col_in,
                    const float* x_in, int64_t B, int64_t N, int64_t* row_ptr, double* label, uint32_t* col, uint2* ent,
                    float* xs, hipStream_t st) {
  (void)N;
  hipLaunchKernelGGL(k_explode, dim3(grid_for(std::max<int64_t>(B, 1) * 16, kBlock, 256 * 8)), dim3(kBlock), 0, st,
                     row_ptr_in, label_in, xoff, col_in, x_in, B, row_ptr, label, col, ent, xs);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_select_rows(const BatchDev& src, const int64_t* rows, const int64_t* row_ptr_in, int64_t B, BatchDev& dst,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_select_rows, dim3(grid_for(std::max<int64_t>(B, 1) * 16, kBlock, 256 * 8)), dim3(kBlock), 0, st,
                     src.row_ptr.as<int64_t>(), src.col.as<uint32_t>(), src.xs.as<float>(), src.label.as<double>(), rows,
                     row_ptr_in, B, dst.row_ptr.as<int64_t>(), dst.label.as<double>(), dst.col.as<uint32_t>(),
                     dst.ent.as<uint2>(), dst.xs.as<float>());
  FM_HIP_CHECK(hipGetLastError());
}

void launch_split_rebase(const BatchDev& b, const int64_t* split_rows, int32_t n_splits, int64_t* split_rp,
                         hipStream_t st) {
  const int64_t B = b.n_rows;
  FM_HIP_CHECK(hipMemsetAsync(split_rp, 0, sizeof(int64_t) * (B + n_splits), st));
  if (B == 0) return;
  hipLaunchKernelGGL(k_split_rebase, dim3(grid_for(B * 16, kBlock, 256 * 8)), dim3(kBlock), 0, st,
                     b.row_ptr.as<int64_t>(), split_rows, n_splits, B, b.ent.as<uint2>(), split_rp);
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
