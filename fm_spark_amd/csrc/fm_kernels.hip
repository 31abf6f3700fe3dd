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
#include <cstdlib>

#include "fm_device.h"

namespace fmhip {

namespace {

constexpr int kBlock = 256;
#ifndef FM_UPD_PF
#define FM_UPD_PF 4
#endif
#ifndef FM_HDR_PAD
#define FM_HDR_PAD 1
#endif
#ifndef FM_UPD_CH
#define FM_UPD_CH 4
#endif
constexpr int kUpdateChunks = FM_UPD_CH;  // 64-entry chunks per update wave

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

// ------------------------------------------------------------------------ forward
// PARTIAL: the sharded owner's pass (fm_shard.hip).  "Samples" are (source rank, sample)
// pairs of the entries this owner received; the output per pair is the partial row
// [sum v*x (kp) | sum v^2 x^2 | sum w*x | 0 0] (fp32) instead of S / yhat / loss.
template <int GS, int TEAM, bool PARTIAL>
__global__ __launch_bounds__(kBlock) void k_forward(TableView T, const int64_t* __restrict__ row_ptr,
                                                    const uint32_t* __restrict__ col,
                                                    const uint2* __restrict__ ent,
                                                    const float* __restrict__ label, int64_t B,
                                                    double w0, double cumE, float* __restrict__ S_out,
                                                    float2* __restrict__ yl_out, double2* __restrict__ loss_part) {
  constexpr int RPP = TEAM / GS;  // entries per pass
  constexpr int TPB = kBlock / TEAM;
  constexpr int U = 4;            // passes in flight
  const int tid = threadIdx.x;
  const int tl = tid % TEAM;
  const int g = tl % GS;
  const int rs = tl / GS;
  const int kp = T.kp;
  const bool qok = g * 4 < kp;
  double loss_acc = 0.0, nloss = 0.0;

  for (int64_t s = (int64_t)blockIdx.x * TPB + tid / TEAM; s < B; s += (int64_t)gridDim.x * TPB) {
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, vv = 0.0, wx = 0.0;
    for (int64_t eb = e0 + rs; eb < e1; eb += U * RPP) {
      uint32_t id[U];
      float x[U];
      bool ok[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int64_t e = eb + j * RPP;
        ok[j] = e < e1;
        id[j] = ok[j] ? col[e] : 0u;
        x[j] = ok[j] ? __uint_as_float(ent[e].y) : 0.f;
      }
      RowHdr h[U];
      float4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        if (ok[j]) {
          h[j] = *T.hdr(id[j]);
          v[j] = qok ? reinterpret_cast<const float4*>(T.v(id[j]))[g] : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          h[j] = RowHdr{0.f, -1, 0.0};
          v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        float w;
        current_row(h[j], v[j], w, cumE);
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
    }
    if (PARTIAL) {
      const int W = kp + 4;
      if (rs == 0 && qok)
        *reinterpret_cast<float4*>(S_out + s * W + g * 4) = make_float4((float)a0, (float)a1, (float)a2, (float)a3);
      if (tl == 0) *reinterpret_cast<float4*>(S_out + s * W + kp) = make_float4((float)vv, (float)wx, 0.f, 0.f);
      continue;
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
  if (PARTIAL) return;
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
  const float* S;   // per-sample rows of s_stride_q quads (vfxiSum first)
  const float2* yl; // {yhat, y} of sample s at yl[s * yl_stride]
  int s_stride_q;
  int yl_stride;
  double* part;     // [nranges][2][kp + 1]
  int64_t nranges;  // ranges of L sorted entries, one wave each
  int64_t L;        // entries per range (64 * CH)
  StepParams p;
  uint32_t* ucnt;  // [update blocks]
  float* emit;     // replicated mode: per-slot gradient sums [rows][kp + 4] instead of the update
};

// Per-entry scalars of the current chunk, staged in LDS for the G-lanes-per-entry phase.
struct EntInfo {
  uint32_t key;
  int32_t s;
  float x;
  int32_t flags;  // valid | writes<<1 | complete<<2 | present<<3 | slot<<4 | start_lane<<8
  double r;       // yhat - y
  double ac;      // pending L1 of the row
};

// One wave per range of CH consecutive chunks of 64 sorted entries (L = 64 * CH entries).
//  Phase 1, one lane per entry: run structure (pieces of equal keys inside the chunk), the
//    row header and the sample's (yhat, y); the linear gradient is scanned here.
//  Phase 2, G lanes per entry (one float4 quad each), E = 64/G entries per round: S and V rows
//    move as whole rows (16 rows per wave-instruction for k = 16); the loads of up to four
//    rounds are in flight together, then the segmented scan (lane stride G, carries between
//    rounds) and the write-back.
//  Runs continue across the chunks of a range through register carries, so only runs crossing
//    a range boundary leave fp64 partials (slot 0: the range's first piece when its run began
//    before the range; slot 1: the last piece when its run continues past the range).  The
//    next chunk's entries are loaded while the current chunk is processed.
//  CH > 1 needs nq <= G (one quad-chunk), which the launcher guarantees.
template <int G, int CH>
__global__ __launch_bounds__(kBlock) void k_segment_update(SegArgs a) {
  constexpr int E = 64 / G;           // entries per round
  constexpr int PF = G < FM_UPD_PF ? G : FM_UPD_PF;  // rounds whose loads are issued together
  __shared__ EntInfo info[kBlock / 64][64];
  __shared__ float wnew_s[kBlock / 64][64];
  __shared__ uint32_t wcnt[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const TableView& T = a.T;
  const int kp = T.kp, nq = kp >> 2;
#if FM_HDR_PAD
  const int hq_end = (nq + 4) & ~3;  // end of the 64-B granule holding the header (in quads)
#else
  const int hq_end = nq + 1;
#endif
  const int64_t rg = (int64_t)blockIdx.x * (kBlock / 64) + wave;
  const int64_t r0 = rg * a.L;
  const uint32_t kNone = 0xFFFFFFFFu;
  const float4* __restrict__ S4 = reinterpret_cast<const float4*>(a.S);
  EntInfo* inf = info[wave];
  const int q_in = lane % G;  // this lane's quad inside a quad-chunk
  const int j_in = lane / G;  // this lane's entry inside a round

  uint32_t ucount = 0;
  double cw = 0.0;                                          // open piece's running w sum
  double cv0 = 0.0, cv1 = 0.0, cv2 = 0.0, cv3 = 0.0;        // ... and V sums (this lane's quad)
  bool open_started = false;  // the piece open at the previous chunk's end began in this range
  uint32_t prev_last = (r0 > 0 && r0 < a.N) ? a.skeys[r0 - 1] : kNone;
  int64_t pp = r0 + lane;
  bool valid = r0 < a.N && pp < a.N;
  uint32_t key = valid ? a.skeys[pp] : kNone;
  uint2 en = valid ? a.sents[pp] : make_uint2(0u, 0u);

  for (int c = 0; c < CH; ++c) {
    const int64_t p0 = r0 + (int64_t)c * 64;
    if (p0 >= a.N) break;  // wave-uniform
    // prefetch the next chunk of the range
    const int64_t pn = p0 + 64 + lane;
    const bool nvalid = (c + 1 < CH) && pn < a.N;
    const uint32_t nkey = nvalid ? a.skeys[pn] : kNone;
    const uint2 nen = nvalid ? a.sents[pn] : make_uint2(0u, 0u);

    uint32_t prev_key = __shfl_up(key, 1);
    uint32_t next_key = __shfl_down(key, 1);
    if (lane == 0) prev_key = prev_last;
    if (lane == 63) next_key = (p0 + 64 < a.N) ? a.skeys[p0 + 64] : kNone;
    if (pp == a.N - 1) next_key = kNone;
    const int s = (int)en.x;
    const float xf = __uint_as_float(en.y);
    const double x = (double)xf;
    const RowHdr h = valid ? (*T.hdr(key)) : RowHdr{0.f, -1, 0.0};  // read before any write-back
    const float2 yl = valid ? a.yl[(int64_t)s * a.yl_stride] : make_float2(0.f, 0.f);

    const bool last_chunk = (c == CH - 1) || (p0 + 64 >= a.N);
    const bool seg_start = valid && key != prev_key;  // a run of this key starts here
    const bool seg_end = valid && key != next_key;     // ... ends here
    const bool piece_head = valid && (lane == 0 || seg_start);
    const bool writes = valid && (seg_end || (lane == 63 && last_chunk));
    const uint64_t heads = __ballot(piece_head);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t hm = heads & upto;
    const int start_lane = hm ? 63 - __clzll(hm) : 0;
    const uint64_t starts = __ballot(seg_start);
    ucount += (uint32_t)__popcll(starts);
    // the lane-0 piece continues a piece of the previous chunk of this range
    const bool cont = c > 0 && !(starts & 1ull);
    const int dist = valid ? lane - start_lane : 0;
    int nsteps = 0;
    while (nsteps < 6 && __ballot(dist >= (1 << nsteps))) ++nsteps;
    const bool head_is_start = ((starts >> start_lane) & 1ull) || (start_lane == 0 && cont && open_started);
    const bool complete = head_is_start && seg_end;
    const int slot = head_is_start ? 1 : 0;
    const bool present = h.t >= 0;
    const double ac = present ? a.p.cumE - h.cum : 0.0;  // pending L1 of this row
    const double yhat = yl.x, y = yl.y;

    // ---- linear term: g_w = deltaWi * pred - label (SGD.scala:145)
    double gw = valid ? x * yhat - y : 0.0;
    gw = seg_scan(gw, lane, start_lane, nsteps);
    if (cont && start_lane == 0) gw += cw;
    cw = __shfl(gw, 63);
    if (writes) {
      if (complete && a.emit) {  // [.. | sum g_w | touched]
        *reinterpret_cast<float2*>(a.emit + (int64_t)key * (kp + 4) + kp) = make_float2((float)gw, 1.f);
      } else if (complete) {  // the header is stored with the V row in phase 2
        float w = present ? h.w : 0.f;
        if (ac > 0.0) w = shrink_f(w, ac);
        wnew_s[wave][lane] = upd_w(w, gw, a.p);  // SGD.scala:150, :171, :179
      } else {
        a.part[(rg * 2 + slot) * (int64_t)(kp + 1)] = gw;
      }
    }
    open_started = __shfl((int)head_is_start, 63) != 0;
    prev_last = __shfl(key, 63);

    // ---- interaction term: g_V = (vfxiSum*x - (v*x)*x) * (pred - label) (Model.scala:201-204,
    //      SGD.scala:146)
    EntInfo me;
    me.key = key;
    me.s = s;
    me.x = xf;
    me.flags = (valid ? 1 : 0) | (writes ? 2 : 0) | (complete ? 4 : 0) | (present ? 8 : 0) | (slot << 4) |
               (start_lane << 8);
    me.r = yhat - y;
    me.ac = ac;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    inf[lane] = me;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int qc = 0; qc < nq; qc += G) {
      const int q = qc + q_in;
      const bool qok = q < nq;
#pragma unroll 1
      for (int rb = 0; rb < G; rb += PF) {
        EntInfo ei[PF];
        float4 sq[PF], v[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) ei[u] = inf[(rb + u) * E + j_in];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          const bool vj = (ei[u].flags & 1) && qok;
          sq[u] = vj ? S4[(int64_t)ei[u].s * a.s_stride_q + q] : make_float4(0.f, 0.f, 0.f, 0.f);
          v[u] = (vj && (ei[u].flags & 8)) ? reinterpret_cast<const float4*>(T.v(ei[u].key))[q]
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          const int rd = rb + u;
          const int j = rd * E + j_in;  // entry (lane of phase 1) this lane serves
          const int fl = ei[u].flags;
          const bool vj = (fl & 1) && qok;
          const int sl = fl >> 8;
          if (ei[u].ac > 0.0) v[u] = shrink4(v[u], ei[u].ac);
          const double xd = ei[u].x, rj = ei[u].r;
          double c0 = vj ? ((double)sq[u].x * xd - ((double)v[u].x * xd) * xd) * rj : 0.0;
          double c1 = vj ? ((double)sq[u].y * xd - ((double)v[u].y * xd) * xd) * rj : 0.0;
          double c2 = vj ? ((double)sq[u].z * xd - ((double)v[u].z * xd) * xd) * rj : 0.0;
          double c3 = vj ? ((double)sq[u].w * xd - ((double)v[u].w * xd) * xd) * rj : 0.0;
          // segmented scan over this round's entries (lane stride G), fixed tree order
          const int lo = sl > rd * E ? sl : rd * E;  // first entry of the piece inside this round
#pragma unroll
          for (int o = 1; o < E; o <<= 1) {
            if (o < (1 << nsteps)) {  // wave-uniform: skip steps no piece is long enough for
              const double t0 = __shfl_up(c0, o * G), t1 = __shfl_up(c1, o * G);
              const double t2 = __shfl_up(c2, o * G), t3 = __shfl_up(c3, o * G);
              if (j - o >= lo) {
                c0 += t0; c1 += t1; c2 += t2; c3 += t3;
              }
            }
          }
          // the piece started in an earlier round, or continues from the previous chunk
          if (sl < rd * E || (rd == 0 && sl == 0 && cont)) {
            c0 += cv0; c1 += cv1; c2 += cv2; c3 += cv3;
          }
          const int last = (E - 1) * G + q_in;  // the round's last entry, same quad
          cv0 = __shfl(c0, last); cv1 = __shfl(c1, last);
          cv2 = __shfl(c2, last); cv3 = __shfl(c3, last);
          if ((fl & 1) && (fl & 2)) {
            if ((fl & 4) && a.emit) {
              if (qok)
                reinterpret_cast<float4*>(a.emit + (int64_t)ei[u].key * (kp + 4))[q] =
                    make_float4((float)c0, (float)c1, (float)c2, (float)c3);
            } else if (fl & 4) {
              float4* rec = reinterpret_cast<float4*>(T.v(ei[u].key));
              if (qok)
                rec[q] = make_float4(upd_v(v[u].x, c0, a.p), upd_v(v[u].y, c1, a.p), upd_v(v[u].z, c2, a.p),
                                     upd_v(v[u].w, c3, a.p));
              if (qc + G >= nq) {
                // last quad-chunk: the header and the zero pad of its 64-B granule, stored by the
                // same lanes so every granule of the record is written whole (see store_hdr)
                for (int hq = nq + q_in; hq < hq_end; hq += G) {
                  float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
                  if (hq == nq) {
                    RowHdr o;
                    o.w = wnew_s[wave][j];
                    o.t = a.p.epoch + 1;
                    o.cum = a.p.cum_next;
                    hv = *reinterpret_cast<const float4*>(&o);
                  }
                  rec[hq] = hv;
                }
              }
            } else if (qok) {
              double* prow = a.part + (((rg * 2 + ((fl >> 4) & 1)) * (int64_t)(kp + 1)) + 1 + 4 * q);
              prow[0] = c0;
              prow[1] = c1;
              prow[2] = c2;
              prow[3] = c3;
            }
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    key = nkey;
    en = nen;
    pp += 64;
    valid = nvalid;
  }
  if (lane == 0) wcnt[wave] = ucount;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += wcnt[w];
    a.ucnt[blockIdx.x] = t;
  }
}

// Runs that cross range boundaries: the range holding the run's first entry owns it; one wave
// per owner sums the following ranges' head partials in range order with lanes over the k+1
// columns (a lane alone when the run ends in the next range).  Block 0 also closes the step with fixed-order reductions.
__global__ __launch_bounds__(kBlock) void k_segment_combine(SegArgs a, const double2* __restrict__ loss_part,
                                                            int64_t n_loss_blocks, int64_t n_ucnt,
                                                            double* __restrict__ stats_out) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int kp = a.T.kp;
  const int64_t W = kp + 1;
  if (blockIdx.x == 0) {
    __shared__ double rl[kBlock], rc[kBlock], ru[kBlock];
    double l = 0.0, c = 0.0, u = 0.0;
    for (int64_t i = tid; i < n_loss_blocks; i += kBlock) {
      l += loss_part[i].x;
      c += loss_part[i].y;
    }
    for (int64_t i = tid; i < n_ucnt; i += kBlock) u += (double)a.ucnt[i];
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
  const int64_t chunk = (int64_t)blockIdx.x * kBlock + tid;  // range index
  const int64_t L = a.L;
  bool owner = false;
  uint32_t key = 0;
  if (chunk < a.nranges) {
    const int64_t p0 = chunk * L;
    const int64_t p1 = p0 + L < a.N ? p0 + L : a.N;
    if (p1 < a.N) {
      key = a.skeys[p1 - 1];
      // the chunk's last run continues into the next chunk and starts inside this chunk
      owner = a.skeys[p1] == key && !(a.skeys[p0] == key && p0 > 0 && a.skeys[p0 - 1] == key);
    }
  }
  const TableView& T = a.T;
  // common case: the run ends inside the next chunk -> this lane combines the two partials
  bool two = false;
  if (owner) {
    const int64_t c2 = chunk + 2;
    two = !(c2 < a.nranges && a.skeys[c2 * L] == key);
  }
  if (owner && two && a.emit) {
    const double* pt = a.part + (chunk * 2 + 1) * W;
    const double* ph = a.part + ((chunk + 1) * 2) * W;
    float* gr = a.emit + (int64_t)key * (kp + 4);
    for (int f = 0; f < kp; ++f) gr[f] = (float)(pt[1 + f] + ph[1 + f]);
    *reinterpret_cast<float2*>(gr + kp) = make_float2((float)(pt[0] + ph[0]), 1.f);
  } else if (owner && two) {
    const double* pt = a.part + (chunk * 2 + 1) * W;
    const double* ph = a.part + ((chunk + 1) * 2) * W;
    const RowHdr h = *T.hdr(key);
    const bool present = h.t >= 0;
    const double ac = present ? a.p.cumE - h.cum : 0.0;
    float w = present ? h.w : 0.f;
    if (ac > 0.0) w = shrink_f(w, ac);
    float* vrow = T.v(key);
    for (int q = 0; q < (kp >> 2); ++q) {
      float4 v = present ? reinterpret_cast<const float4*>(vrow)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (ac > 0.0) v = shrink4(v, ac);
      const double g0 = pt[1 + 4 * q + 0] + ph[1 + 4 * q + 0];
      const double g1 = pt[1 + 4 * q + 1] + ph[1 + 4 * q + 1];
      const double g2 = pt[1 + 4 * q + 2] + ph[1 + 4 * q + 2];
      const double g3 = pt[1 + 4 * q + 3] + ph[1 + 4 * q + 3];
      reinterpret_cast<float4*>(vrow)[q] =
          make_float4(upd_v(v.x, g0, a.p), upd_v(v.y, g1, a.p), upd_v(v.z, g2, a.p), upd_v(v.w, g3, a.p));
    }
    RowHdr o;
    o.w = upd_w(w, pt[0] + ph[0], a.p);
    o.t = a.p.epoch + 1;
    o.cum = a.p.cum_next;
    store_hdr(T, key, o);
  }
  // long runs (hot features): one wave per run, lanes over the k+1 columns, chunk order
  uint64_t owners = __ballot(owner && !two);
  while (owners) {
    const int l = __ffsll((unsigned long long)owners) - 1;
    owners &= owners - 1;
    const int64_t c0 = __shfl(chunk, l);
    const uint32_t k0 = __shfl(key, l);
    // end of the run: first chunk after c0 whose first key differs
    int64_t cend = c0 + 1;
    for (;;) {
      const int64_t c = cend + lane;
      const bool cont = c < a.nranges && a.skeys[c * L] == k0;
      const uint64_t m = __ballot(cont);
      if (m == ~0ull) {
        cend += 64;
        continue;
      }
      cend += __ffsll((unsigned long long)~m) - 1;
      break;
    }
    const RowHdr h = *T.hdr(k0);
    const bool present = h.t >= 0;
    const double ac = present ? a.p.cumE - h.cum : 0.0;
    float wnew = 0.f;
    for (int f0 = 0; f0 < W; f0 += 64) {
      const int f = f0 + lane;
      if (f < W) {
        double g = a.part[(c0 * 2 + 1) * W + f];
        int64_t c = c0 + 1;
        for (; c + 4 <= cend; c += 4) {
          const double g0 = a.part[((c + 0) * 2) * W + f];
          const double g1 = a.part[((c + 1) * 2) * W + f];
          const double g2 = a.part[((c + 2) * 2) * W + f];
          const double g3 = a.part[((c + 3) * 2) * W + f];
          g += g0;
          g += g1;
          g += g2;
          g += g3;
        }
        for (; c < cend; ++c) g += a.part[(c * 2) * W + f];
        if (a.emit) {
          float* gr = a.emit + (int64_t)k0 * (kp + 4);
          if (f == 0) *reinterpret_cast<float2*>(gr + kp) = make_float2((float)g, 1.f);
          else gr[f - 1] = (float)g;
        } else if (f == 0) {
          float w = present ? h.w : 0.f;
          if (ac > 0.0) w = shrink_f(w, ac);
          wnew = upd_w(w, g, a.p);
        } else {
          float v = present ? T.v(k0)[f - 1] : 0.f;
          if (ac > 0.0) v = shrink_f(v, ac);
          T.v(k0)[f - 1] = upd_v(v, g, a.p);
        }
      }
    }
    if (lane == 0 && !a.emit) {
      RowHdr o;
      o.w = wnew;
      o.t = a.p.epoch + 1;
      o.cum = a.p.cum_next;
      store_hdr(T, k0, o);
    }
  }
}

// ------------------------------------------------------------- replicated apply
// Every rank holds the whole table; the gradient sums of all ranks were all-reduced into
// grad[rows][kp + 4] = [sum g_V | sum g_w | touched | 0].  G lanes per row: the update + L1
// of SGD.scala:150-181 on touched rows (untouched rows take their L1 lazily, as always).
template <int G>
__global__ __launch_bounds__(kBlock) void k_repl_apply(TableView T, const float* __restrict__ grad, StepParams p,
                                                       unsigned long long* __restrict__ n_touched) {
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
  // integer count: deterministic
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) touched += __shfl_xor(touched, o);
  if ((threadIdx.x & 63) == 0 && touched) atomicAdd(n_touched, (unsigned long long)touched);
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
                              uint64_t seed, double sd, int32_t epoch, double cumE) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids ? (int64_t)ids[i] : id_begin + i;
    if (id % T.shard_count != T.shard_index) continue;
    const int64_t slot = id / T.shard_count;
    if (slot >= T.rows) continue;
    RowHdr o;
    o.w = gauss_draw(seed, id, -1, sd);
    o.t = epoch;
    o.cum = cumE;
    for (int f = 0; f < T.kp; ++f) T.v(slot)[f] = f < T.k ? gauss_draw(seed, id, f, sd) : 0.f;
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

// FactorizationMachinesModel.predict/transform (Model.scala:69-133), one thread per sample.
// Global ids arrive in b.col; ids >= num_features or absent from the model are dropped.
__global__ void k_predict(TableView T, const int64_t* __restrict__ row_ptr, const uint32_t* __restrict__ col,
                          const uint2* __restrict__ ent, int64_t B, int64_t num_features, double cumE,
                          double w0, double lo, double hi, double* __restrict__ pred) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B; s += (int64_t)gridDim.x * blockDim.x) {
    double acc[64];
    for (int f = 0; f < 64; ++f) acc[f] = 0.0;
    double wx = 0.0, vv = 0.0;
    int n = 0;
    for (int64_t e = row_ptr[s]; e < row_ptr[s + 1]; ++e) {
      const int64_t id = col[e];
      if (id >= num_features) continue;
      const RowHdr h = (*T.hdr(id));
      if (h.t < 0) continue;
      const double a = cumE - h.cum;
      const double x = (double)__uint_as_float(ent[e].y);
      const float w = a > 0.0 ? shrink_f(h.w, a) : h.w;
      wx += (double)w * x;
      double v2 = 0.0;
      for (int f = 0; f < T.k; ++f) {
        float v = T.v(id)[f];
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
                            const uint2* __restrict__ ent, const float* __restrict__ label, int64_t B,
                            double cumE, double w0, double* pred, double* loss, double* dw, double* dv,
                            int32_t* absent) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B; s += (int64_t)gridDim.x * blockDim.x) {
    double acc[64];
    for (int f = 0; f < 64; ++f) acc[f] = 0.0;
    double wx = 0.0, vv = 0.0;
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t id = col[e];
      const RowHdr h = (*T.hdr(id));
      if (h.t < 0) {
        *absent = 1;
        continue;
      }
      const double a = cumE - h.cum;
      const double x = (double)__uint_as_float(ent[e].y);
      const float w = a > 0.0 ? shrink_f(h.w, a) : h.w;
      wx += (double)w * x;
      double v2 = 0.0;
      for (int f = 0; f < T.k; ++f) {
        float v = T.v(id)[f];
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
      const RowHdr h = (*T.hdr(id));
      const double x = (double)__uint_as_float(ent[e].y);
      if (pred) pred[e] = yhat;
      if (loss) loss[e] = d * d;
      if (dw) dw[e] = x;
      if (dv) {
        const double a = h.t >= 0 ? cumE - h.cum : 0.0;
        for (int f = 0; f < T.k; ++f) {
          float v = h.t >= 0 ? T.v(id)[f] : 0.f;
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
                  int64_t* nblk, float* partial_out) {
  constexpr int TPB = kBlock / TEAM;
  int64_t blocks = (b.n_rows + TPB - 1) / TPB;
  if (blocks > 256 * 8) blocks = 256 * 8;
  if (blocks < 1) blocks = 1;
  *nblk = blocks;
  w.loss_part.ensure(sizeof(double2) * blocks);
  if (partial_out)
    hipLaunchKernelGGL((k_forward<GS, TEAM, true>), dim3((unsigned)blocks), dim3(kBlock), 0, st, T,
                       b.row_ptr.as<int64_t>(), b.col.as<uint32_t>(), b.ent.as<uint2>(), nullptr, b.n_rows, p.w0,
                       p.cumE, partial_out, nullptr, nullptr);
  else
    hipLaunchKernelGGL((k_forward<GS, TEAM, false>), dim3((unsigned)blocks), dim3(kBlock), 0, st, T,
                       b.row_ptr.as<int64_t>(), b.col.as<uint32_t>(), b.ent.as<uint2>(), b.label.as<float>(),
                       b.n_rows, p.w0, p.cumE, w.S.as<float>(), w.yl.as<float2>(), w.loss_part.as<double2>());
}

}  // namespace

void launch_forward(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p, hipStream_t st,
                    int64_t* n_fwd_blocks, float* partial_out) {
  const int nq = T.kp / 4;
  if (nq <= 1) launch_fwd_t<1, 16>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 2) launch_fwd_t<2, 16>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 4) launch_fwd_t<4, 16>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 8) launch_fwd_t<8, 16>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 16) launch_fwd_t<16, 16>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 32) launch_fwd_t<32, 32>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else if (nq <= 64) launch_fwd_t<64, 64>(T, b, w, p, st, n_fwd_blocks, partial_out);
  else FM_REQUIRE(false, "dimFactorization > 256 is not supported");
  FM_HIP_CHECK(hipGetLastError());
}

void launch_segment_update(const TableView& T, const BatchDev& b, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_fwd_blocks,
                           double* stats_out, hipStream_t st, float* emit) {
  SegSource src{w.S.as<float>(), T.kp / 4, w.yl.as<float2>(), 1};
  launch_segment_update(T, b.nnz, src, w, p, skeys, sents, n_fwd_blocks, stats_out, st, emit);
}

void launch_segment_update(const TableView& T, int64_t N, const SegSource& src, StepWork& w, const StepParams& p,
                           const uint32_t* skeys, const uint2* sents, int64_t n_fwd_blocks, double* stats_out,
                           hipStream_t st, float* emit) {
  const int nq = T.kp / 4;
  const int G = nq <= 1 ? 1 : nq <= 2 ? 2 : nq <= 4 ? 4 : nq <= 8 ? 8 : 16;
  const int CH = nq <= G ? kUpdateChunks : 1;  // carries across chunks need one quad-chunk
  const int64_t L = 64 * (int64_t)CH;
  const int64_t nranges = (N + L - 1) / L;
  w.part.ensure(sizeof(double) * (size_t)(nranges > 0 ? nranges : 1) * 2 * (T.kp + 1));
  const int64_t ublocks = (nranges + (kBlock / 64) - 1) / (kBlock / 64);
  w.ucnt.ensure(sizeof(uint32_t) * (size_t)(ublocks > 0 ? ublocks : 1));
  SegArgs a;
  a.T = T;
  a.skeys = skeys;
  a.sents = sents;
  a.N = N;
  a.S = src.S;
  a.yl = src.yl;
  a.s_stride_q = src.s_stride_q;
  a.yl_stride = src.yl_stride;
  a.part = w.part.as<double>();
  a.nranges = nranges;
  a.L = L;
  a.p = p;
  a.ucnt = w.ucnt.as<uint32_t>();
  a.emit = emit;
  if (nranges > 0) {
    const dim3 grid((unsigned)ublocks), blk(kBlock);
    if (nq > G) {
      hipLaunchKernelGGL((k_segment_update<16, 1>), grid, blk, 0, st, a);
    } else if (G == 1) {
      hipLaunchKernelGGL((k_segment_update<1, kUpdateChunks>), grid, blk, 0, st, a);
    } else if (G == 2) {
      hipLaunchKernelGGL((k_segment_update<2, kUpdateChunks>), grid, blk, 0, st, a);
    } else if (G == 4) {
      hipLaunchKernelGGL((k_segment_update<4, kUpdateChunks>), grid, blk, 0, st, a);
    } else if (G == 8) {
      hipLaunchKernelGGL((k_segment_update<8, kUpdateChunks>), grid, blk, 0, st, a);
    } else {
      hipLaunchKernelGGL((k_segment_update<16, kUpdateChunks>), grid, blk, 0, st, a);
    }
    FM_HIP_CHECK(hipGetLastError());
  }
  int64_t cblocks = (nranges + kBlock - 1) / kBlock;
  if (cblocks < 1) cblocks = 1;
  hipLaunchKernelGGL(k_segment_combine, dim3((unsigned)cblocks), dim3(kBlock), 0, st, a,
                     w.loss_part.as<double2>(), n_fwd_blocks, nranges > 0 ? ublocks : (int64_t)0, stats_out);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_init_random(const TableView& T, const int32_t* ids, int64_t n, int64_t id_begin, uint64_t seed,
                        double sd, int32_t epoch, double cumE, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_init_random, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, id_begin, seed, sd,
                     epoch, cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_load_rows(const TableView& T, const int32_t* ids, int64_t n, const double* w, const double* V,
                      int32_t epoch, double cumE, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_load_rows, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, T, ids, n, w, V, epoch, cumE);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_table_reset(const TableView& T, hipStream_t st) {
  if (T.rows <= 0) return;
  FM_HIP_CHECK(hipMemsetAsync(T.rec, 0, sizeof(float) * (size_t)T.rows * T.stride, st));
  hipLaunchKernelGGL(k_table_reset, dim3(grid_for(T.rows, kBlock)), dim3(kBlock), 0, st, T);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_repl_apply(const TableView& T, const float* grad, const StepParams& p, unsigned long long* n_touched,
                       hipStream_t st) {
  FM_HIP_CHECK(hipMemsetAsync(n_touched, 0, sizeof(unsigned long long), st));
  if (T.rows <= 0) return;
  const int nq = T.kp / 4;
  const int G = nq <= 1 ? 1 : nq <= 2 ? 2 : nq <= 4 ? 4 : nq <= 8 ? 8 : 16;
  const unsigned grid = grid_for(T.rows * G, kBlock);
  switch (G) {
    case 1: hipLaunchKernelGGL(k_repl_apply<1>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, n_touched); break;
    case 2: hipLaunchKernelGGL(k_repl_apply<2>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, n_touched); break;
    case 4: hipLaunchKernelGGL(k_repl_apply<4>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, n_touched); break;
    case 8: hipLaunchKernelGGL(k_repl_apply<8>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, n_touched); break;
    default: hipLaunchKernelGGL(k_repl_apply<16>, dim3(grid), dim3(kBlock), 0, st, T, grad, p, n_touched); break;
  }
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

void launch_predict(const TableView& T, const BatchDev& b, double cumE, int64_t num_features, double w0,
                    double lo, double hi, double* pred, hipStream_t st) {
  FM_REQUIRE(T.k <= 64, "fm_predict supports dimFactorization <= 64");
  FM_REQUIRE(T.shard_count == 1, "fm_predict needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  hipLaunchKernelGGL(k_predict, dim3(grid_for(b.n_rows, kBlock)), dim3(kBlock), 0, st, T, b.row_ptr.as<int64_t>(),
                     b.col.as<uint32_t>(), b.ent.as<uint2>(), b.n_rows, num_features, cumE, w0, lo, hi, pred);
  FM_HIP_CHECK(hipGetLastError());
}

void launch_loss_grad(const TableView& T, const BatchDev& b, double cumE, double w0, double* pred, double* loss,
                      double* dw, double* dv, int32_t* absent_flag, hipStream_t st) {
  FM_REQUIRE(T.k <= 64, "fm_loss_grad supports dimFactorization <= 64");
  FM_REQUIRE(T.shard_count == 1, "fm_loss_grad needs the whole table (shard_count == 1)");
  if (b.n_rows <= 0) return;
  hipLaunchKernelGGL(k_loss_grad, dim3(grid_for(b.n_rows, kBlock)), dim3(kBlock), 0, st, T,
                     b.row_ptr.as<int64_t>(), b.col.as<uint32_t>(), b.ent.as<uint2>(), b.label.as<float>(),
                     b.n_rows, cumE, w0, pred, loss, dw, dv, absent_flag);
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
