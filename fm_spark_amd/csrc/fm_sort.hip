// Stable LSD radix sort of (uint32 key, uint32 payload) pairs for gfx950.
//
// Replaces the reference's shuffle-by-featureId groupBy (FactorizationMachinesSGD.scala:148,
// FactorizationMachinesModel.scala:191 window) with a deterministic grouping: equal keys end
// up contiguous and in their original (CSR) order, so every per-feature sum downstream runs
// in a fixed order and the step is bitwise reproducible.
//
// Per pass (RB-bit digit, 9..10 bits: 27-bit feature slots take 3 passes of 9 bits; tiles of both
// kernels grouped by XCD):
//   count   : one 512-thread block per 4096-key tile, LDS histogram  -> counts[tile][digit]
//   chunk   : one block per 16 tiles, exclusive scan down each digit  -> counts, chunk sums
//   top     : 32 digits per block, exclusive scan of the chunk sums   -> chunk prefixes, digit totals
//   scatter : each wave ranks its 512 keys with RB ballots per round (wave64 match), the
//             block stages the tile in LDS in digit order, then writes runs coalesced; tiles
//             are mapped to XCDs in contiguous groups.
// The per-tile counts are tile-major: a tile's 2^RB counts are one contiguous row, written and read
// in 16 L2 requests (digit-major, the same counts cost one request per digit per tile, 1024 per tile
// between the count and the scatter, a third of a c3 pass's L2 requests; the step is bound by the
// L2 request rate).
// HBM traffic per pass: 4 B (count) + (4 + P) B read + (4 + P) B write per pair.
#include <type_traits>

#include "fm_device.h"
#include "fm_internal.h"

namespace fmhip {

namespace {

constexpr int kMaxRB = 11;   // digit width at most (the bucket sort's top-bit pass)
// the LSD passes' digits at most / at least (27-bit feature slots: 3 passes of 9 bits; 7- and 8-bit
// digits, 4 passes at c3, measured slower in the step: DESIGN.md §5)
constexpr int kLsdMaxRB = 10;
// 8 waves x 8 keys per lane; two blocks (16 waves) per CU (8192-key tiles on 1024-thread blocks
// measured slower in the step: DESIGN.md §5)
constexpr int kBlock = 512;
constexpr int kWaves = kBlock / 64;
constexpr int kMinRB = 9;
// digits per thread in the block scans (a block wider than the radix: one, on the first R threads)
template <int R>
constexpr int digits_per_thread() { return R >= kBlock ? R / kBlock : 1; }
constexpr int kRounds = 8;   // keys per thread per tile
constexpr int kTile = kBlock * kRounds;  // 4096 keys per tile
constexpr int kMaxRadix = 1 << kMaxRB;
// the bucket sort's top-bit pass at most (an 11-bit scatter on 1024-thread blocks outgrows the LDS)
constexpr int kBktMaxH = kBlock >= 1024 ? 10 : kMaxRB;
constexpr int kChunk = 16;   // tiles per chunk of the count scan

// Tile of a block: the tiles of one XCD (blocks b = x mod 8 are dispatched to XCD x) are
// contiguous, so a digit's runs written by neighbouring tiles meet in the same L2 and leave it as
// whole 64-B granules (a partly written granule costs a read-modify-write in HBM;
// tools/traffic_cal.hip), and a digit row's line of per-tile counts is written by one L2.
__device__ __forceinline__ int64_t tile_of_block(int64_t ntiles) {
  const int64_t per = (ntiles + 7) / 8;
  return (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
}

inline int64_t blocks_for_tiles(int64_t ntiles) { return (ntiles + 7) / 8 * 8; }

static_assert(kTile % (4 * kBlock) == 0, "count block must divide the tile into uint4 rounds");

// The bucket sort's oversized buckets (below): segments of the phase-1 output, each cut into
// 4096-key tiles, sorted by the same three kernels; their tile count is known on the device only.
struct BigPlan {
  const uint4* seg;      // {start, size, first tile, bucket} per segment
  const uint32_t* tseg;  // tile -> segment
  const uint32_t* meta;  // {segments, tiles}
};

// Block -> tile for a tile count T read on the device (XCD-grouped as above); -1 past the end.
__device__ __forceinline__ int64_t big_tile_of_block(uint32_t T) {
  const uint32_t per = (T + 7) / 8;
  const uint32_t q = blockIdx.x / 8;
  if (q >= per) return -1;
  const int64_t t = (int64_t)(blockIdx.x % 8) * per + q;
  return t < T ? t : -1;
}

// Tile of a block: keys [base, end) of it (end: the array's or the segment's end), its column in
// the per-digit counts, and (BIG) the segment.
struct TileGeo {
  int64_t tile, base, end;
  uint4 seg;
};

template <bool BIG>
__device__ __forceinline__ bool tile_geo(TileGeo& g, int64_t n, int64_t ntiles, const BigPlan& bp) {
  if constexpr (BIG) {
    g.tile = big_tile_of_block(bp.meta[1]);
    if (g.tile < 0) return false;
    g.seg = bp.seg[bp.tseg[g.tile]];
    g.base = (int64_t)g.seg.x + (g.tile - (int64_t)g.seg.z) * kTile;
    g.end = (int64_t)g.seg.x + g.seg.y;
  } else {
    g.tile = tile_of_block(ntiles);
    if (g.tile >= ntiles) return false;
    g.base = g.tile * kTile;
    g.end = n;
  }
  return true;
}

template <int RB, bool BIG = false>
__global__ __launch_bounds__(kBlock) void k_radix_count(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                        uint32_t* __restrict__ counts, int64_t ntiles,
                                                        BigPlan bp, bool vec) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  __shared__ uint32_t hist[R];
  TileGeo g;
  if (!tile_geo<BIG>(g, n, ntiles, bp)) return;  // block-uniform
  for (int d = threadIdx.x; d < R; d += kBlock) hist[d] = 0;
  lds_barrier();
  const int64_t base = g.base;
  // uint4 reads of whole tiles when the keys are 16-byte aligned (a split view of a dataset starts
  // anywhere; segments of the big path too)
  if (!BIG && vec && base + kTile <= g.end) {
    const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
    for (int i = 0; i < kTile / (4 * kBlock); ++i) {
      const uint4 q = k4[i * kBlock + threadIdx.x];
      atomicAdd(&hist[(q.x >> shift) & M], 1u);
      atomicAdd(&hist[(q.y >> shift) & M], 1u);
      atomicAdd(&hist[(q.z >> shift) & M], 1u);
      atomicAdd(&hist[(q.w >> shift) & M], 1u);
    }
  } else {
    for (int i = 0; i < kTile / kBlock; ++i) {
      const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
      if (idx < g.end) atomicAdd(&hist[(keys[idx] >> shift) & M], 1u);
    }
  }
  lds_barrier();
  for (int d = threadIdx.x; d < R; d += kBlock) counts[g.tile * R + d] = hist[d];
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// The count scan, level 1: block c takes tiles [16 c, 16 c + 16) and replaces each tile's counts by
// the digit's exclusive prefix within the chunk; the chunk's sums -> csum[c][digit].  BIG: over the
// device's tile count plus one empty tile past the end (its prefix: the segments' ends).
template <int RB, bool BIG = false>
__global__ __launch_bounds__(kBlock) void k_radix_chunk_scan(uint32_t* __restrict__ counts, int64_t ntiles,
                                                             uint32_t* __restrict__ csum, BigPlan bp) {
  constexpr int R = 1 << RB;
  constexpr int D = digits_per_thread<R>();
  const int64_t nt = BIG ? (int64_t)bp.meta[1] : ntiles;
  const int64_t ext = nt + (BIG ? 1 : 0);
  const int64_t t0 = (int64_t)blockIdx.x * kChunk;
  if (t0 >= ext || (int)threadIdx.x >= R) return;
  uint32_t v[kChunk][D];
#pragma unroll
  for (int j = 0; j < kChunk; ++j)
#pragma unroll
    for (int i = 0; i < D; ++i) v[j][i] = t0 + j < nt ? counts[(t0 + j) * R + threadIdx.x + i * kBlock] : 0u;
  uint32_t run[D];
#pragma unroll
  for (int i = 0; i < D; ++i) run[i] = 0;
#pragma unroll
  for (int j = 0; j < kChunk; ++j) {
    if (t0 + j < ext) {
#pragma unroll
      for (int i = 0; i < D; ++i) {
        counts[(t0 + j) * R + threadIdx.x + i * kBlock] = run[i];
        run[i] += v[j][i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < D; ++i) csum[(int64_t)blockIdx.x * R + threadIdx.x + i * kBlock] = run[i];
}

// The same on 256-thread blocks for the LSD passes: block (c, slice) takes tiles [16 c, 16 c + 16) of
// the 256 digits of its slice, one digit per thread -- a small block finds room on a CU beside the
// step's and the sort's blocks sooner (c3 0.964-0.967 ms per step against 0.967-0.971 with one
// 512-thread block per chunk, c2 0.167-0.173 against 0.170-0.176, c5 within the noise; three
// alternating reps, profiles/r05_b/ab)
template <int RB>
__global__ __launch_bounds__(256) void k_radix_chunk_scan256(uint32_t* __restrict__ counts, int64_t ntiles,
                                                             uint32_t* __restrict__ csum) {
  constexpr int R = 1 << RB;
  constexpr int TB = R < 256 ? R : 256;
  constexpr int S = R / TB;  // digit slices
  const int64_t c = blockIdx.x / S;
  const int d = (int)(blockIdx.x % S) * TB + threadIdx.x;
  const int64_t t0 = c * kChunk;
  uint32_t v[kChunk];
#pragma unroll
  for (int j = 0; j < kChunk; ++j) v[j] = t0 + j < ntiles ? counts[(t0 + j) * R + d] : 0u;
  uint32_t run = 0;
#pragma unroll
  for (int j = 0; j < kChunk; ++j) {
    if (t0 + j < ntiles) counts[(t0 + j) * R + d] = run;
    run += v[j];
  }
  csum[c * R + d] = run;
}

// The count scan, level 2: 32 digits per 256-thread block (a small block finds room on a CU beside
// the sort's and the step's blocks sooner), 8 slices of the chunks per digit; csum ->
// the digit's exclusive prefix over chunks, digit_tot[d] = the digit's total (not BIG).
template <bool BIG = false>
__global__ __launch_bounds__(256) void k_radix_chunk_top(uint32_t* __restrict__ csum, int64_t nchunks, int R,
                                                         uint32_t* __restrict__ digit_tot, BigPlan bp) {
  constexpr int kDig = 32, kSl = 8;
  __shared__ uint32_t part[kSl][kDig];
  const int dl = threadIdx.x % kDig, sl = threadIdx.x / kDig;
  const int d = blockIdx.x * kDig + dl;
  const int64_t nch = BIG ? ((int64_t)bp.meta[1] + 1 + kChunk - 1) / kChunk : nchunks;
  const int64_t per = (nch + kSl - 1) / kSl;
  const int64_t c0 = min(nch, sl * per), c1 = min(nch, c0 + per);
  uint32_t s = 0;
#pragma unroll 8
  for (int64_t c = c0; c < c1; ++c) s += csum[c * R + d];
  part[sl][dl] = s;
  __syncthreads();
  if (sl == 0) {
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < kSl; ++q) {
      const uint32_t x = part[q][dl];
      part[q][dl] = run;
      run += x;
    }
    if (!BIG) digit_tot[d] = run;
  }
  __syncthreads();
  uint32_t run = part[sl][dl];
#pragma unroll 8
  for (int64_t c = c0; c < c1; ++c) {
    const uint32_t x = csum[c * R + d];
    csum[c * R + d] = run;
    run += x;
  }
}

// Block-wide exclusive scan of R values held as D = R / kBlock consecutive values per thread.
template <int D>
__device__ __forceinline__ void block_excl_scan(uint32_t (&v)[D], uint32_t* wsum, int lane, int wave) {
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < D; ++i) t += v[i];
  const uint32_t incl = wave_incl_scan_u32(t, lane);
  if (lane == 63) wsum[wave] = incl;
  lds_barrier();
  uint32_t run = incl - t;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) run += (w < wave) ? wsum[w] : 0u;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const uint32_t c = v[i];
    v[i] = run;
    run += c;
  }
}

template <class P>
__device__ __forceinline__ P implicit_payload(int64_t idx);
template <>
__device__ __forceinline__ uint32_t implicit_payload<uint32_t>(int64_t idx) {
  return (uint32_t)idx;
}
template <>
__device__ __forceinline__ uint2 implicit_payload<uint2>(int64_t idx) {
  return make_uint2((uint32_t)idx, 0u);
}

template <class P, int RB, bool BIG = false>
__global__ __launch_bounds__(kBlock) void k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                          const P* __restrict__ vals_in,
                                                          uint32_t* __restrict__ keys_out,
                                                          P* __restrict__ vals_out, int64_t n,
                                                          int shift, const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ csum,
                                                          const uint32_t* __restrict__ digit_tot,
                                                          int64_t ntiles, BigPlan bp) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  constexpr int D = digits_per_thread<R>();  // digits per thread in the block scans
  const bool own = (int)threadIdx.x * D < R;  // this thread holds digits in the block scans
  // per-wave digit counts and their prefixes stay below the 4096-key tile: 16-bit counters for the
  // 10-bit digits keep the block at 74 KB of LDS, two blocks per CU (32-bit: 90 KB, one block)
  using HistT = typename std::conditional<(RB >= 10), uint16_t, uint32_t>::type;
  static_assert(kTile < 65536 || RB < 10, "16-bit tile histograms need tiles below 64K keys");
  __shared__ uint32_t s_keys[kTile];
  __shared__ P s_vals[kTile];
  __shared__ HistT wave_hist[kWaves][R];
  __shared__ uint32_t tile_start[R];
  __shared__ uint32_t glob_off[R];
  __shared__ uint32_t wsum[kWaves];

  TileGeo g;
  if (!tile_geo<BIG>(g, n, ntiles, bp)) return;  // block-uniform
  const int64_t tile = g.tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile_base = g.base;
  const int64_t wbase = tile_base + (int64_t)wave * (kTile / kWaves);
  uint32_t my_key[kRounds], my_rank[kRounds];
  P my_val[kRounds];
  // the tile's loads first: in flight while the digit offsets below are read and scanned
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    const bool valid = idx < g.end;
    my_key[r] = valid ? keys_in[idx] : 0u;
    my_val[r] = valid ? (vals_in ? vals_in[idx] : implicit_payload<P>(idx)) : P{};
  }
#pragma unroll
  for (int w = 0; w < kWaves; ++w)
    for (int d = tid; d < R; d += kBlock) wave_hist[w][d] = 0;

  // global base of (digit, this tile): exclusive scan of digit totals + row prefix.  BIG: the
  // segment's digit totals and prefixes are differences of the rows' running prefixes at its first
  // tile, at this tile and past its last tile.
  // a tile's running prefix of digit d: its chunk's prefix + its own prefix within the chunk
  auto prefix = [&](int64_t t, int d) { return csum[(t / kChunk) * R + d] + counts[t * R + d]; };
  if constexpr (BIG) {
    const int64_t h = g.seg.z, e = h + (g.seg.y + kTile - 1) / kTile;
    uint32_t v[D], at_h[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      at_h[i] = own ? prefix(h, tid * D + i) : 0u;
      v[i] = own ? prefix(e, tid * D + i) - at_h[i] : 0u;
    }
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (own) glob_off[tid * D + i] = g.seg.x + v[i] + prefix(tile, tid * D + i) - at_h[i];
  } else {
    uint32_t v[D];
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = own ? digit_tot[tid * D + i] : 0u;
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (own) glob_off[tid * D + i] = v[i] + prefix(tile, tid * D + i);
  }
  lds_barrier();

#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    const bool valid = idx < g.end;
    const uint32_t d = (my_key[r] >> shift) & M;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
    const uint32_t cnt = (uint32_t)__popcll(peers);
    const uint32_t prev = wave_hist[wave][d];
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) wave_hist[wave][d] = (HistT)(prev + cnt);
    __builtin_amdgcn_wave_barrier();
    my_rank[r] = valid ? prev + below : 0xFFFFFFFFu;
  }
  lds_barrier();

  // per-digit wave bases (exclusive over waves) and the tile's digit starts.
  {
    uint32_t v[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int d = tid * D + i;
      uint32_t acc = 0;
      if (own) {
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
          const uint32_t c = wave_hist[w][d];
          wave_hist[w][d] = (HistT)acc;
          acc += c;
        }
      }
      v[i] = acc;
    }
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      if (own) {
        tile_start[tid * D + i] = v[i];
        glob_off[tid * D + i] -= v[i];  // destination of staged element j of digit d: glob_off[d] + j
      }
    }
  }
  lds_barrier();

#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    if (my_rank[r] != 0xFFFFFFFFu) {
      const uint32_t d = (my_key[r] >> shift) & M;
      const uint32_t pos = tile_start[d] + wave_hist[wave][d] + my_rank[r];
      s_keys[pos] = my_key[r];
      s_vals[pos] = my_val[r];
    }
  }
  lds_barrier();

  const int64_t rem = g.end - tile_base;
  const int tile_n = rem < kTile ? (int)rem : kTile;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {  // unrolled: the rounds' LDS reads are issued together
    const int j = r * kBlock + tid;
    if (j >= tile_n) break;
    const uint32_t key = s_keys[j];
    const uint32_t d = (key >> shift) & M;
    const uint32_t dest = glob_off[d] + (uint32_t)j;
    keys_out[dest] = key;
    vals_out[dest] = s_vals[j];
  }
}

// ----------------------------------------------------------------------------- bucket sort
// Two-phase stable sort of (feature slot, entry) pairs, 52 B per pair instead of the LSD passes' 84
// (and 45 when only the multi runs are kept):
//   phase 1  one radix pass above (count / scan / scatter) on the top H bits: every pair lands in
//            its bucket, in input order;
//   phase 2  one 512-thread block per bucket (k_bucket_sort) orders the bucket by its low L bits in
//            LDS -- one or two in-LDS passes of <= 9 bits over packed words {sub-key << (32 - L) |
//            index in bucket}, the ranks from wave ballots, each lane holding its wave's part of the
//            bucket in registers -- and writes it out, gathering payloads by index from the bucket's
//            own (L2-resident) range.
// A feature's run never leaves its bucket, so phase 2 also knows every run whole: in SPLIT mode (the
// fused step's view, fm_kernels.hip "Singleton rows") it keeps only the entries of runs of two or
// more, compacted at the start of the bucket's range, and counts the rest; k_bucket_offsets scans
// the per-bucket counts and k_bucket_compact closes the gaps.  That replaces the split kernels
// (a count pass over all sorted keys, a scan, a scatter) that ran on the step's main stream.
// A bucket larger than the LDS image (a hot feature's run with its neighbours, or a bucket of one
// hot feature alone) is left by phase 2 to the "big path": the oversized buckets form a list of
// segments of the phase-1 output (k_big_plan), cut into 4096-key tiles, and the LSD kernels above
// order every segment by its low L bits at once, one or two 9-bit passes across all CUs; in SPLIT mode
// three more kernels (k_big_split_*) keep each segment's multi entries.  A skewed batch's hot buckets
// therefore cost what the same keys cost in the LSD sort, not one block's walk of a huge bucket.
constexpr int kBB = 512;           // phase-2 block: 8 waves, two blocks per CU (the image takes 60 KB)
constexpr int kBW = kBB / 64;
constexpr int kBktCap = 30 * kBB;  // a bucket up to this size is ordered in LDS
constexpr int kBktRB = 9;          // digit bits of one in-bucket pass (512 digits)
constexpr int kBktNR = kBktCap / kBB;  // packed words per lane at most
constexpr int kBktU = 4;           // output rounds of kBB entries whose loads are issued together
static_assert(kBktCap <= 32768, "packed LDS words hold a 15-bit index next to a 17-bit sub-key");

struct BktShared {
  uint32_t arr[kBktCap];            // packed {sub, idx} in the order of the previous pass
  uint32_t cnt[kBW][1 << kBktRB];   // per-wave digit counts -> running destinations
  uint32_t wsum[kBktU][kBW];
  uint32_t misc[4];
};

__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid, int rb) {
  uint64_t peers = __ballot(valid);
  for (int b = 0; b < rb; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Exclusive scan of one value per thread over the phase-2 block (wsum: kBW words).
__device__ __forceinline__ uint32_t bkt_excl_scan(uint32_t v, uint32_t* wsum, int lane, int wave) {
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) wsum[wave] = incl;
  lds_barrier();
  uint32_t pre = incl - v;
#pragma unroll
  for (int w = 0; w < kBW; ++w) pre += (w < wave) ? wsum[w] : 0u;
  lds_barrier();
  return pre;
}

struct BktIO {
  const uint32_t* keys;  // the bucket's keys (phase-1 output)
  const uint2* vals;     // its payloads
  uint32_t* okeys;       // where the bucket's range starts in the output
  uint2* ovals;
  uint32_t hi;           // bucket << L
  uint32_t lmask;        // (1 << L) - 1
  int ib;                // 32 - L: index bits of the packed LDS word
};

// In-LDS pass for a bucket of m <= kBktCap entries, in place in S.arr (digit (sub >> shift) &
// (2^rb - 1), rb <= 9: the ranks take rb ballots per 64 entries).
template <bool FROM_KEYS>
__device__ __forceinline__ void bucket_pass_lds(BktShared& S, const BktIO& io, uint32_t m, int shift, int rb) {
  const int R = 1 << rb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t M = (uint32_t)R - 1u;
  const int dsh = io.ib + shift;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t part = ((m + kBW - 1) / kBW + 63u) & ~63u;
  const uint32_t lo = min(m, (uint32_t)wave * part);
  const int nvw = (int)(min(m, lo + part) - lo);
  uint32_t v[kBktNR], loc[kBktNR];
#pragma unroll
  for (int r = 0; r < kBktNR; ++r) {
    const uint32_t e = lo + r * 64 + lane;
    v[r] = 0;
    if (r * 64 + lane < nvw) v[r] = FROM_KEYS ? (((io.keys[e] & io.lmask) << io.ib) | e) : S.arr[e];
  }
  for (int d = tid; d < kBW * R; d += kBB) S.cnt[d / R][d % R] = 0;
  lds_barrier();  // every part is in registers: S.arr may be overwritten below
#pragma unroll
  for (int r = 0; r < kBktNR; ++r) {
    if (r * 64 >= nvw) break;
    const bool valid = r * 64 + lane < nvw;
    const uint32_t d = (v[r] >> dsh) & M;
    const uint64_t peers = digit_peers(d, valid, rb);
    const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
    const uint32_t prev = S.cnt[wave][d];
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) S.cnt[wave][d] = prev + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
    loc[r] = prev + below;
  }
  lds_barrier();
  uint32_t t = 0;
  if (tid < R) {
#pragma unroll
    for (int w = 0; w < kBW; ++w) {
      const uint32_t x = S.cnt[w][tid];
      S.cnt[w][tid] = t;
      t += x;
    }
  }
  const uint32_t base = bkt_excl_scan(t, S.wsum[0], lane, wave);
  if (tid < R) {
#pragma unroll
    for (int w = 0; w < kBW; ++w) S.cnt[w][tid] += base;
  }
  lds_barrier();
#pragma unroll
  for (int r = 0; r < kBktNR; ++r) {
    if (r * 64 + lane < nvw) S.arr[S.cnt[wave][(v[r] >> dsh) & M] + loc[r]] = v[r];
  }
  lds_barrier();
}

// Phase 2: block b sorts bucket b (btot[b] pairs starting at the sum of the buckets below it), if
// it fits the LDS image (else: the big path).  SPLIT: the bucket's multi entries go compacted to the
// start of its range of keys_out / vals_out, bstat[b] = {multi entries, singleton runs}; else the
// whole bucket, in order.
template <bool SPLIT>
__global__ __launch_bounds__(kBB) void k_bucket_sort(const uint32_t* __restrict__ keys_in,
                                                     const uint2* __restrict__ vals_in, uint32_t* __restrict__ keys_out,
                                                     uint2* __restrict__ vals_out, const uint32_t* __restrict__ btot,
                                                     int L, uint2* __restrict__ bstat) {
  __shared__ BktShared S;
  const int b = (int)blockIdx.x;
  const uint32_t m = btot[b];
  const uint32_t cap = min((uint32_t)kBktCap, 1u << min(32 - L, 31));
  if (m > cap) return;  // block-uniform: the big path's
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t acc = 0;
  for (int i = tid; i < b; i += kBB) acc += btot[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) S.wsum[0][wave] = acc;
  lds_barrier();
  uint32_t start = 0;
#pragma unroll
  for (int w = 0; w < kBW; ++w) start += S.wsum[0][w];
  lds_barrier();  // wsum is reused below
  if (m == 0) {   // block-uniform
    if (SPLIT && tid == 0) bstat[b] = make_uint2(0u, 0u);
    return;
  }
  BktIO io;
  io.keys = keys_in + start;
  io.vals = vals_in + start;
  io.okeys = keys_out + start;
  io.ovals = vals_out + start;
  io.hi = (uint32_t)b << L;
  io.lmask = (1u << L) - 1u;
  io.ib = 32 - L;
  uint32_t mcnt = 0;
  {
    bucket_pass_lds<true>(S, io, m, 0, L < kBktRB ? L : kBktRB);
    if (L > kBktRB) bucket_pass_lds<false>(S, io, m, kBktRB, L - kBktRB);
    // the bucket in order in S.arr: coalesced key and payload writes, payloads gathered by index from
    // the bucket's own range
    const uint32_t imask = (1u << io.ib) - 1u;
    for (uint32_t j0 = 0; j0 < m; j0 += kBktU * kBB) {
      uint32_t w[kBktU], pos[kBktU];
      bool keep[kBktU];
#pragma unroll
      for (int u = 0; u < kBktU; ++u) {
        const uint32_t j = j0 + u * kBB + tid;
        w[u] = j < m ? S.arr[j] : 0u;
        pos[u] = j;
        keep[u] = j < m;
        if (SPLIT) {
          const uint32_t sub = w[u] >> io.ib;
          const bool same_prev = j < m && j > 0 && (S.arr[j - 1] >> io.ib) == sub;
          const bool same_next = j + 1 < m && (S.arr[j + 1] >> io.ib) == sub;
          keep[u] = same_prev || same_next;
          const uint64_t bm = __ballot(keep[u]);
          pos[u] = (uint32_t)__popcll(bm & lt_mask);
          if (lane == 0) S.wsum[u][wave] = (uint32_t)__popcll(bm);
        }
      }
      if (SPLIT) {
        lds_barrier();
        uint32_t base = mcnt;
#pragma unroll
        for (int u = 0; u < kBktU; ++u) {
          uint32_t pre = 0, tot = 0;
#pragma unroll
          for (int wv = 0; wv < kBW; ++wv) {
            const uint32_t c = S.wsum[u][wv];
            pre += wv < wave ? c : 0u;
            tot += c;
          }
          pos[u] += base + pre;
          base += tot;
        }
        mcnt = base;
        lds_barrier();  // wsum is rewritten by the next rounds
      }
      uint2 pv[kBktU];
#pragma unroll
      for (int u = 0; u < kBktU; ++u)
        if (keep[u]) pv[u] = io.vals[w[u] & imask];
#pragma unroll
      for (int u = 0; u < kBktU; ++u) {
        if (keep[u]) {
          io.okeys[pos[u]] = io.hi | (w[u] >> io.ib);
          io.ovals[pos[u]] = pv[u];
        }
      }
    }
  }
  if (SPLIT && tid == 0) bstat[b] = make_uint2(mcnt, m - mcnt);
}

// The big path's plan, one block: the oversized buckets (btot[b] > cap) as segments {start, size,
// first tile, bucket} in bucket order, every tile's segment, meta = {segments, tiles}.
__global__ __launch_bounds__(kBB) void k_big_plan(const uint32_t* __restrict__ btot, int nb, uint32_t cap,
                                                  uint4* __restrict__ seg, uint32_t* __restrict__ tseg,
                                                  uint32_t* __restrict__ meta) {
  __shared__ uint32_t wsum[kBW];
  __shared__ uint32_t tot[3];
  __shared__ uint32_t first[kMaxRadix];  // first tile of each segment
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t c_start = 0, c_seg = 0, c_tiles = 0;  // block-uniform carries
  for (int b0 = 0; b0 < nb; b0 += kBB) {
    const int b = b0 + tid;
    const uint32_t sz = b < nb ? btot[b] : 0u;
    const uint32_t big = sz > cap ? 1u : 0u;
    const uint32_t tl = big ? (sz + kTile - 1) / kTile : 0u;
    const uint32_t start = bkt_excl_scan(sz, wsum, lane, wave);
    const uint32_t j = bkt_excl_scan(big, wsum, lane, wave);
    const uint32_t t0 = bkt_excl_scan(tl, wsum, lane, wave);
    if (big) {
      seg[c_seg + j] = make_uint4(c_start + start, sz, c_tiles + t0, (uint32_t)b);
      first[c_seg + j] = c_tiles + t0;
    }
    if (tid == kBB - 1) {
      tot[0] = start + sz;
      tot[1] = j + big;
      tot[2] = t0 + tl;
    }
    lds_barrier();
    c_start += tot[0];
    c_seg += tot[1];
    c_tiles += tot[2];
    lds_barrier();
  }
  // a tile's segment: the last one starting at or before it
  for (uint32_t t = tid; t < c_tiles; t += kBB) {
    uint32_t lo = 0, hi = c_seg - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) / 2;
      if (first[mid] <= t)
        lo = mid;
      else
        hi = mid - 1;
    }
    tseg[t] = lo;
  }
  if (tid == 0) {
    meta[0] = c_seg;
    meta[1] = c_tiles;
  }
}

// Is the sorted entry idx of segment [lo, end) in a run of two or more?
__device__ __forceinline__ bool big_multi(const uint32_t* __restrict__ keys, int64_t idx, int64_t lo, int64_t end,
                                          uint32_t key) {
  return (idx > lo && keys[idx - 1] == key) || (idx + 1 < end && keys[idx + 1] == key);
}

// SPLIT, big path: multi entries per sorted tile -> mt[tile].
__global__ __launch_bounds__(kBlock) void k_big_split_count(const uint32_t* __restrict__ keys, BigPlan bp,
                                                            uint32_t* __restrict__ mt) {
  __shared__ uint32_t wsum[kWaves];
  TileGeo g;
  if (!tile_geo<true>(g, 0, 0, bp)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = g.base + (int64_t)r * kBlock + threadIdx.x;
    if (idx < g.end) c += big_multi(keys, idx, g.seg.x, g.end, keys[idx]) ? 1u : 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) wsum[wave] = c;
  lds_barrier();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += wsum[w];
    mt[g.tile] = t;
  }
}

// SPLIT, big path, one block: mt -> exclusive prefix over all tiles (mt[tiles] = total), and each
// oversized bucket's bstat = {multi entries, singleton runs}.
__global__ __launch_bounds__(kBB) void k_big_split_scan(BigPlan bp, uint32_t* __restrict__ mt,
                                                        uint2* __restrict__ bstat) {
  __shared__ uint32_t wsum[kBW];
  __shared__ uint32_t tot;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t T = bp.meta[1], nseg = bp.meta[0];
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < T; t0 += kBB) {
    const uint32_t t = t0 + tid;
    const uint32_t v = t < T ? mt[t] : 0u;
    const uint32_t pre = bkt_excl_scan(v, wsum, lane, wave);
    if (t < T) mt[t] = carry + pre;
    if (tid == kBB - 1) tot = pre + v;
    lds_barrier();
    carry += tot;
    lds_barrier();
  }
  if (tid == 0) mt[T] = carry;
  __syncthreads();  // the block's global writes of mt, visible to all its threads
  for (uint32_t j = tid; j < nseg; j += kBB) {
    const uint4 s = bp.seg[j];
    const uint32_t e = s.z + (s.y + kTile - 1) / kTile;
    const uint32_t multi = mt[e] - mt[s.z];
    bstat[s.w] = make_uint2(multi, s.y - multi);
  }
}

// SPLIT, big path: each sorted tile's multi entries straight to their place in the dense multi view
// (the bucket's offset there, boff[b].y, + the tile's prefix within the segment), stable.  Each wave
// walks its own 512 entries.
__global__ __launch_bounds__(kBlock) void k_big_split_write(const uint32_t* __restrict__ keys,
                                                            const uint2* __restrict__ vals, BigPlan bp,
                                                            const uint32_t* __restrict__ mt,
                                                            const uint2* __restrict__ boff,
                                                            uint32_t* __restrict__ mkeys, uint2* __restrict__ mvals) {
  __shared__ uint32_t wsum[kWaves];
  TileGeo g;
  if (!tile_geo<true>(g, 0, 0, bp)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t wbase = g.base + (int64_t)wave * (kTile / kWaves);
  uint32_t key[kRounds];
  bool multi[kRounds];
  uint32_t c = 0;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    key[r] = idx < g.end ? keys[idx] : 0u;
    multi[r] = idx < g.end && big_multi(keys, idx, g.seg.x, g.end, key[r]);
    c += (uint32_t)__popcll(__ballot(multi[r]));
  }
  if (lane == 0) wsum[wave] = c;
  lds_barrier();
  uint32_t dst = boff[g.seg.w].y + mt[g.tile] - mt[g.seg.z];
#pragma unroll
  for (int w = 0; w < kWaves; ++w) dst += w < wave ? wsum[w] : 0u;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const uint64_t bm = __ballot(multi[r]);
    if (multi[r]) {
      const uint32_t d = dst + (uint32_t)__popcll(bm & lt_mask);
      mkeys[d] = key[r];
      mvals[d] = vals[wbase + (int64_t)r * 64 + lane];
    }
    dst += (uint32_t)__popcll(bm);
  }
}

// SPLIT: the buckets' starts (from their sizes) and the multi view's offsets (from their multi
// counts), exclusive scans over at most 1024 buckets; n_out[0] = multi entries, n_out[1] = singleton
// runs.  One block.
__global__ __launch_bounds__(kBB) void k_bucket_offsets(const uint32_t* __restrict__ btot,
                                                        const uint2* __restrict__ bstat, int nb,
                                                        uint2* __restrict__ boff, int64_t* __restrict__ n_out) {
  __shared__ uint32_t wsum[kBW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t c_start = 0, c_moff = 0, c_sing = 0;  // block-uniform carries
  for (int b0 = 0; b0 < nb; b0 += kBB) {
    const int b = b0 + tid;
    const uint32_t sz = b < nb ? btot[b] : 0u;
    const uint2 st = b < nb ? bstat[b] : make_uint2(0u, 0u);
    const uint32_t start = bkt_excl_scan(sz, wsum, lane, wave);
    const uint32_t moff = bkt_excl_scan(st.x, wsum, lane, wave);
    const uint32_t sing = bkt_excl_scan(st.y, wsum, lane, wave);
    if (b < nb) boff[b] = make_uint2(c_start + start, c_moff + moff);
    // the round's totals, from its last thread
    if (tid == kBB - 1) {
      wsum[0] = start + sz;
      wsum[1] = moff + st.x;
      wsum[2] = sing + st.y;
    }
    lds_barrier();
    c_start += wsum[0];
    c_moff += wsum[1];
    c_sing += wsum[2];
    lds_barrier();
  }
  if (tid == 0) {
    n_out[0] = (int64_t)c_moff;
    n_out[1] = (int64_t)c_sing;
  }
}

// SPLIT: bucket b's multi entries, compacted at its range's start in the gapped view, to their
// place in the dense multi view.  One block per bucket that fits the LDS image (the big path's
// buckets went there directly).
__global__ __launch_bounds__(256) void k_bucket_compact(const uint32_t* __restrict__ gkeys,
                                                        const uint2* __restrict__ gvals,
                                                        const uint2* __restrict__ bstat,
                                                        const uint2* __restrict__ boff, const uint32_t* __restrict__ btot,
                                                        uint32_t cap, uint32_t* __restrict__ mkeys,
                                                        uint2* __restrict__ mvals) {
  const int b = blockIdx.x;
  if (btot[b] > cap) return;
  const uint32_t n = bstat[b].x;
  const uint2 o = boff[b];
  for (uint32_t j = threadIdx.x; j < n; j += 256) {
    mkeys[o.y + j] = gkeys[o.x + j];
    mvals[o.y + j] = gvals[o.x + j];
  }
}

}  // namespace

// Rows of 2^RB counts the counts buffer holds for a sort of ntiles tiles: the tiles' (and one
// past them), then the chunks' sums.
inline int64_t count_rows(int64_t ntiles) { return ntiles + 1 + (ntiles + 1 + kChunk - 1) / kChunk; }

void SortWork::ensure(int64_t n) {
  if (n <= cap) return;
  const int64_t c = n + n / 8 + 4096;
  keys_a.ensure(sizeof(uint32_t) * c);
  keys_b.ensure(sizeof(uint32_t) * c);
  vals_a.ensure(sizeof(uint64_t) * c);  // payloads up to 8 bytes
  vals_b.ensure(sizeof(uint64_t) * c);
  const int64_t ntiles = (c + kTile - 1) / kTile;
  counts.ensure(sizeof(uint32_t) * kMaxRadix * count_rows(ntiles));
  digit_tot.ensure(sizeof(uint32_t) * kMaxRadix);  // digit totals (the bucket sort: bucket sizes)
  bstat.ensure(sizeof(uint2) * kMaxRadix * 2);         // per bucket {multi, singleton runs}, then {start, moff}
  cap = c;
}

template <class P, int RB>
static void radix_pass_impl(const uint32_t* kin, const P* vin, uint32_t* ko, P* vo, int64_t n, int shift,
                       SortWork& w, int64_t ntiles, hipStream_t st) {
  const BigPlan none{};
  uint32_t* counts = w.counts.as<uint32_t>();
  uint32_t* csum = counts + (ntiles + 1) * (int64_t(1) << RB);
  const int64_t nchunks = (ntiles + kChunk - 1) / kChunk;
  // (count and chunk scan fused into one kernel, a block walking its chunk's 16 tiles, measured
  // slower: 0.349 against 0.317 ms standalone)
  const bool vec = (reinterpret_cast<uintptr_t>(kin) & 15u) == 0;
  hipLaunchKernelGGL(k_radix_count<RB>, dim3((unsigned)blocks_for_tiles(ntiles)), dim3(kBlock), 0, st, kin, n, shift,
                     counts, ntiles, none, vec);
  constexpr int TB = (1 << RB) < 256 ? (1 << RB) : 256;
  hipLaunchKernelGGL(k_radix_chunk_scan256<RB>, dim3((unsigned)(nchunks * ((1 << RB) / TB))), dim3(TB), 0, st, counts,
                     ntiles, csum);
  hipLaunchKernelGGL(k_radix_chunk_top<false>, dim3((1u << RB) / 32), dim3(256), 0, st, csum, nchunks, 1 << RB,
                     w.digit_tot.as<uint32_t>(), none);
  hipLaunchKernelGGL((k_radix_scatter<P, RB>), dim3((unsigned)blocks_for_tiles(ntiles)), dim3(kBlock), 0, st, kin,
                     vin, ko, vo, n, shift, (const uint32_t*)counts, (const uint32_t*)csum,
                     (const uint32_t*)w.digit_tot.as<uint32_t>(), ntiles, none);
  FM_HIP_CHECK(hipGetLastError());
}

template <class P, int RB>
static void radix_pass(const uint32_t* kin, const P* vin, uint32_t* ko, P* vo, int64_t n, int shift,
                       SortWork& w, int64_t ntiles, hipStream_t st) {
  radix_pass_impl<P, RB>(kin, vin, ko, vo, n, shift, w, ntiles, st);
}

// Digit width: the fewest passes of at most kMaxRB bits, spread evenly (27-bit feature
// slots: 3 passes of 9 bits), never narrower than kMinRB bits.
inline int digit_bits(int key_bits, int* passes) {
  const int kb = key_bits < 1 ? 1 : key_bits;
  int p = (kb + kLsdMaxRB - 1) / kLsdMaxRB;
  int rb = (kb + p - 1) / p;
  if (rb < kMinRB) rb = kMinRB;
  p = (kb + rb - 1) / rb;
  *passes = p;
  return rb;
}

template <class P>
static void radix_sort_impl(SortWork& w, const uint32_t* keys_in, const P* vals_in, int64_t n, int key_bits,
                            hipStream_t st, const uint32_t** keys_out, const P** vals_out,
                            uint32_t* final_keys = nullptr, P* final_vals = nullptr, int lo_bit = 0) {
  FM_REQUIRE(n >= 0 && n < (int64_t(1) << 32) - 1, "sort size out of range");
  w.ensure(n > 0 ? n : 1);
  if (n == 0) {
    *keys_out = w.keys_a.as<uint32_t>();
    *vals_out = w.vals_a.as<P>();
    return;
  }
  int passes = 0;
  const int rb = digit_bits(key_bits, &passes);
  const int64_t ntiles = (n + kTile - 1) / kTile;
  FM_REQUIRE(ntiles < (int64_t(1) << 31), "too many sort tiles");
  const uint32_t* kin = keys_in;
  const P* vin = vals_in;
  uint32_t* kbuf[2] = {w.keys_a.as<uint32_t>(), w.keys_b.as<uint32_t>()};
  P* vbuf[2] = {w.vals_a.as<P>(), w.vals_b.as<P>()};
  int which = 0;
  for (int p = 0; p < passes; ++p) {
    const int shift = lo_bit + rb * p;
    const bool last = p == passes - 1 && final_keys != nullptr;
    uint32_t* ko = last ? final_keys : kbuf[which];
    P* vo = last ? final_vals : vbuf[which];
    switch (rb) {
      case 6: radix_pass<P, 6>(kin, vin, ko, vo, n, shift, w, ntiles, st); break;
      case 7: radix_pass<P, 7>(kin, vin, ko, vo, n, shift, w, ntiles, st); break;
      case 8: radix_pass<P, 8>(kin, vin, ko, vo, n, shift, w, ntiles, st); break;
      case 9: radix_pass<P, 9>(kin, vin, ko, vo, n, shift, w, ntiles, st); break;
      default: radix_pass<P, 10>(kin, vin, ko, vo, n, shift, w, ntiles, st); break;
    }
    kin = ko;
    vin = vo;
    which ^= 1;
  }
  *keys_out = kin;
  *vals_out = vin;
}

void radix_sort_pairs(SortWork& w, const uint32_t* keys_in, const uint32_t* vals_in, int64_t n, int key_bits,
                      hipStream_t st, const uint32_t** keys_out, const uint32_t** vals_out) {
  radix_sort_impl<uint32_t>(w, keys_in, vals_in, n, key_bits, st, keys_out, vals_out);
}

void radix_sort_pairs64_bits(SortWork& w, const uint32_t* keys_in, const uint2* vals_in, int64_t n, int lo_bit,
                             int hi_bit, hipStream_t st, uint32_t* final_keys, uint2* final_vals) {
  FM_REQUIRE(lo_bit >= 0 && hi_bit > lo_bit && hi_bit <= 32, "bad sort bit range");
  const uint32_t* ko = nullptr;
  const uint2* vo = nullptr;
  radix_sort_impl<uint2>(w, keys_in, vals_in, n, hi_bit - lo_bit, st, &ko, &vo, final_keys, final_vals, lo_bit);
}

void radix_sort_pairs64(SortWork& w, const uint32_t* keys_in, const uint2* vals_in, int64_t n, int key_bits,
                        hipStream_t st, const uint32_t** keys_out, const uint2** vals_out, uint32_t* final_keys,
                        uint2* final_vals) {
  radix_sort_impl<uint2>(w, keys_in, vals_in, n, key_bits, st, keys_out, vals_out, final_keys, final_vals);
}

}  // namespace fmhip

namespace fmhip {

// One LSD pass of the big path over the device-planned tiles (at most big_tiles of them).
template <int RB>
static void big_pass(const uint32_t* sk, const uint2* sv, uint32_t* dk, uint2* dv, int shift, SortWork& w,
                     const BigPlan& bp, int64_t big_tiles, hipStream_t st) {
  uint32_t* counts = w.counts.as<uint32_t>();
  uint32_t* csum = counts + (big_tiles + 1) * (int64_t(1) << RB);
  const unsigned gb = (unsigned)blocks_for_tiles(big_tiles);
  const unsigned gc = (unsigned)((big_tiles + 1 + kChunk - 1) / kChunk);
  hipLaunchKernelGGL((k_radix_count<RB, true>), dim3(gb), dim3(kBlock), 0, st, sk, (int64_t)0, shift, counts, (int64_t)0,
                     bp, false);
  hipLaunchKernelGGL((k_radix_chunk_scan<RB, true>), dim3(gc), dim3(kBlock), 0, st, counts, (int64_t)0, csum, bp);
  hipLaunchKernelGGL(k_radix_chunk_top<true>, dim3((1u << RB) / 32), dim3(256), 0, st, csum, (int64_t)0, 1 << RB,
                     (uint32_t*)nullptr, bp);
  hipLaunchKernelGGL((k_radix_scatter<uint2, RB, true>), dim3(gb), dim3(kBlock), 0, st, sk, sv, dk, dv, (int64_t)0,
                     shift, (const uint32_t*)counts, (const uint32_t*)csum, (const uint32_t*)nullptr, (int64_t)0, bp);
}

int bucket_hi_bits(int64_t n, int key_bits) {
  if (n < 1 || n >= (int64_t(1) << 32) - 1) return 0;
  // buckets of about a third of the LDS image on average (hot features fill some to the image and
  // beyond), 9 to 11 top bits
  int H = 9;
  while (H < kBktMaxH && n / (int64_t(1) << H) > kBktCap / 3) ++H;
  if (key_bits < H + 1 || key_bits - H > 2 * kBktRB) return 0;  // one pass would do / too many low bits
  return H;
}

bool bucket_sort_pairs64(SortWork& w, const uint32_t* keys_in, const uint2* vals_in, int64_t n, int key_bits,
                         hipStream_t st, uint32_t* final_keys, uint2* final_vals, int64_t* split_out) {
  const int H = bucket_hi_bits(n, key_bits);
  if (H == 0) return false;
  FM_REQUIRE(final_keys && final_vals && vals_in, "bucket sort: null buffer");
  const int L = key_bits - H;
  const int nb = 1 << H;
  const uint32_t cap = std::min<uint32_t>((uint32_t)kBktCap, 1u << std::min(32 - L, 31));
  const int64_t ntiles = (n + kTile - 1) / kTile;
  // the big path: oversized buckets number at most n / (cap + 1), each adds at most one partial tile
  const int64_t big_tiles = ntiles + n / ((int64_t)cap + 1) + 1;
  // the big path's digits: one pass of 9..11 bits for L <= 11, else two of 9 (a digit reaching above
  // bit L holds bucket bits, constant in a segment)
  const int big_rb = L <= 9 ? 9 : L <= kBktMaxH ? L : kBktRB;
  const int passes = L <= kBktMaxH ? 1 : 2;
  w.ensure(n);
  // every buffer sized before the first launch (growing one drains the device)
  const size_t cnt_bytes = sizeof(uint32_t) * std::max<int64_t>((int64_t)kMaxRadix * count_rows((w.cap + kTile - 1) / kTile),
                                                                 ((int64_t)1 << big_rb) * count_rows(big_tiles));
  w.counts.ensure(cnt_bytes);
  const size_t scr_keys = ((sizeof(uint32_t) * (size_t)w.cap) + 255) & ~size_t(255);
  w.bscratch.ensure(scr_keys + sizeof(uint2) * (size_t)w.cap);  // the big path's middle pass
  const size_t seg_bytes = sizeof(uint4) * kMaxRadix, tseg_bytes = (sizeof(uint32_t) * big_tiles + 15) & ~size_t(15);
  w.bplan.ensure(seg_bytes + tseg_bytes + 16 + sizeof(uint32_t) * (big_tiles + 1));
  char* plan = w.bplan.as<char>();
  uint4* seg = reinterpret_cast<uint4*>(plan);
  uint32_t* tseg = reinterpret_cast<uint32_t*>(plan + seg_bytes);
  uint32_t* meta = reinterpret_cast<uint32_t*>(plan + seg_bytes + tseg_bytes);
  uint32_t* mt = meta + 4;
  const BigPlan bp{seg, tseg, meta};

  uint32_t* kbuf[2] = {w.keys_a.as<uint32_t>(), w.keys_b.as<uint32_t>()};
  uint2* vbuf[2] = {w.vals_a.as<uint2>(), w.vals_b.as<uint2>()};
  uint32_t* skeys = w.bscratch.as<uint32_t>();
  uint2* svals = reinterpret_cast<uint2*>(w.bscratch.as<char>() + scr_keys);
  const uint32_t* kin = keys_in;
  if ((reinterpret_cast<uintptr_t>(keys_in) & 15u) != 0) {  // the count kernel reads uint4
    FM_HIP_CHECK(hipMemcpyAsync(kbuf[1], keys_in, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, st));
    kin = kbuf[1];
  }
  // phase 1: the top H bits
  switch (H) {
    case 9: radix_pass<uint2, 9>(kin, vals_in, kbuf[0], vbuf[0], n, L, w, ntiles, st); break;
    case 10: radix_pass<uint2, 10>(kin, vals_in, kbuf[0], vbuf[0], n, L, w, ntiles, st); break;
    default:
      if constexpr (kBktMaxH >= 11) radix_pass<uint2, 11>(kin, vals_in, kbuf[0], vbuf[0], n, L, w, ntiles, st);
      break;
  }
  const uint32_t* btot = w.digit_tot.as<uint32_t>();
  uint2* bstat = w.bstat.as<uint2>();
  uint2* boff = bstat + kMaxRadix;
  hipLaunchKernelGGL(k_big_plan, dim3(1), dim3(kBB), 0, st, btot, nb, cap, seg, tseg, meta);
  // phase 2 (SPLIT: into the gapped view kbuf[1] / vbuf[1], the multi entries at each bucket's start)
  uint32_t* pk = split_out ? kbuf[1] : final_keys;
  uint2* pv = split_out ? vbuf[1] : final_vals;
  if (split_out)
    hipLaunchKernelGGL(k_bucket_sort<true>, dim3(nb), dim3(kBB), 0, st, kbuf[0], vbuf[0], pk, pv, btot, L, bstat);
  else
    hipLaunchKernelGGL(k_bucket_sort<false>, dim3(nb), dim3(kBB), 0, st, kbuf[0], vbuf[0], pk, pv, btot, L, bstat);
  // the big path: LSD passes over the low L bits of every oversized bucket; its sorted segments end
  // in the final buffers, or (SPLIT) where k_big_split_write reads them
  const unsigned gb = (unsigned)blocks_for_tiles(big_tiles);  // the split kernels' grid
  const uint32_t* sk = kbuf[0];
  const uint2* sv = vbuf[0];
  for (int p = 0; p < passes; ++p) {
    const bool last = p == passes - 1;
    uint32_t* dk = !last ? skeys : split_out ? (passes == 1 ? skeys : kbuf[0]) : final_keys;
    uint2* dv = !last ? svals : split_out ? (passes == 1 ? svals : vbuf[0]) : final_vals;
    switch (big_rb) {
      case 9: big_pass<9>(sk, sv, dk, dv, big_rb * p, w, bp, big_tiles, st); break;
      case 10: big_pass<10>(sk, sv, dk, dv, big_rb * p, w, bp, big_tiles, st); break;
      default:
        if constexpr (kBktMaxH >= 11) big_pass<11>(sk, sv, dk, dv, big_rb * p, w, bp, big_tiles, st);
        break;
    }
    sk = dk;
    sv = dv;
  }
  if (split_out) {
    // the big path's multi counts, every bucket's offsets, then the multi entries into the final
    // buffers: the big path's by tile, the others' by closing the gapped view's gaps
    hipLaunchKernelGGL(k_big_split_count, dim3(gb), dim3(kBlock), 0, st, sk, bp, mt);
    hipLaunchKernelGGL(k_big_split_scan, dim3(1), dim3(kBB), 0, st, bp, mt, bstat);
    hipLaunchKernelGGL(k_bucket_offsets, dim3(1), dim3(kBB), 0, st, btot, (const uint2*)bstat, nb, boff, split_out);
    hipLaunchKernelGGL(k_big_split_write, dim3(gb), dim3(kBlock), 0, st, sk, sv, bp, (const uint32_t*)mt,
                       (const uint2*)boff, final_keys, final_vals);
    hipLaunchKernelGGL(k_bucket_compact, dim3(nb), dim3(256), 0, st, kbuf[1], vbuf[1], (const uint2*)bstat,
                       (const uint2*)boff, btot, cap, final_keys, final_vals);
  }
  FM_HIP_CHECK(hipGetLastError());
  return true;
}

}  // namespace fmhip
