// Stable LSD radix sort of (uint32 key, uint32 payload) pairs for gfx950.
//
// Replaces the reference's shuffle-by-featureId groupBy (FactorizationMachinesSGD.scala:148,
// FactorizationMachinesModel.scala:191 window) with a deterministic grouping: equal keys end
// up contiguous and in their original (CSR) order, so every per-feature sum downstream runs
// in a fixed order and the step is bitwise reproducible.
//
// Per pass (RB-bit digit, 9..10 bits: 27-bit feature slots take 3 passes of 9 bits; tiles of both
// kernels grouped by XCD):
//   count   : one 512-thread block per 4096-key tile, LDS histogram  -> counts[digit][tile]
//   scan    : one block per digit, exclusive scan along tiles        -> counts, digit totals
//   scatter : each wave ranks its 512 keys with RB ballots per round (wave64 match), the
//             block stages the tile in LDS in digit order, then writes runs coalesced; tiles
//             are mapped to XCDs in contiguous groups.
// HBM traffic per pass: 4 B (count) + (4 + P) B read + (4 + P) B write per pair.
#include <type_traits>

#include "fm_device.h"
#include "fm_internal.h"

namespace fmhip {

namespace {

#ifndef FM_SORT_MAXRB
#define FM_SORT_MAXRB 10
#endif

#ifndef FM_SORT_CWAVE
#define FM_SORT_CWAVE 0  // count: one LDS histogram per wave (less same-address atomic contention)
#endif
#ifndef FM_SORT_H16
#define FM_SORT_H16 0  // 16-bit tile histograms for every digit width (always for 10-bit digits)
#endif
#ifndef FM_SORT_CXCD
#define FM_SORT_CXCD 1  // count: tiles mapped to XCDs like the scatter's (a count row's line is written by one L2)
#endif

#ifndef FM_SORT_BLOCK
#define FM_SORT_BLOCK 512
#endif
constexpr int kBlock = FM_SORT_BLOCK;  // 512: 8 waves x 8 keys per lane; two blocks (16 waves) per CU
static_assert(kBlock == 256 || kBlock == 512, "sort block must be 256 or 512 threads");
constexpr int kWaves = kBlock / 64;
constexpr int kMinRB = kBlock == 512 ? 9 : 8;  // the block scans hold R / kBlock >= 1 digits per thread
#ifndef FM_SORT_ROUNDS
#define FM_SORT_ROUNDS (4096 / FM_SORT_BLOCK)  // 4096-key tiles whatever the block size
#endif
constexpr int kRounds = FM_SORT_ROUNDS;  // keys per thread per tile
constexpr int kTile = kBlock * kRounds;  // 4096 keys per tile (unless FM_SORT_ROUNDS is overridden on purpose)
constexpr int kMaxRadix = 1 << 10;

// Tile of a block.  With FM_SORT_XCD the tiles of one XCD (blocks b = x mod 8 are dispatched
// to XCD x) are contiguous, so a digit's runs written by neighbouring tiles meet in the same L2
// and leave it as whole 64-B granules (a partly written granule costs a read-modify-write in
// HBM; tools/traffic_cal.hip).
__device__ __forceinline__ int64_t tile_of_block(int64_t ntiles) {
  const int64_t per = (ntiles + 7) / 8;
  return (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
}

inline int64_t blocks_for_tiles(int64_t ntiles) { return (ntiles + 7) / 8 * 8; }

// Experiment switch: the count and scan kernels on small blocks (4 waves; one wave per digit row),
// which slot into the room the step's 4-wave forward / update blocks free (in the step an 8-wave
// count or scan block takes 30 - 95 us instead of 7 - 17 alone).  Measured slower: the step is
// throughput-bound, not bound by these kernels' wait for CU room.
#ifndef FM_SORT_SMALLBLK
#define FM_SORT_SMALLBLK 0  // measured: c3 step 1.069-1.072 vs 1.053-1.062 ms with the 8-wave blocks (off)
#endif
constexpr int kCntBlock = FM_SORT_SMALLBLK ? 256 : kBlock;
static_assert(kTile % (4 * kCntBlock) == 0, "count block must divide the tile into uint4 rounds");

template <int RB>
__global__ __launch_bounds__(kCntBlock) void k_radix_count(const uint32_t* __restrict__ keys, int64_t n,
                                                           int shift, uint32_t* __restrict__ counts,
                                                           int64_t ntiles) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  constexpr int HW = FM_SORT_CWAVE ? kCntBlock / 64 : 1;
  __shared__ uint32_t hist_all[HW][R];
  uint32_t* hist = hist_all[FM_SORT_CWAVE ? (threadIdx.x >> 6) : 0];
#if FM_SORT_CXCD
  const int64_t tile = tile_of_block(ntiles);
  if (tile >= ntiles) return;  // block-uniform
#else
  const int64_t tile = blockIdx.x;
#endif
  for (int d = threadIdx.x; d < HW * R; d += kCntBlock) hist_all[d / R][d % R] = 0;
  lds_barrier();
  const int64_t base = tile * kTile;
  if (base + kTile <= n) {
    const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
    for (int i = 0; i < kTile / (4 * kCntBlock); ++i) {
      const uint4 q = ld_stream(k4 + i * kCntBlock + threadIdx.x, FM_NT_SORTLD);
      atomicAdd(&hist[(q.x >> shift) & M], 1u);
      atomicAdd(&hist[(q.y >> shift) & M], 1u);
      atomicAdd(&hist[(q.z >> shift) & M], 1u);
      atomicAdd(&hist[(q.w >> shift) & M], 1u);
    }
  } else {
    for (int i = 0; i < kTile / kCntBlock; ++i) {
      const int64_t idx = base + (int64_t)i * kCntBlock + threadIdx.x;
      if (idx < n) atomicAdd(&hist[(keys[idx] >> shift) & M], 1u);
    }
  }
  lds_barrier();
  for (int d = threadIdx.x; d < R; d += kCntBlock) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < HW; ++w) c += hist_all[w][d];
    counts[(int64_t)d * ntiles + tile] = c;
  }
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// Exclusive scan of each digit's row counts[d][0..ntiles), row totals -> digit_tot[d].
__global__ __launch_bounds__(kBlock) void k_radix_scan_rows(uint32_t* __restrict__ counts, int64_t ntiles,
                                                            uint32_t* __restrict__ digit_tot) {
  __shared__ uint32_t wsum[kWaves];
  uint32_t* row = counts + (int64_t)blockIdx.x * ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t b = 0; b < ntiles; b += kBlock) {
    const int64_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? row[i] : 0u;
    const uint32_t incl = wave_incl_scan_u32(v, lane);
    if (lane == 63) wsum[wave] = incl;
    lds_barrier();
    uint32_t wpre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t s = wsum[w];
      wpre += (w < wave) ? s : 0u;
      tot += s;
    }
    if (i < ntiles) row[i] = carry + wpre + incl - v;
    carry += tot;
    lds_barrier();
  }
  if (threadIdx.x == 0) digit_tot[blockIdx.x] = carry;
}

// The same scan with one wave per digit row (4 rows per 256-thread block): each lane takes 8
// consecutive tile counts per round, all loads of a round in flight together.
__global__ __launch_bounds__(256) void k_radix_scan_rows_w(uint32_t* __restrict__ counts, int64_t ntiles,
                                                           uint32_t* __restrict__ digit_tot, int R) {
  constexpr int J = 8;
  const int lane = threadIdx.x & 63;
  const int d = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= R) return;  // wave-uniform
  uint32_t* row = counts + (int64_t)d * ntiles;
  uint32_t carry = 0;
  for (int64_t c0 = 0; c0 < ntiles; c0 += 64 * J) {
    const int64_t b = c0 + (int64_t)lane * J;
    uint32_t v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = b + j < ntiles ? row[b + j] : 0u;
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint32_t x = v[j];
      v[j] = sum;
      sum += x;
    }
    const uint32_t incl = wave_incl_scan_u32(sum, lane);
    const uint32_t pre = carry + incl - sum;
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (b + j < ntiles) row[b + j] = pre + v[j];
    carry += __shfl(incl, 63);
  }
  if (lane == 0) digit_tot[d] = carry;
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

template <class P, int RB>
__global__ __launch_bounds__(kBlock) void k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                          const P* __restrict__ vals_in,
                                                          uint32_t* __restrict__ keys_out,
                                                          P* __restrict__ vals_out, int64_t n,
                                                          int shift, const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ digit_tot,
                                                          int64_t ntiles) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  constexpr int D = R / kBlock;  // digits per thread in the block scans
  // per-wave digit counts and their prefixes stay below the 4096-key tile: 16-bit counters for the
  // 10-bit digits keep the block at 74 KB of LDS, two blocks per CU (32-bit: 90 KB, one block)
  using HistT = typename std::conditional<(RB >= 10 || FM_SORT_H16), uint16_t, uint32_t>::type;
  static_assert(kTile < 65536 || RB < 10, "16-bit tile histograms need tiles below 64K keys");
  __shared__ uint32_t s_keys[kTile];
  __shared__ P s_vals[kTile];
  __shared__ HistT wave_hist[kWaves][R];
  __shared__ uint32_t tile_start[R];
  __shared__ uint32_t glob_off[R];
  __shared__ uint32_t wsum[kWaves];

  const int64_t tile = tile_of_block(ntiles);
  if (tile >= ntiles) return;  // block-uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile_base = tile * kTile;
  const int64_t wbase = tile_base + (int64_t)wave * (kTile / kWaves);
  uint32_t my_key[kRounds], my_rank[kRounds];
  P my_val[kRounds];
  // the tile's loads first: in flight while the digit offsets below are read and scanned
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    const bool valid = idx < n;
    my_key[r] = valid ? ld_stream(keys_in + idx, FM_NT_SORTLD) : 0u;
    my_val[r] = valid ? (vals_in ? ld_stream(vals_in + idx, FM_NT_SORTLD) : implicit_payload<P>(idx)) : P{};
  }
#pragma unroll
  for (int w = 0; w < kWaves; ++w)
    for (int d = tid; d < R; d += kBlock) wave_hist[w][d] = 0;

  // global base of (digit, this tile): exclusive scan of digit totals + row prefix.
  {
    uint32_t v[D];
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = digit_tot[tid * D + i];
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i) glob_off[tid * D + i] = v[i] + counts[(int64_t)(tid * D + i) * ntiles + tile];
  }
  lds_barrier();

#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    const bool valid = idx < n;
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
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const uint32_t c = wave_hist[w][d];
        wave_hist[w][d] = (HistT)acc;
        acc += c;
      }
      v[i] = acc;
    }
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      tile_start[tid * D + i] = v[i];
      glob_off[tid * D + i] -= v[i];  // destination of staged element j of digit d: glob_off[d] + j
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

  const int64_t rem = n - tile_base;
  const int tile_n = rem < kTile ? (int)rem : kTile;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {  // unrolled: the rounds' LDS reads are issued together
    const int j = r * kBlock + tid;
    if (j >= tile_n) break;
    const uint32_t key = s_keys[j];
    const uint32_t d = (key >> shift) & M;
#ifdef FM_SORT_ABL_LINEAR  // measurement only (wrong order): tile written in place
    const uint32_t dest = (uint32_t)(tile_base + j) + 0u * glob_off[d];
#else
    const uint32_t dest = glob_off[d] + (uint32_t)j;
#endif
#if FM_NT_SORT
    __builtin_nontemporal_store(key, keys_out + dest);
    if constexpr (sizeof(P) == 8) {
      const uint2 v = *reinterpret_cast<const uint2*>(&s_vals[j]);
      __builtin_nontemporal_store((unsigned long long)v.x | ((unsigned long long)v.y << 32),
                                  reinterpret_cast<unsigned long long*>(vals_out) + dest);
    } else {
      __builtin_nontemporal_store(*reinterpret_cast<const uint32_t*>(&s_vals[j]),
                                  reinterpret_cast<uint32_t*>(vals_out) + dest);
    }
#else
    keys_out[dest] = key;
    vals_out[dest] = s_vals[j];
#endif
  }
}

// ----------------------------------------------------------------------------- bucket sort
// Two-phase stable sort for large inputs with 12..28-bit keys.  Phase 1 is one radix pass above
// (count / scan / scatter) on the top H bits: every key lands in its bucket, in input order.
// Phase 2 runs one block per bucket over the low L = key_bits - H bits: two LSD passes (one when
// L <= 9) whose intermediate order stays in LDS as one packed word per entry, {sub-key << (32 - L)
// | index in bucket}; the last pass writes the bucket's keys and gathers its payloads from the
// bucket's own (L2-resident) range.  A bucket larger than the LDS image (a hot feature's run) keeps
// that intermediate order in a global scratch instead and is processed in LDS-sized chunks.
// HBM bytes per pair (P = 8): 4 + 12 + 12 (phase 1) + 12 + 12 (phase 2) = 52, against 84 for
// three LSD passes.
#ifndef FM_BKT_BLOCK
#define FM_BKT_BLOCK 1024  // phase-2 block: 16 waves, one block per CU (the LDS image takes 120 KB)
#endif
#ifndef FM_BKT_CAP
#define FM_BKT_CAP (30 * FM_BKT_BLOCK)
#endif
#ifndef FM_BKT_G
#define FM_BKT_G 8  // rounds of 64 entries per wave whose loads are issued together
#endif
constexpr int kBB = FM_BKT_BLOCK;             // phase-2 block
constexpr int kBW = kBB / 64;
constexpr int kBktCap = FM_BKT_CAP;           // a bucket up to this size keeps its order in LDS
constexpr int kBktMaxRB = 9;                  // digit bits of one in-bucket pass (<= 512 digits: one per thread)
static_assert(kBktCap <= 32768, "packed LDS words hold a 15-bit index next to a 17-bit sub-key");
static_assert(kBB == 512 || kBB == 1024, "phase-2 block of 8 or 16 waves");

struct BktShared {
  uint32_t arr[kBktCap];                // packed {sub, idx} in the order of the previous pass
  uint32_t cnt[kBW][1 << kBktMaxRB];    // per-wave digit counts -> running destinations
  uint32_t wsum[kBW];
};

enum BktSrc { kSrcKeys = 0, kSrcLds = 1, kSrcScratch = 2 };
enum BktDst { kDstLds = 0, kDstScratch = 1, kDstOut = 2 };  // kSrcLds / kDstLds: chunked variants, unused

__device__ __forceinline__ uint64_t digit_peers(uint32_t d, bool valid, int rb) {
  uint64_t peers = __ballot(valid);
  for (int b = 0; b < rb; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Exclusive scan of one value per thread over the 512-thread block.
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

template <bool GSYNC>
__device__ __forceinline__ void bkt_sync() {
  if (GSYNC)
    __syncthreads();  // the pass exchanges through global scratch: workgroup fence on global too
  else
    lds_barrier();
}

template <class P>
struct BktIO {
  const uint32_t* keys;  // bucket's keys (phase-1 output)
  const P* vals;         // bucket's payloads (phase-1 output)
  uint32_t* okeys;
  P* ovals;
  uint2* scratch;        // {sub, idx} per entry (oversized buckets)
  uint32_t hi;           // bucket << L
  uint32_t lmask;        // (1 << L) - 1
  int ib;                // 32 - L: index bits of the packed LDS word
};

// One stable counting pass over the m entries of a bucket by digit (sub >> shift) & (2^rb - 1),
// from SRC to DST.  Wave w owns the contiguous part [w p, (w + 1) p) of the bucket: a histogram
// sweep, a scan over (digit, wave), then a rank sweep with wave-private running counts.  Both
// sweeps take G rounds of 64 entries at a time so that their loads (and the last pass's payload
// gathers) are in flight together.
template <int SRC, int DST, bool GSYNC, class P>
__device__ __forceinline__ void bucket_pass(BktShared& S, const BktIO<P>& io, uint32_t m, int shift, int rb) {
  constexpr int G = FM_BKT_G;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = 1 << rb;
  const uint32_t M = (uint32_t)R - 1u;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t imask = (io.ib >= 32) ? 0xFFFFFFFFu : ((1u << io.ib) - 1u);
  const uint32_t part = ((m + kBW - 1) / kBW + 63u) & ~63u;
  const uint32_t lo = min(m, (uint32_t)wave * part), hi = min(m, lo + part);

  auto load = [&](uint32_t e, uint32_t& sub, uint32_t& idx) {
    if (SRC == kSrcKeys) {
      sub = io.keys[e] & io.lmask;
      idx = e;
    } else if (SRC == kSrcLds) {
      const uint32_t v = S.arr[e];
      sub = v >> io.ib;
      idx = v & imask;
    } else {
      const uint2 v = io.scratch[e];
      sub = v.x;
      idx = v.y;
    }
  };

  for (int d = tid; d < kBW * R; d += kBB) S.cnt[d / R][d % R] = 0;
  bkt_sync<GSYNC>();
  for (uint32_t e0 = lo; e0 < hi; e0 += 64 * G) {
    uint32_t sub[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t e = e0 + u * 64 + lane;
      uint32_t idx;
      sub[u] = 0;
      if (e < hi) load(e, sub[u], idx);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t e = e0 + u * 64 + lane;
      const bool valid = e < hi;
      const uint32_t d = (sub[u] >> shift) & M;
      const uint64_t peers = digit_peers(d, valid, rb);
      if (valid && __popcll(peers & lt_mask) == 0) S.cnt[wave][d] += (uint32_t)__popcll(peers);
    }
  }
  bkt_sync<GSYNC>();
  // destinations of (digit, wave): the digit's base + the counts of the earlier waves
  uint32_t t = 0;
  if (tid < R) {
#pragma unroll
    for (int w = 0; w < kBW; ++w) {
      const uint32_t x = S.cnt[w][tid];
      S.cnt[w][tid] = t;
      t += x;
    }
  }
  const uint32_t base = bkt_excl_scan(t, S.wsum, lane, wave);
  if (tid < R) {
#pragma unroll
    for (int w = 0; w < kBW; ++w) S.cnt[w][tid] += base;
  }
  lds_barrier();
  for (uint32_t e0 = lo; e0 < hi; e0 += 64 * G) {
    uint32_t sub[G], idx[G], pos[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t e = e0 + u * 64 + lane;
      sub[u] = 0;
      idx[u] = 0;
      if (e < hi) load(e, sub[u], idx[u]);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const uint32_t e = e0 + u * 64 + lane;
      const bool valid = e < hi;
      const uint32_t d = (sub[u] >> shift) & M;
      const uint64_t peers = digit_peers(d, valid, rb);
      const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
      const uint32_t prev = S.cnt[wave][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) S.cnt[wave][d] = prev + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      pos[u] = prev + below;
    }
    if (DST == kDstOut) {
      P v[G];
#pragma unroll
      for (int u = 0; u < G; ++u)
        if (e0 + u * 64 + lane < hi) v[u] = io.vals[idx[u]];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if (e0 + u * 64 + lane < hi) {
          io.okeys[pos[u]] = io.hi | sub[u];
          io.ovals[pos[u]] = v[u];
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if (e0 + u * 64 + lane < hi) {
          if (DST == kDstLds)
            S.arr[pos[u]] = (sub[u] << io.ib) | idx[u];
          else
            io.scratch[pos[u]] = make_uint2(sub[u], idx[u]);
        }
      }
    }
  }
  bkt_sync<GSYNC>();  // the next pass reads what this one wrote and resets cnt
}

// In-LDS pass for a bucket of m <= kBktCap entries, in place in S.arr: each lane holds its wave's
// part of the bucket in registers (packed {sub << ib | idx} words, read from the bucket's keys on the
// first pass), ranks it with one ballot sweep whose wave-private running counts end as the wave's
// digit histogram, and once every part is read and the (digit, wave) bases are scanned, stores each
// word at its destination.
constexpr int kBktNR = kBktCap / kBB;  // words per lane at most
static_assert(kBktCap % kBB == 0, "the LDS image must be a multiple of the block");

template <bool FROM_KEYS, class P>
__device__ __forceinline__ void bucket_pass_lds(BktShared& S, const BktIO<P>& io, uint32_t m, int shift) {
  constexpr int rb = kBktMaxRB;  // digits (sub >> shift) & 511: bits above L are zero
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int R = 1 << rb;
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
  const uint32_t base = bkt_excl_scan(t, S.wsum, lane, wave);
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

// Phase-2 dispatch order: buckets that outgrow the LDS image (hot features: their block walks the
// bucket through global scratch, several times longer) first, so they start with the first wave of
// blocks instead of forming the kernel's tail; then the rest in bucket order.  One block.
__global__ __launch_bounds__(kBB) void k_bucket_order(const uint32_t* __restrict__ btot, int nb,
                                                      uint32_t* __restrict__ order) {
  __shared__ uint32_t wsum[kBW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t carry = 0;  // block-uniform
  for (int pass = 0; pass < 2; ++pass) {
    for (int b0 = 0; b0 < nb; b0 += kBB) {
      const int b = b0 + tid;
      const bool big = b < nb && btot[b] > (uint32_t)kBktCap / 2;  // the largest first (c4: 16K image)
      const uint32_t f = (b < nb && (pass == 0 ? big : !big)) ? 1u : 0u;
      const uint32_t pre = bkt_excl_scan(f, wsum, lane, wave);
      if (f) order[carry + pre] = (uint32_t)b;
      uint32_t t = 0;
#pragma unroll
      for (int w = 0; w < kBW; ++w) t += wsum[w];
      lds_barrier();
      carry += t;
    }
  }
}

// Phase 2: block b sorts bucket b (btot[b] entries starting at the sum of the buckets below it).
template <class P>
__global__ __launch_bounds__(kBB) void k_bucket_sort(const uint32_t* __restrict__ keys_in, const P* __restrict__ vals_in,
                                                     uint32_t* __restrict__ keys_out, P* __restrict__ vals_out,
                                                     const uint32_t* __restrict__ btot, int L,
                                                     uint2* __restrict__ scratch,
                                                     const uint32_t* __restrict__ order) {
  __shared__ BktShared S;
  const int b = order ? (int)order[blockIdx.x] : (int)blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t acc = 0;
  for (int i = tid; i < b; i += kBB) acc += btot[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) S.wsum[wave] = acc;
  lds_barrier();
  uint32_t start = 0;
#pragma unroll
  for (int w = 0; w < kBW; ++w) start += S.wsum[w];
  const uint32_t m = btot[b];
  if (m == 0) return;  // block-uniform
  lds_barrier();       // wsum is reused by the scans
  BktIO<P> io;
  io.keys = keys_in + start;
  io.vals = vals_in + start;
  io.okeys = keys_out + start;
  io.ovals = vals_out + start;
  io.scratch = scratch + start;
  io.hi = (uint32_t)b << L;
  io.lmask = (1u << L) - 1u;
  io.ib = 32 - L;
  const int rb0 = L <= kBktMaxRB ? L : L / 2, rb1 = L - rb0;
  // the packed word holds the index in ib = 32 - L bits: 15 at c3's L = 17, 14 at c4's L = 18
  const uint32_t cap = min((uint32_t)kBktCap, 1u << min(io.ib, 31));
  if (m <= cap) {
    bucket_pass_lds<true>(S, io, m, 0);
    if (L > kBktMaxRB) bucket_pass_lds<false>(S, io, m, kBktMaxRB);
    // the bucket in order in S.arr: coalesced key and payload writes, payloads gathered by index
    // from the bucket's own range
    const uint32_t imask = (io.ib >= 32) ? 0xFFFFFFFFu : ((1u << io.ib) - 1u);
    constexpr int U = 4;
    for (uint32_t j0 = 0; j0 < m; j0 += U * kBB) {
      uint32_t w[U];
      P pv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + u * kBB + tid;
        w[u] = j < m ? S.arr[j] : 0u;
        if (j < m) pv[u] = io.vals[w[u] & imask];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + u * kBB + tid;
        if (j < m) {
          io.okeys[j] = io.hi | (w[u] >> io.ib);
          io.ovals[j] = pv[u];
        }
      }
    }
  } else if (rb1 == 0) {
    bucket_pass<kSrcKeys, kDstOut, false>(S, io, m, 0, L);
  } else {
    bucket_pass<kSrcKeys, kDstScratch, true>(S, io, m, 0, rb0);
    bucket_pass<kSrcScratch, kDstOut, true>(S, io, m, rb0, rb1);
  }
}

}  // namespace

void SortWork::ensure(int64_t n) {
  if (n <= cap) return;
  const int64_t c = n + n / 8 + 4096;
  keys_a.ensure(sizeof(uint32_t) * c);
  keys_b.ensure(sizeof(uint32_t) * c);
  vals_a.ensure(sizeof(uint64_t) * c);  // payloads up to 8 bytes
  vals_b.ensure(sizeof(uint64_t) * c);
  const int64_t ntiles = (c + kTile - 1) / kTile;
  counts.ensure(sizeof(uint32_t) * kMaxRadix * ntiles);
  digit_tot.ensure(sizeof(uint32_t) * kMaxRadix * 2);  // digit totals + the bucket sort's block order
  cap = c;
}

template <class P, int RB>
static void radix_pass_impl(const uint32_t* kin, const P* vin, uint32_t* ko, P* vo, int64_t n, int shift,
                       SortWork& w, int64_t ntiles, hipStream_t st) {
  hipLaunchKernelGGL(k_radix_count<RB>, dim3((unsigned)(FM_SORT_CXCD ? blocks_for_tiles(ntiles) : ntiles)), dim3(kCntBlock), 0, st, kin, n, shift,
                     w.counts.as<uint32_t>(), ntiles);
  if (FM_SORT_SMALLBLK)
    hipLaunchKernelGGL(k_radix_scan_rows_w, dim3((1u << RB) / 4), dim3(256), 0, st, w.counts.as<uint32_t>(), ntiles,
                       w.digit_tot.as<uint32_t>(), 1 << RB);
  else
    hipLaunchKernelGGL(k_radix_scan_rows, dim3(1u << RB), dim3(kBlock), 0, st, w.counts.as<uint32_t>(), ntiles,
                       w.digit_tot.as<uint32_t>());
  hipLaunchKernelGGL((k_radix_scatter<P, RB>), dim3((unsigned)blocks_for_tiles(ntiles)), dim3(kBlock), 0, st, kin,
                     vin, ko, vo, n, shift, w.counts.as<uint32_t>(), w.digit_tot.as<uint32_t>(), ntiles);
  FM_HIP_CHECK(hipGetLastError());
}

template <class P, int RB>
static void radix_pass(const uint32_t* kin, const P* vin, uint32_t* ko, P* vo, int64_t n, int shift,
                       SortWork& w, int64_t ntiles, hipStream_t st) {
  if constexpr ((1 << RB) >= kBlock) {
    radix_pass_impl<P, RB>(kin, vin, ko, vo, n, shift, w, ntiles, st);
  } else {
    FM_REQUIRE(false, "sort digit narrower than the block");
  }
}

// Digit width: the fewest passes of at most FM_SORT_MAXRB bits, spread evenly (27-bit feature
// slots: 3 passes of 9 bits), never narrower than kMinRB bits.
inline int digit_bits(int key_bits, int* passes) {
  const int kb = key_bits < 1 ? 1 : key_bits;
  int p = (kb + FM_SORT_MAXRB - 1) / FM_SORT_MAXRB;
  int rb = (kb + p - 1) / p;
  if (rb < kMinRB) rb = kMinRB;
  p = (kb + rb - 1) / rb;
  *passes = p;
  return rb;
}

// Top-bit count of the bucket sort (0: the LSD passes).  Buckets average n / 2^H entries (about
// 5K - 10K, below the LDS image of kBktCap); the low L = key_bits - H bits take one or two in-bucket
// passes of <= 9 bits.  Needs a payload array (the index payload of radix_sort_pairs stays LSD) and
// keys from bit 0.
#ifndef FM_SORT_BUCKET
#define FM_SORT_BUCKET 0  // default off until the GPU A/B lands (FM_SORT_BUCKET=1 at run time switches it on)
#endif
#ifndef FM_SORT_BUCKET_MIN
#define FM_SORT_BUCKET_MIN (1 << 20)
#endif
static int bucket_hi_bits(int64_t n, int key_bits, int lo_bit, bool has_vals) {
  const char* env = getenv("FM_SORT_BUCKET");  // read per call: tests and A/B runs switch it
  const bool on = env ? atoi(env) != 0 : FM_SORT_BUCKET != 0;
  const char* env_min = getenv("FM_SORT_BUCKET_MIN");
  const int64_t min_n = env_min ? atoll(env_min) : (int64_t)FM_SORT_BUCKET_MIN;
  if (!on || !has_vals || lo_bit != 0 || n < min_n || n < 1) return 0;
  if (key_bits < 12 || key_bits > 10 + 2 * kBktMaxRB) return 0;
  const int H = (n / 512 > 8192 || key_bits - 9 > 2 * kBktMaxRB) ? 10 : 9;
  return key_bits - H >= 1 ? H : 0;
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
  // the count kernel reads keys as uint4 when the tile is full: needs 16-byte alignment
  const bool aligned = (reinterpret_cast<uintptr_t>(keys_in) & 15u) == 0;
  const int H = bucket_hi_bits(n, key_bits, lo_bit, vals_in != nullptr);
  if (H > 0) {
    // phase 1: one pass on the top H bits into kbuf[0]; phase 2: one block per bucket
    const int L = key_bits - H;
    if (!aligned) {
      FM_HIP_CHECK(hipMemcpyAsync(kbuf[1], keys_in, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, st));
      kin = kbuf[1];
    }
    if (H == 9)
      radix_pass<P, 9>(kin, vin, kbuf[0], vbuf[0], n, L, w, ntiles, st);
    else
      radix_pass<P, 10>(kin, vin, kbuf[0], vbuf[0], n, L, w, ntiles, st);
    w.scratch.ensure(sizeof(uint2) * w.cap);  // {sub, idx} of oversized buckets, only on this path
    uint32_t* ko = final_keys ? final_keys : kbuf[1];
    P* vo = final_vals ? final_vals : vbuf[1];
    // the bucket order lives past the digit totals (kMaxRadix words each)
    uint32_t* order = w.digit_tot.as<uint32_t>() + kMaxRadix;
    hipLaunchKernelGGL(k_bucket_order, dim3(1), dim3(kBB), 0, st, w.digit_tot.as<uint32_t>(), 1 << H, order);
    hipLaunchKernelGGL(k_bucket_sort<P>, dim3(1u << H), dim3(kBB), 0, st, kbuf[0], vbuf[0], ko, vo,
                       w.digit_tot.as<uint32_t>(), L, w.scratch.as<uint2>(), (const uint32_t*)order);
    FM_HIP_CHECK(hipGetLastError());
    *keys_out = ko;
    *vals_out = vo;
    return;
  }
  for (int p = 0; p < passes; ++p) {
    const int shift = lo_bit + rb * p;
    if (p == 0 && !aligned) {
      FM_HIP_CHECK(hipMemcpyAsync(kbuf[1], keys_in, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, st));
      kin = kbuf[1];
    }
    const bool last = p == passes - 1 && final_keys != nullptr;
    uint32_t* ko = last ? final_keys : kbuf[which];
    P* vo = last ? final_vals : vbuf[which];
    switch (rb) {
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
