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
//   chunk   : one 256-thread block per 16 tiles x 256 digits, exclusive scan down each digit
//             -> counts, chunk sums
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

// the digits at most / at least (27-bit feature slots: 3 passes of 9 bits; 7- and 8-bit digits, 4
// passes at c3, measured slower in the step: DESIGN.md §5)
constexpr int kMaxRB = 10;
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

// Tile of a block: keys [base, end) of it, and its row in the per-tile digit counts.
struct TileGeo {
  int64_t tile, base, end;
};

__device__ __forceinline__ bool tile_geo(TileGeo& g, int64_t n, int64_t ntiles) {
  g.tile = tile_of_block(ntiles);
  if (g.tile >= ntiles) return false;
  g.base = g.tile * kTile;
  g.end = n;
  return true;
}

template <int RB>
__global__ __launch_bounds__(kBlock) void k_radix_count(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                        uint32_t* __restrict__ counts, int64_t ntiles, bool vec) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  __shared__ uint32_t hist[R];
  TileGeo g;
  if (!tile_geo(g, n, ntiles)) return;  // block-uniform
  const int64_t base = g.base;
  // the tile's keys are loaded first, all together (from clamped addresses: a guarded load waits
  // out its round trip before the next is issued), and in flight while the histogram is cleared;
  // uint4 reads of whole tiles when the keys are 16-byte aligned (a split view of a dataset starts
  // anywhere)
  constexpr int NV = kTile / (4 * kBlock), NS = kTile / kBlock;
  const bool wide = vec && base + kTile <= g.end;  // block-uniform
  uint4 q[NV];
  uint32_t kk[NS];
  if (wide) {
    const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
    for (int i = 0; i < NV; ++i) q[i] = k4[i * kBlock + threadIdx.x];
  } else {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
      kk[i] = keys[idx < g.end ? idx : g.end - 1];
    }
  }
  for (int d = threadIdx.x; d < R; d += kBlock) hist[d] = 0;
  lds_barrier();
  if (wide) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      atomicAdd(&hist[(q[i].x >> shift) & M], 1u);
      atomicAdd(&hist[(q[i].y >> shift) & M], 1u);
      atomicAdd(&hist[(q[i].z >> shift) & M], 1u);
      atomicAdd(&hist[(q[i].w >> shift) & M], 1u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NS; ++i)
      if (base + (int64_t)i * kBlock + threadIdx.x < g.end) atomicAdd(&hist[(kk[i] >> shift) & M], 1u);
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

// The count scan, level 1: block (c, slice) takes tiles [16 c, 16 c + 16) of the 256 digits of its
// slice, one digit per thread, and replaces each tile's counts by the digit's exclusive prefix
// within the chunk; the chunk's sums -> csum[c][digit].  256-thread blocks find room on a CU beside
// the step's and the sort's blocks sooner than the 512-thread block per chunk of round 4 (c3
// 0.964-0.967 ms per step against 0.967-0.971, c2 0.167-0.173 against 0.170-0.176, c5 within the
// noise; three alternating reps, profiles/r05_b/ab)
template <int RB>
__global__ __launch_bounds__(256) void k_radix_chunk_scan(uint32_t* __restrict__ counts, int64_t ntiles,
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
// the digit's exclusive prefix over chunks, digit_tot[d] = the digit's total.
__global__ __launch_bounds__(256) void k_radix_chunk_top(uint32_t* __restrict__ csum, int64_t nchunks, int R,
                                                         uint32_t* __restrict__ digit_tot) {
  constexpr int kDig = 32, kSl = 8;
  __shared__ uint32_t part[kSl][kDig];
  const int dl = threadIdx.x % kDig, sl = threadIdx.x / kDig;
  const int d = blockIdx.x * kDig + dl;
  const int64_t nch = nchunks;
  const int64_t per = (nch + kSl - 1) / kSl;
  const int64_t c0 = min(nch, sl * per), c1 = min(nch, c0 + per);
  // kTopLd chunks' sums loaded together per round trip (clamped addresses), in chunk order
  constexpr int kTopLd = 8;
  uint32_t s = 0;
  for (int64_t cb = c0; cb < c1; cb += kTopLd) {
    uint32_t x[kTopLd];
#pragma unroll
    for (int j = 0; j < kTopLd; ++j) x[j] = csum[(cb + j < c1 ? cb + j : c1 - 1) * R + d];
#pragma unroll
    for (int j = 0; j < kTopLd; ++j) s += cb + j < c1 ? x[j] : 0u;
  }
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
    digit_tot[d] = run;
  }
  __syncthreads();
  uint32_t run = part[sl][dl];
  for (int64_t cb = c0; cb < c1; cb += kTopLd) {
    uint32_t x[kTopLd];
#pragma unroll
    for (int j = 0; j < kTopLd; ++j) x[j] = csum[(cb + j < c1 ? cb + j : c1 - 1) * R + d];
#pragma unroll
    for (int j = 0; j < kTopLd; ++j) {
      if (cb + j < c1) csum[(cb + j) * R + d] = run;
      run += cb + j < c1 ? x[j] : 0u;
    }
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

// IMPLICIT: the payload is each key's index (vals_in is null, the first pass of a sort); a template
// parameter, so every instantiation issues a fixed number of loads and the block scan waits only
// for its own
template <class P, int RB, bool IMPLICIT>
__global__ __launch_bounds__(kBlock) void k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                          const P* __restrict__ vals_in,
                                                          uint32_t* __restrict__ keys_out,
                                                          P* __restrict__ vals_out, int64_t n,
                                                          int shift, const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ csum,
                                                          const uint32_t* __restrict__ digit_tot,
                                                          int64_t ntiles) {
  constexpr int R = 1 << RB;
  constexpr uint32_t M = R - 1;
  constexpr int D = digits_per_thread<R>();  // digits per thread in the block scans
  const bool own = R >= kBlock || (int)threadIdx.x * D < R;  // this thread holds digits in the block scans (all of
  // them when R >= kBlock: no branch, so the digit loads below are issued where they stand)
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
  if (!tile_geo(g, n, ntiles)) return;  // block-uniform
  const int64_t tile = g.tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile_base = g.base;
  const int64_t wbase = tile_base + (int64_t)wave * (kTile / kWaves);
  uint32_t my_key[kRounds], my_rank[kRounds];
  P my_val[kRounds];
  // the digit offsets' loads first (the block scan below waits for them; clamped addresses, no
  // branch around them), then the tile's, in flight through the scan
  uint32_t tot[D], pcs[D], pct[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const int d = own ? tid * D + i : 0;
    tot[i] = digit_tot[d];
    pcs[i] = csum[(tile / kChunk) * R + d];
    pct[i] = counts[tile * R + d];
  }
  // (from clamped addresses, unguarded: a lane past the end loads the last key and is left out of
  // every ballot and store below by its own validity test)
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    my_key[r] = keys_in[idx < g.end ? idx : g.end - 1];
  }
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t idx = wbase + (int64_t)r * 64 + lane;
    if constexpr (IMPLICIT) my_val[r] = P{};  // made at the staging store
    else my_val[r] = vals_in[idx < g.end ? idx : g.end - 1];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the loads above in this order, ahead of the scan
#pragma unroll
  for (int w = 0; w < kWaves; ++w)
    for (int d = tid; d < R; d += kBlock) wave_hist[w][d] = 0;

  // global base of (digit, this tile): exclusive scan of digit totals + the tile's running prefix
  // of the digit (its chunk's prefix + its own prefix within the chunk)
  {
    uint32_t v[D];
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = own ? tot[i] : 0u;
    block_excl_scan<D>(v, wsum, lane, wave);
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (own) glob_off[tid * D + i] = v[i] + (pcs[i] + pct[i]);
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
      s_vals[pos] = IMPLICIT ? implicit_payload<P>(wbase + (int64_t)r * 64 + lane) : my_val[r];
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
  digit_tot.ensure(sizeof(uint32_t) * kMaxRadix);  // digit totals
  cap = c;
}

template <class P, int RB>
static void radix_pass_impl(const uint32_t* kin, const P* vin, uint32_t* ko, P* vo, int64_t n, int shift,
                       SortWork& w, int64_t ntiles, hipStream_t st) {
  uint32_t* counts = w.counts.as<uint32_t>();
  uint32_t* csum = counts + (ntiles + 1) * (int64_t(1) << RB);
  const int64_t nchunks = (ntiles + kChunk - 1) / kChunk;
  // (count and chunk scan fused into one kernel, a block walking its chunk's 16 tiles, measured
  // slower: 0.349 against 0.317 ms standalone)
  const bool vec = (reinterpret_cast<uintptr_t>(kin) & 15u) == 0;
  hipLaunchKernelGGL(k_radix_count<RB>, dim3((unsigned)blocks_for_tiles(ntiles)), dim3(kBlock), 0, st, kin, n, shift,
                     counts, ntiles, vec);
  // (one launch for the whole count scan of a small sort -- 32 digits per 256-thread block, 8 slices
  // of the tiles per digit -- measured 0.185-0.188 against 0.170-0.172 ms per c2 step and 0.188-0.190
  // against 0.190 at c5, three alternating reps, profiles/r05_d/ab: not taken)
  constexpr int TB = (1 << RB) < 256 ? (1 << RB) : 256;
  hipLaunchKernelGGL(k_radix_chunk_scan<RB>, dim3((unsigned)(nchunks * ((1 << RB) / TB))), dim3(TB), 0, st, counts,
                     ntiles, csum);
  hipLaunchKernelGGL(k_radix_chunk_top, dim3((1u << RB) / 32), dim3(256), 0, st, csum, nchunks, 1 << RB,
                     w.digit_tot.as<uint32_t>());
  auto scatter = vin ? k_radix_scatter<P, RB, false> : k_radix_scatter<P, RB, true>;
  hipLaunchKernelGGL(scatter, dim3((unsigned)blocks_for_tiles(ntiles)), dim3(kBlock), 0, st, kin, vin, ko, vo, n,
                     shift, (const uint32_t*)counts, (const uint32_t*)csum,
                     (const uint32_t*)w.digit_tot.as<uint32_t>(), ntiles);
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
  int p = (kb + kMaxRB - 1) / kMaxRB;
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
