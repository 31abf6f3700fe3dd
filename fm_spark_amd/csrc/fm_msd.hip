// Two-level grouping of a batch's entries by feature slot: the reference's groupBy featureId
// (FactorizationMachinesSGD.scala:148-155, the VectorSum window of FactorizationMachinesModel.scala:191),
// stable, so that every per-feature sum downstream runs in CSR order and the step stays bitwise
// reproducible -- and bitwise the step of the three LSD passes (fm_sort.hip): a stable sort by slot
// has one result.
//
//   level 1 (fm_batch_prepare, side stream): ONE stable radix pass on the slot's top hb bits
//            (fm_sort.hip's count / scan / scatter kernels): the entries grouped into 2^hb buckets of
//            about 8K-30K entries, the bucket sizes kept with the batch;
//   level 2 (k_msd_buckets): one 1024-thread block per bucket sorts the bucket by the low sh bits in
//            LDS (a 128-KB image of 32K words {low bits, local index}: 1-2 ballot-ranked passes of
//            <= 9 bits), then either writes the sorted bucket back (the unfused step's view), or -- the
//            fused step, at the step on the main stream -- finds the runs, keeps only the runs of two or
//            more entries (the multi view, compacted across buckets by a decoupled look-back on
//            per-bucket {multi, singleton} counts) and tags each multi run's row with the step's epoch.
//
// What it replaces per c3 batch (10.2M entries, 27-bit slots): the second and third LSD passes (each
// a count, two scans and a scatter whose digit runs of 8 entries cost about 0.5 L2 requests per
// entry) and the split's count / scan / scatter passes over the sorted view.  Level 2 reads each
// entry once, coalesced, and writes only the multi entries.
//
// Buckets larger than the LDS image (a hot slot and its bucket mates, or adversarial input) take a
// slower path in the same block: stable LSD passes through global memory in 32K-entry pieces.
#include "fm_device.h"
#include "fm_internal.h"

namespace fmhip {

namespace {

constexpr int kMB = 1024;               // threads per bucket block
constexpr int kMW = kMB / 64;           // 16 waves
constexpr int kMR = 32;                 // entries per lane
constexpr int kMCap = kMB * kMR;        // 32768 entries sorted in LDS
constexpr int kMIdx = 15;               // local index bits of an LDS word
static_assert((1 << kMIdx) == kMCap, "the local index must address the LDS image");
constexpr int kMLow = 32 - kMIdx;       // low slot bits an LDS word carries (17)
constexpr int kMDig = 9;                // digit bits per pass at most
constexpr int kMRad = 1 << kMDig;
constexpr uint32_t kNoWord = 0xFFFFFFFFu;  // a position past the bucket's end: sorts last
constexpr unsigned kSpinMax = 1u << 22;    // look-back polls before giving up (never reached)
constexpr int kPresortGrid = 32;           // blocks of k_msd_presort (most exit at once: no oversized bucket)

struct MsdLds {
  uint32_t w[kMCap];        // the bucket's words, then the payload exchange
  uint16_t h[kMW][kMRad];   // per-wave digit counts -> offsets
  uint32_t ds[kMRad];       // digit starts within the block
  uint32_t run[kMRad];      // oversized bucket: running digit offsets over its pieces
  uint32_t gh[2][kMRad];    // oversized bucket: digit histograms of its passes
  uint32_t ws[kMW];         // wave sums
  uint32_t wt[kMW];         // wave totals of the multi entries
  uint32_t misc[4];
  unsigned long long base[2];
};

struct MsdArgs {
  const uint32_t* keys;     // level-1 output grouped by bucket (or the batch itself: one bucket)
  const uint2* vals;
  uint32_t* keys_a;         // oversized buckets: the input region (may be overwritten) and a second
  uint2* vals_a;            // buffer of the same size, ping-pong
  uint32_t* keys_b;
  uint2* vals_b;
  const uint32_t* btot;     // [nbk] bucket sizes; null: one bucket of n1 entries
  int64_t n1;
  int nbk, sh;
  uint32_t* okeys;          // sorted view (full) / multi view (split)
  uint2* ovals;
  int64_t* n_out;           // split: {multi entries, singleton runs}
  unsigned long long* status;  // split: [nbk] look-back words, then the ticket and an error word
  TableView T;              // split: multi tags (tag != 0)
  int32_t epoch;
  int tag;
};

// v unchanged, but opaque to the compiler: a digit or LDS address computed from it before a barrier is
// recomputed after it instead of being kept live across it (32 of each per lane would spill)
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

// A buffer resource over [p, p + bytes) built from wave-uniform values (readfirstlane: the compiler
// cannot prove a value read from LDS uniform, and would wrap every buffer op in a waterfall loop,
// cdna_hip_programming.md T20): loads through it take a 32-bit per-lane offset (one VGPR, not a
// 64-bit address per load in flight) and read 0 past the end, so no clamping.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t ld32(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// exclusive scan over the block's 1024 threads (one value each); the total -> *tot
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, MsdLds& S, int lane, int wave, uint32_t* tot) {
  const uint32_t incl = wave_incl_scan(v, lane);
  if (lane == 63) S.ws[wave] = incl;
  lds_barrier();
  uint32_t pre = 0, t = 0;
#pragma unroll
  for (int w = 0; w < kMW; ++w) {
    const uint32_t x = S.ws[w];
    pre += w < wave ? x : 0u;
    t += x;
  }
  lds_barrier();
  *tot = t;
  return pre + incl - v;
}

// The block's words: wave w holds positions [w nr 64, (w + 1) nr 64), nr = ceil(n / 1024) rounds of 64 (so
// the work follows the bucket's size, not the LDS image's), positions >= n hold kNoWord.
// One stable counting pass over them (position order: wave, round, lane) by the
// digit (word >> sh) & (2^nb - 1), in two sweeps so that no per-word rank is held in registers:
//   block_offsets: the per-wave digit counts (16-bit counters, two per 32-bit LDS word, LDS atomics)
//                  -> S.h[wave][d] = where wave `wave`'s first word of digit d goes (start + the block's
//                  digit start when `absolute`, else the offset within the digit); the digit total of
//                  thread d (< 2^nb) -> *dtot
//   place        : per round, the word's rank among its wave's equal digits (wave64 ballots) added to
//                  the wave's running counter, which the round's first lane of the digit advances.
__device__ __forceinline__ void block_offsets(const uint32_t (&wd)[kMR], int nr, int sh, int nb, bool absolute,
                                              MsdLds& S, int lane, int wave, uint32_t* dtot) {
  const int R = 1 << nb;
  const uint32_t M = (uint32_t)R - 1;
  uint32_t* h32 = reinterpret_cast<uint32_t*>(&S.h[0][0]);
  for (int i = threadIdx.x; i < kMW * kMRad / 2; i += kMB) h32[i] = 0;
  lds_barrier();
  uint32_t* hw = h32 + wave * (kMRad / 2);
#pragma unroll
  for (int r = 0; r < kMR; ++r) {
    if (r < nr) {  // block-uniform
      const uint32_t d = (wd[r] >> sh) & M;
      atomicAdd(&hw[d >> 1], 1u << ((d & 1u) * 16u));  // <= 2048 per wave and digit: no carry
    }
  }
  lds_barrier();
  const int tid = threadIdx.x;
  uint32_t acc = 0;
  if (tid < R) {
#pragma unroll
    for (int w = 0; w < kMW; ++w) {
      const uint32_t c = S.h[w][tid];
      S.h[w][tid] = (uint16_t)acc;
      acc += c;
    }
  }
  uint32_t t;
  const uint32_t ex = block_excl_scan(tid < R ? acc : 0u, S, lane, wave, &t);
  if (absolute && tid < R) {
#pragma unroll
    for (int w = 0; w < kMW; ++w) S.h[w][tid] = (uint16_t)(S.h[w][tid] + ex);  // positions < 2^15
  }
  *dtot = acc;
  lds_barrier();
}

__device__ __forceinline__ uint32_t place(uint32_t w, int sh, uint32_t M, MsdLds& S, int wave, uint64_t lt) {
  const uint32_t d = (w >> sh) & M;
  // all kMDig ballots for every width: a digit's bits above nb are 0 in every lane, so their ballots
  // keep every peer (no branch per bit)
  uint64_t peers = ~0ull;
#pragma unroll
  for (int b = 0; b < kMDig; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  const uint32_t below = (uint32_t)__popcll(peers & lt);
  const uint32_t cnt = (uint32_t)__popcll(peers);
  const uint32_t prev = S.h[wave][d];
  __builtin_amdgcn_wave_barrier();
  if (below == 0) S.h[wave][d] = (uint16_t)(prev + cnt);
  __builtin_amdgcn_wave_barrier();
  return prev + below;
}

// one LDS pass: the words re-ordered stably by their digit, read back in position order
__device__ __forceinline__ void lds_pass(uint32_t (&wd)[kMR], int nr, int sh, int nb, MsdLds& S, uint64_t lt,
                                         int lane, int wave) {
  uint32_t dt;
  block_offsets(wd, nr, sh, nb, true, S, lane, wave, &dt);
  const uint32_t M = (1u << nb) - 1;
#pragma unroll
  for (int r = 0; r < kMR; ++r) {
    if (r < nr) {
      const uint32_t w = opaque(wd[r]);  // the digits of block_offsets recomputed, not kept live
      S.w[place(w, sh, M, S, wave, lt)] = w;
    }
  }
  lds_barrier();
#pragma unroll
  for (int r = 0; r < kMR; ++r)
    if (r < nr) wd[r] = S.w[(wave * nr + r) * 64 + lane];
}

// the passes' digit widths over sh bits: ceil(sh / 9) passes, as even as possible
__device__ __forceinline__ int npasses(int sh) { return (sh + kMDig - 1) / kMDig; }
__device__ __forceinline__ int pass_bits(int sh, int P, int i) { return sh / P + (i < sh % P ? 1 : 0); }

// global stores of this block made visible to its own later loads (another wave may hold the lines
// in this CU's L1): every wave drains its stores, one agent-scope acquire drops the L1
__device__ __forceinline__ void block_global_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// The bucket's multi base and singleton base over the buckets before it: decoupled look-back on
// the per-bucket words {flag: 1 = own counts, 2 = inclusive prefix; multi (31 bits); singles (31
// bits)}, stored and loaded as single 8-byte agent-scope atomics (the value is the flag: no fence,
// cdna_hip_programming.md §6 Guideline 16 R2).  Buckets are taken in ticket order, so every bucket a
// block waits for has a running (or finished) block that publishes without waiting.  Wave 0 only.
__device__ __forceinline__ void look_back(const MsdArgs& a, int b, uint32_t nm, uint32_t ns, MsdLds& S, int lane) {
  unsigned long long accm = 0, accs = 0;
  if (b > 0) {
    int64_t j0 = b - 1;
    unsigned spins = 0;
    while (true) {
      const int64_t j = j0 - lane;
      const unsigned long long v =
          j >= 0 ? __hip_atomic_load(&a.status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (2ull << 62);
      const unsigned f = (unsigned)(v >> 62);
      const uint64_t inc = __ballot(f == 2u);
      const int stop = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
      const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1ull);
      if (__ballot(f == 0u) & need) {
        if (++spins > kSpinMax) {  // never expected: the kernel ends with a wrong base, flagged
          if (lane == 0)
            __hip_atomic_store(&a.status[a.nbk + 1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      const bool use = lane <= stop;
      accm += wave_sum<unsigned long long>(use ? (v >> 31) & 0x7FFFFFFFull : 0ull);
      accs += wave_sum<unsigned long long>(use ? v & 0x7FFFFFFFull : 0ull);
      if (stop < 64) break;
      j0 -= 64;
    }
    if (lane == 0)
      __hip_atomic_store(&a.status[b], (2ull << 62) | ((accm + nm) << 31) | (accs + ns), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) {
    S.base[0] = accm;
    S.base[1] = accs;
    if (b == a.nbk - 1) {
      a.n_out[0] = (int64_t)(accm + nm);
      a.n_out[1] = (int64_t)(accs + ns);
    }
  }
}

__device__ __forceinline__ void publish_own(const MsdArgs& a, int b, uint32_t nm, uint32_t ns) {
  __hip_atomic_store(&a.status[b],
                     ((b == 0 ? 2ull : 1ull) << 62) | ((unsigned long long)nm << 31) | (unsigned long long)ns,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the block's counts summed (nm, ns per thread) -> S.misc[0..1]; S.wt[wave] = the wave's multi count
__device__ __forceinline__ void block_counts(uint32_t nm, uint32_t ns, MsdLds& S, int lane, int wave) {
  const uint32_t wm = wave_sum<uint32_t>(nm), wsn = wave_sum<uint32_t>(ns);
  if (lane == 0) {
    S.wt[wave] = wm;
    S.ws[wave] = wsn;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    uint32_t a = 0, c = 0;
    for (int w = 0; w < kMW; ++w) {
      a += S.wt[w];
      c += S.ws[w];
    }
    S.misc[0] = a;
    S.misc[1] = c;
  }
  lds_barrier();
}

// multi tags of the runs opening at this thread's tagged positions (keys[r] its slots): the rows'
// t words are read for all positions of a group before any is written, unconditionally (a row
// without a tag reads row 0's word: one shared line), so the loads go out together
template <int G>
__device__ __forceinline__ void write_tags(const TableView& T, int32_t epoch, const uint32_t (&key)[G], uint32_t tag) {
  int32_t tv[G];
#pragma unroll
  for (int r = 0; r < G; ++r) tv[r] = T.hdr((tag >> r) & 1u ? key[r] : 0u)->t;
#pragma unroll
  for (int r = 0; r < G; ++r)
    if ((tag >> r) & 1u) T.hdr(key[r])->t = multi_tag(epoch, tv[r] >= 0);
}

template <bool SPLIT>
__device__ void bucket_small(const MsdArgs& a, MsdLds& S, int b, int64_t base, int n, uint32_t hi, uint32_t lowmask,
                             int lane, int wave, uint64_t lt) {
  const int nr = (n + kMB - 1) / kMB;  // rounds per wave (block-uniform)
  const int w0 = wave * nr * 64;      // the wave's first position
  // the bucket's keys and payloads through buffer resources (32-bit offsets, 0 past the end)
  const __amdgpu_buffer_rsrc_t kr = rsrc_of(a.keys + base, (uint32_t)n * 4u);
  const __amdgpu_buffer_rsrc_t vr = rsrc_of(a.vals + base, (uint32_t)n * 8u);
  uint32_t wd[kMR];
#pragma unroll
  for (int r = 0; r < kMR; ++r) {
    if (r < nr) {
      const int q = w0 + r * 64 + lane;
      const uint32_t k = ld32(kr, (uint32_t)q * 4u);
      wd[r] = q < n ? ((k & lowmask) << kMIdx) | (uint32_t)q : kNoWord;
    } else {
      wd[r] = kNoWord;
    }
  }
  const int sh = a.sh;
  const int P = npasses(sh);
  int done = 0;
  for (int i = 0; i < P; ++i) {
    const int nb = pass_bits(sh, P, i);
    lds_pass(wd, nr, kMIdx + done, nb, S, lt, lane, wave);
    done += nb;
  }
  if (P == 0) {
#pragma unroll
    for (int r = 0; r < kMR; ++r)
      if (r < nr) S.w[w0 + r * 64 + lane] = wd[r];
  }
  lds_barrier();
  // runs: the sorted words' neighbours from the LDS image
  uint32_t mult = 0, first = 0;
#pragma unroll
  for (int r = 0; r < kMR; ++r) {
    if (r < nr) {
      const int p = w0 + r * 64 + lane;
      const uint32_t lk = opaque(wd[r]) >> kMIdx;
      const uint32_t pk = S.w[p > 0 ? p - 1 : 0] >> kMIdx;
      const uint32_t nk = S.w[p + 1 < kMCap ? p + 1 : p] >> kMIdx;
      const bool valid = p < n;
      const bool hp = p > 0 && pk == lk, hn = p + 1 < n && nk == lk;
      mult |= (uint32_t)(valid && (hp || hn)) << r;
      first |= (uint32_t)(valid && !hp) << r;
    }
  }
  if (SPLIT) {
    block_counts((uint32_t)__popc(mult), (uint32_t)__popc(first & ~mult), S, lane, wave);
    const uint32_t nm = S.misc[0], ns = S.misc[1];
    if (threadIdx.x == 0) publish_own(a, b, nm, ns);
    if (wave == 0) look_back(a, b, nm, ns, S, lane);
    if (a.tag) {
      const uint32_t tg = mult & first;
#pragma unroll
      for (int g = 0; g < kMR; g += 8) {
        if (g < nr) {
          uint32_t key[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) key[r] = hi | (opaque(wd[g + r]) >> kMIdx);
          write_tags<8>(a.T, a.epoch, key, tg >> g);
        }
      }
    }
  }
  lds_barrier();  // the neighbour reads done (and the look-back's base posted)
  // payload: the samples, then the x bits, each through the LDS image by local index
  if (n == 0) return;  // block-uniform (an empty bucket has published its counts)
  uint32_t sm[kMR];
  for (int c = 0; c < 2; ++c) {
#pragma unroll
    for (int h = 0; h < kMR; h += 8) {
      if (h < nr) {
        uint32_t u[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int q = w0 + (h + r) * 64 + lane;
          u[r] = ld32(vr, (uint32_t)q * 8u + 4u * c);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int q = w0 + (h + r) * 64 + lane;
          if (h + r < nr && q < n) S.w[q] = u[r];
        }
      }
    }
    lds_barrier();
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < kMR; ++r)
        if (r < nr) sm[r] = S.w[opaque(wd[r]) & (kMCap - 1)];
      lds_barrier();
    }
  }
  if (!SPLIT) {
    uint32_t* __restrict__ ok = a.okeys + base;
    uint2* __restrict__ ov = a.ovals + base;
#pragma unroll
    for (int r = 0; r < kMR; ++r) {
      if (r < nr) {
        const int p = w0 + r * 64 + lane;
        const uint32_t w = opaque(wd[r]);
        const uint32_t x = S.w[w & (kMCap - 1)];
        if (p < n) {
          ok[p] = hi | (w >> kMIdx);
          ov[p] = make_uint2(sm[r], x);
        }
      }
    }
  } else {
    // multi entries in position order: the bucket's base, the waves before, the rounds before
    int64_t o = (int64_t)S.base[0];
#pragma unroll
    for (int w = 0; w < kMW; ++w) o += w < wave ? S.wt[w] : 0u;
#pragma unroll
    for (int r = 0; r < kMR; ++r) {
      if (r < nr) {
        const bool m = (mult >> r) & 1u;
        const uint64_t bm = __ballot(m);
        const uint32_t w = opaque(wd[r]);
        const uint32_t x = S.w[w & (kMCap - 1)];
        if (m) {
          const int64_t d = o + __popcll(bm & lt);
          a.okeys[d] = hi | (w >> kMIdx);
          a.ovals[d] = make_uint2(sm[r], x);
        }
        o += __popcll(bm);
      }
    }
  }
}

// A bucket beyond the LDS image (k_msd_presort, launched before k_msd_buckets): stable LSD passes over
// its low bits through global memory, 32K-entry pieces ranked in LDS with running digit offsets.  The
// sorted bucket ends in the input region (split: the step's multi sweeps read it there) or in the
// sorted view (full).
template <bool SPLIT>
__device__ void big_sort(const MsdArgs& a, MsdLds& S, int64_t base, int64_t n, uint32_t hi, uint32_t lowmask, int lane,
                         int wave, uint64_t lt) {
  const int tid = threadIdx.x;
  const int sh = a.sh;
  const int P = npasses(sh);
  // the digit histograms of every pass in one read of the keys
  for (int i = tid; i < 2 * kMRad; i += kMB) (&S.gh[0][0])[i] = 0;
  lds_barrier();
  for (int64_t q0 = 0; q0 < n; q0 += kMB) {
    const int64_t q = q0 + tid;
    if (q < n) {
      const uint32_t lk = a.keys[base + q] & lowmask;
      int done = 0;
      for (int i = 0; i < P; ++i) {
        const int nb = pass_bits(sh, P, i);
        atomicAdd(&S.gh[i][(lk >> done) & ((1u << nb) - 1)], 1u);
        done += nb;
      }
    }
  }
  lds_barrier();
  const uint32_t* sk = a.keys;
  const uint2* sv = a.vals;
  int done = 0;
  for (int i = 0; i < P; ++i) {
    const int nb = pass_bits(sh, P, i);
    const int R = 1 << nb;
    const uint32_t M = (uint32_t)R - 1;
    // split: A -> B -> A (an odd count ends in B: copied back below); full: ... -> B -> the sorted view
    const bool last_to_b = SPLIT ? (i & 1) == 0 : ((P - 1 - i) & 1) != 0;
    uint32_t* dk = last_to_b ? a.keys_b : (SPLIT ? a.keys_a : a.okeys);
    uint2* dv = last_to_b ? a.vals_b : (SPLIT ? a.vals_a : a.ovals);
    {
      uint32_t t;
      const uint32_t ex = block_excl_scan(tid < R ? S.gh[i][tid] : 0u, S, lane, wave, &t);
      if (tid < R) S.run[tid] = ex;
    }
    lds_barrier();
    for (int64_t pc = 0; pc < n; pc += kMCap) {
      const int m = (int)(n - pc < kMCap ? n - pc : kMCap);
      const int nr = (m + kMB - 1) / kMB, w0 = wave * nr * 64;
      uint32_t wd[kMR], dt;
#pragma unroll
      for (int r = 0; r < kMR; ++r) {
        const int q = w0 + r * 64 + lane;
        const uint32_t k = sk[base + pc + (q < m ? q : m - 1)];
        wd[r] = r < nr && q < m ? ((k & lowmask) << kMIdx) | (uint32_t)q : kNoWord;
      }
      block_offsets(wd, nr, kMIdx + done, nb, false, S, lane, wave, &dt);
#pragma unroll
      for (int r = 0; r < kMR; ++r) {
        if (r >= nr) continue;
        const int q = w0 + r * 64 + lane;
        const uint32_t w = opaque(wd[r]);
        const uint32_t rank = place(w, kMIdx + done, M, S, wave, lt);  // every lane: the ballots
        if (q < m) {
          const uint32_t d = (w >> (kMIdx + done)) & M;
          const int64_t dest = base + S.run[d] + rank;
          dk[dest] = hi | (w >> kMIdx);
          dv[dest] = sv[base + pc + q];
        }
      }
      lds_barrier();
      if (tid < R) S.run[tid] += dt;
      lds_barrier();
    }
    block_global_sync();
    sk = dk;
    sv = dv;
    done += nb;
  }
  // an odd pass count (split) or no pass at all (full): one copy to where the bucket is expected
  const bool copy = SPLIT ? (P & 1) != 0 : P == 0;
  if (copy) {
    uint32_t* dk = SPLIT ? a.keys_a : a.okeys;
    uint2* dv = SPLIT ? a.vals_a : a.ovals;
    for (int64_t q = tid; q < n; q += kMB) {
      dk[base + q] = sk[base + q];
      dv[base + q] = sv[base + q];
    }
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(kMB) void k_msd_presort(MsdArgs a) {
  __shared__ MsdLds S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint32_t v = tid < a.nbk ? a.btot[tid] : 0u;
  uint32_t t, nbig;
  const uint32_t st = block_excl_scan(v, S, lane, wave, &t);
  // the oversized buckets listed in bucket order (the same list in every block), in S.w, which
  // big_sort does not use; block g takes entries g, g + grid, ...
  const bool over = v > (uint32_t)kMCap;
  const uint32_t k = block_excl_scan(over ? 1u : 0u, S, lane, wave, &nbig);
  uint32_t* big = S.w;
  if (over) {
    big[3 * k] = tid;
    big[3 * k + 1] = st;
    big[3 * k + 2] = v;
  }
  lds_barrier();
  for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
    const uint32_t b = big[3 * i], base = big[3 * i + 1], n = big[3 * i + 2];
    big_sort<SPLIT>(a, S, base, n, b << a.sh, (1u << a.sh) - 1u, lane, wave, lt);
  }
}

// split mode, a bucket pre-sorted by k_msd_presort (in a.keys / a.vals): two sweeps over it in pieces
// of 8 entries per lane -- counts for the look-back, then the multi entries in order and the tags
__device__ void big_sweeps(const MsdArgs& a, MsdLds& S, int b, int64_t base, int64_t n, int lane, int wave,
                           uint64_t lt) {
  constexpr int G = 8, PW = G * 64, PC = kMB * G;
  const uint32_t* sk = a.keys;
  const uint2* sv = a.vals;
  int64_t o = 0;
  for (int sweep = 0; sweep < 2; ++sweep) {
    uint32_t nm = 0, ns = 0;
    for (int64_t pc = 0; pc < n; pc += PC) {
      uint32_t mult = 0, first = 0;
      uint32_t key[G];
#pragma unroll
      for (int r = 0; r < G; ++r) {
        const int64_t q = pc + wave * PW + r * 64 + lane;
        const int64_t qc = q < n ? q : n - 1;
        key[r] = sk[base + qc];
        const uint32_t pk = sk[base + (qc > 0 ? qc - 1 : 0)];
        const uint32_t nk = sk[base + (qc + 1 < n ? qc + 1 : qc)];
        const bool valid = q < n;
        const bool hp = q > 0 && pk == key[r], hn = q + 1 < n && nk == key[r];
        mult |= (uint32_t)(valid && (hp || hn)) << r;
        first |= (uint32_t)(valid && !hp) << r;
      }
      if (sweep == 0) {
        nm += (uint32_t)__popc(mult);
        ns += (uint32_t)__popc(first & ~mult);
        continue;
      }
      block_counts((uint32_t)__popc(mult), 0u, S, lane, wave);
      int64_t ow = o;
#pragma unroll
      for (int w = 0; w < kMW; ++w) ow += w < wave ? S.wt[w] : 0u;
#pragma unroll
      for (int r = 0; r < G; ++r) {
        const bool mm = (mult >> r) & 1u;
        const uint64_t bm = __ballot(mm);
        if (mm) {
          const int64_t q = pc + wave * PW + r * 64 + lane;
          const int64_t d = ow + __popcll(bm & lt);
          a.okeys[d] = key[r];
          a.ovals[d] = sv[base + q];
        }
        ow += __popcll(bm);
      }
      if (a.tag) write_tags<G>(a.T, a.epoch, key, mult & first);
      o += S.misc[0];
      lds_barrier();
    }
    if (sweep == 0) {
      block_counts(nm, ns, S, lane, wave);
      const uint32_t tm = S.misc[0], ts = S.misc[1];
      if (threadIdx.x == 0) publish_own(a, b, tm, ts);
      if (wave == 0) look_back(a, b, tm, ts, S, lane);
      lds_barrier();
      o = (int64_t)S.base[0];
    }
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(kMB) void k_msd_buckets(MsdArgs a) {
  __shared__ MsdLds S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int b;
  if (SPLIT) {  // buckets in ticket order: every bucket a block's look-back waits for has a running block
    if (tid == 0)
      S.misc[2] = (uint32_t)__hip_atomic_fetch_add(&a.status[a.nbk], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
    b = (int)S.misc[2];
  } else {
    b = blockIdx.x;
  }
  int64_t base = 0, n = a.n1;
  if (a.btot) {
    const uint32_t v = tid < a.nbk ? a.btot[tid] : 0u;
    uint32_t t;
    const uint32_t ex = block_excl_scan(v, S, lane, wave, &t);
    if (tid == b) {
      S.misc[2] = ex;
      S.misc[3] = v;
    }
    lds_barrier();
    base = S.misc[2];
    n = S.misc[3];
    lds_barrier();
  }
  const int sh = a.sh;
  const uint32_t lowmask = (1u << sh) - 1u;
  const uint32_t hi = sh >= 32 ? 0u : (uint32_t)b << sh;
  if (n <= kMCap)
    bucket_small<SPLIT>(a, S, b, base, (int)n, hi, lowmask, lane, wave, lt);
  else if (SPLIT)
    big_sweeps(a, S, b, base, n, lane, wave, lt);
  // (full: an oversized bucket was written by k_msd_presort)
}

}  // namespace

MsdPlan msd_plan(int64_t n, int key_bits) {
  MsdPlan p;
  p.ok = false;
  if (n <= 0 || n >= (int64_t(1) << 31) - 1 || key_bits < 1 || key_bits > 32) return p;
  if (n <= kMCap && key_bits <= kMLow) {  // one bucket, no level-1 pass
    p.ok = true;
    p.hb = 0;
    p.sh = key_bits;
    p.nbk = 1;
    return p;
  }
  // about 8K entries per bucket (c3: 1024 buckets of 10K on average, the largest ~31K), at least 64
  // buckets (fm_sort.hip's scans want >= 32 digits), never more low bits than an LDS word carries
  int hb = 6;
  while (hb < 10 && (n >> hb) > 8192) ++hb;
  if (key_bits - hb > kMLow) hb = key_bits - kMLow;
  if (hb > 10 || hb > key_bits) return p;  // the LSD passes
  p.ok = true;
  p.hb = hb;
  p.sh = key_bits - hb;
  p.nbk = 1 << hb;
  return p;
}

void MsdWork::ensure(int64_t n, int nbk) {
  (void)nbk;
  status.ensure(sizeof(unsigned long long) * (size_t)(kMaxBuckets + 4));
  if (n > cap) {
    const int64_t c = n + n / 8 + 4096;
    keys.ensure(sizeof(uint32_t) * c);
    vals.ensure(sizeof(uint2) * c);
    cap = c;
  }
}

static MsdArgs make_args(const MsdPlan& pl, const uint32_t* keys, const uint2* vals, uint32_t* keys_b, uint2* vals_b,
                         const uint32_t* btot, int64_t n, uint32_t* okeys, uint2* ovals) {
  MsdArgs a{};
  a.keys = keys;
  a.vals = vals;
  a.keys_a = const_cast<uint32_t*>(keys);  // oversized buckets only, whose input is a level-1 buffer
  a.vals_a = const_cast<uint2*>(vals);
  a.keys_b = keys_b;
  a.vals_b = vals_b;
  a.btot = pl.hb > 0 ? btot : nullptr;
  a.n1 = n;
  a.nbk = pl.nbk;
  a.sh = pl.sh;
  a.okeys = okeys;
  a.ovals = ovals;
  return a;
}

void msd_sort_full(const MsdPlan& pl, const uint32_t* keys, const uint2* vals, uint32_t* keys_b, uint2* vals_b,
                   const uint32_t* btot, int64_t n, uint32_t* okeys, uint2* ovals, hipStream_t st) {
  FM_REQUIRE(pl.ok, "two-level grouping not planned");
  MsdArgs a = make_args(pl, keys, vals, keys_b, vals_b, btot, n, okeys, ovals);
  if (pl.hb > 0) hipLaunchKernelGGL(k_msd_presort<false>, dim3(kPresortGrid), dim3(kMB), 0, st, a);
  hipLaunchKernelGGL(k_msd_buckets<false>, dim3((unsigned)pl.nbk), dim3(kMB), 0, st, a);
  FM_HIP_CHECK(hipGetLastError());
}

void msd_split(const MsdPlan& pl, const uint32_t* keys, const uint2* vals, const uint32_t* btot, int64_t n,
               MsdWork& mw, uint32_t* mkeys, uint2* ments, int64_t* n_out, hipStream_t st, const TableView* tag_T,
               int32_t epoch) {
  FM_REQUIRE(pl.ok, "two-level grouping not planned");
  mw.ensure(pl.hb > 0 ? n : 0, pl.nbk);
  // the look-back words, the ticket and the error word, zeroed before every launch (a whole number of
  // 16-byte granules from the allocation's start: cdna_hip_programming.md §6 Guideline 16)
  FM_HIP_CHECK(hipMemsetAsync(mw.status.p, 0, sizeof(unsigned long long) * (size_t)((pl.nbk + 3) & ~1), st));
  MsdArgs a = make_args(pl, keys, vals, mw.keys.as<uint32_t>(), mw.vals.as<uint2>(), btot, n, mkeys, ments);
  a.n_out = n_out;
  a.status = mw.status.as<unsigned long long>();
  if (tag_T) {
    a.T = *tag_T;
    a.tag = 1;
    a.epoch = epoch;
  }
  if (pl.hb > 0) hipLaunchKernelGGL(k_msd_presort<true>, dim3(kPresortGrid), dim3(kMB), 0, st, a);
  hipLaunchKernelGGL(k_msd_buckets<true>, dim3((unsigned)pl.nbk), dim3(kMB), 0, st, a);
  FM_HIP_CHECK(hipGetLastError());
}

}  // namespace fmhip
