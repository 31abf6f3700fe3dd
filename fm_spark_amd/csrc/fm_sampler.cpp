// Host replay of the reference's mini-batch sampler:
//   dfData.randomSplit(Array.fill(maxIter)(miniBatchFraction), 1234L)
//   (FactorizationMachinesSGD.scala:111-112) over rows tagged by
//   monotonically_increasing_id (FactorizationMachinesModel.scala:268-272).
//
// The algorithm is Spark 2.1.0's (spark-sql Dataset.randomSplit -> per-partition ascending
// sort on every column -> SampleExec -> RDD.randomSampleWithRange -> BernoulliCellSampler
// seeded XORShiftRandom(seed + partitionIndex)), with XORShiftRandom.hashSeed built on
// scala 2.11 MurmurHash3.bytesHash.  None of that code is vendored in the reference; this
// restates it (see oracle/spark_sampler.py for the line-by-line derivation).  The sampler is
// host work by nature (a sequential RNG stream per partition and a lexicographic sort of
// variable-length rows, run once per fit rather than once per step).  Partitions are independent
// (each its own sort, its own XORShiftRandom(seed + p)), so they run on the library's host thread
// pool: the same rows, splits and order as one thread, partition after partition.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/fm_hip.h"
#include "fm_hostpool.h"

namespace fmhip {
void set_error(const std::string& msg);
}

namespace {

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

inline uint32_t mix_last(uint32_t h, uint32_t k) {
  k *= 0xCC9E2D51u;
  k = rotl32(k, 15);
  k *= 0x1B873593u;
  return h ^ k;
}

inline uint32_t mix(uint32_t h, uint32_t k) {
  h = mix_last(h, k);
  h = rotl32(h, 13);
  return h * 5u + 0xE6546B64u;
}

uint32_t murmur3_bytes(const uint8_t* d, int64_t len, uint32_t seed) {
  uint32_t h = seed;
  int64_t i = 0;
  for (; len - i >= 4; i += 4) {
    const uint32_t k = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) | ((uint32_t)d[i + 3] << 24);
    h = mix(h, k);
  }
  const int64_t rem = len - i;
  if (rem > 0) {
    uint32_t k = 0;
    if (rem == 3) k ^= (uint32_t)d[i + 2] << 16;
    if (rem >= 2) k ^= (uint32_t)d[i + 1] << 8;
    k ^= (uint32_t)d[i];
    h = mix_last(h, k);
  }
  h ^= (uint32_t)len;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

constexpr uint32_t kArraySeed = 0x3C074A61u;

int64_t hash_seed(int64_t seed) {
  uint8_t bytes[64];
  std::memset(bytes, 0, sizeof(bytes));  // ByteBuffer.allocate(java.lang.Long.SIZE = 64)
  const uint64_t s = (uint64_t)seed;
  for (int i = 0; i < 8; ++i) bytes[i] = (uint8_t)(s >> (56 - 8 * i));  // putLong, big-endian
  const uint32_t lo = murmur3_bytes(bytes, 64, kArraySeed);
  const uint32_t hi = murmur3_bytes(bytes, 64, lo);
  return (int64_t)(((uint64_t)hi << 32) | (uint64_t)lo);
}

struct XorShift {
  uint64_t s;
  explicit XorShift(int64_t seed) : s((uint64_t)hash_seed(seed)) {}
  uint32_t next(int bits) {
    s ^= s << 21;
    s ^= s >> 35;
    s ^= s << 4;
    return (uint32_t)(s & ((uint64_t(1) << bits) - 1));
  }
  double next_double() {
    return (double)(((uint64_t)next(26) << 27) + (uint64_t)next(27)) * 0x1.0p-53;
  }
};

// Spark's nanSafeCompareDoubles: NaN is larger than everything, NaN == NaN, -0.0 == 0.0.
inline int cmp_double(double a, double b) {
  const bool an = std::isnan(a), bn = std::isnan(b);
  if (an && bn) return 0;
  if (an) return 1;
  if (bn) return -1;
  return a < b ? -1 : (a > b ? 1 : 0);
}

template <class T>
inline int cmp_val(T a, T b) {
  return a < b ? -1 : (a > b ? 1 : 0);
}

struct Rows {
  const double* label;
  const int8_t* type;
  const int32_t* size;
  const int64_t* ptr;
  const int32_t* idx;
  const double* val;
  const int64_t* extra;
};

// VectorUDT.sqlType = struct<type: byte, size: int, indices: array<int>, values: array<double>>,
// ascending with nulls first; arrays element-wise, then shorter first.
int cmp_vector(const Rows& R, int64_t a, int64_t b) {
  int c = cmp_val<int>(R.type[a], R.type[b]);
  if (c) return c;
  const int64_t la = R.ptr[a + 1] - R.ptr[a], lb = R.ptr[b + 1] - R.ptr[b];
  if (R.type[a] == 0) {  // sparse: size, indices
    c = cmp_val<int32_t>(R.size[a], R.size[b]);
    if (c) return c;
    const int64_t m = std::min(la, lb);
    for (int64_t i = 0; i < m; ++i) {
      c = cmp_val<int32_t>(R.idx[R.ptr[a] + i], R.idx[R.ptr[b] + i]);
      if (c) return c;
    }
    c = cmp_val<int64_t>(la, lb);
    if (c) return c;
  }
  const int64_t m = std::min(la, lb);
  for (int64_t i = 0; i < m; ++i) {
    c = cmp_double(R.val[R.ptr[a] + i], R.val[R.ptr[b] + i]);
    if (c) return c;
  }
  return cmp_val<int64_t>(la, lb);
}

}  // namespace

extern "C" {

int64_t fm_xorshift_hash_seed(int64_t seed) { return hash_seed(seed); }

int32_t fm_murmur3_bytes_hash(const uint8_t* data, int64_t len, int32_t seed) {
  return (int32_t)murmur3_bytes(data, len, (uint32_t)seed);
}

int fm_xorshift_next_doubles(int64_t seed, int64_t n, double* out) {
  if (n < 0 || (n > 0 && !out)) {
    fmhip::set_error("bad arguments");
    return FM_ERR_ARG;
  }
  XorShift r(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = r.next_double();
  return FM_OK;
}

int fm_random_split(int32_t n_parts, const int64_t* part_ptr, const char* column_order, const double* label,
                    const int8_t* vec_type, const int32_t* vec_size, const int64_t* vec_ptr, const int32_t* vec_idx,
                    const double* vec_val, const int64_t* extra, int32_t n_weights, const double* weights,
                    int64_t seed, int32_t* split_of, int64_t* sample_id, int64_t* order) {
  try {
    if (n_parts < 0 || !part_ptr || !column_order || n_weights < 1 || !weights || !split_of || !sample_id) {
      fmhip::set_error("fm_random_split: bad arguments");
      return FM_ERR_ARG;
    }
    const std::string cols(column_order);
    for (char c : cols) {
      if (c == 'L' && !label) { fmhip::set_error("label column without data"); return FM_ERR_ARG; }
      if (c == 'F' && (!vec_type || !vec_size || !vec_ptr || !vec_val)) {
        fmhip::set_error("features column without data");
        return FM_ERR_ARG;
      }
      if (c == 'I' && !extra) { fmhip::set_error("int64 column without data"); return FM_ERR_ARG; }
      if (c != 'L' && c != 'F' && c != 'I') { fmhip::set_error("column_order must use L, F, I"); return FM_ERR_ARG; }
    }
    // Dataset.randomSplit: require(weights.forall(_ >= 0)); require(weights.sum > 0)
    double total = 0.0;
    for (int32_t i = 0; i < n_weights; ++i) {
      if (!(weights[i] >= 0.0)) { fmhip::set_error("Weights must be nonnegative"); return FM_ERR_ARG; }
      total += weights[i];
    }
    if (!(total > 0.0)) { fmhip::set_error("Sum of weights must be positive"); return FM_ERR_ARG; }
    std::vector<double> cum(n_weights + 1, 0.0);  // weights.map(_ / sum).scanLeft(0.0d)(_ + _)
    for (int32_t i = 0; i < n_weights; ++i) cum[i + 1] = cum[i] + weights[i] / total;
    const Rows R{label, vec_type, vec_size, vec_ptr, vec_idx, vec_val, extra};
    for (int32_t p = 0; p < n_parts; ++p)
      if (part_ptr[p + 1] < part_ptr[p]) { fmhip::set_error("part_ptr must be non-decreasing"); return FM_ERR_ARG; }
    // one job per partition on the host pool (no exception leaves a worker: a failed partition is
    // reported after the join)
    std::atomic<bool> failed{false};
    const std::function<void(int)> job = [&](int p) {
      try {
        const int64_t r0 = part_ptr[p], r1 = part_ptr[p + 1];
        for (int64_t r = r0; r < r1; ++r) sample_id[r] = ((int64_t)p << 33) + (r - r0);
        std::vector<int64_t> ord(r1 - r0);
        std::iota(ord.begin(), ord.end(), r0);
        std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
          for (char c : cols) {
            int x = 0;
            if (c == 'L') x = cmp_double(label[a], label[b]);
            else if (c == 'F') x = cmp_vector(R, a, b);
            else x = cmp_val<int64_t>(extra[a], extra[b]);
            if (x) return x < 0;
          }
          return ((int64_t)p << 33) + (a - r0) < ((int64_t)p << 33) + (b - r0);  // monotonically_increasing_id
        });
        XorShift rng(seed + p);  // BernoulliCellSampler.setSeed(seed + index)
        for (int64_t j = 0; j < (int64_t)ord.size(); ++j) {
          const int64_t r = ord[j];
          if (order) order[r0 + j] = r;
          const double x = rng.next_double();
          int32_t sp = -1;
          for (int32_t i = 0; i < n_weights; ++i) {
            const double lb = cum[i], ub = cum[i + 1];
            if (ub - lb <= 0.0) continue;  // BernoulliCellSampler: empty range keeps nothing
            if (x >= lb && x < ub) {
              sp = i;
              break;
            }
          }
          split_of[r] = sp;
        }
      } catch (...) {
        failed.store(true);
      }
    };
    fmhip::HostPool::get().run(n_parts, job);
    if (failed.load()) {
      fmhip::set_error("fm_random_split: host allocation failed");
      return FM_ERR_OOM;
    }
    return FM_OK;
  } catch (const std::exception& e) {
    fmhip::set_error(e.what());
    return FM_ERR_OOM;
  }
}

}  // extern "C"
