// Host-only checks of libfm_hip.so's CPU code under AddressSanitizer / UBSan (the
// sanitizer story is host-side; GPU ASan is not available on this pool).  Built by
// tests/test_host_sanitizers.py with g++ -fsanitize=address,undefined from the product sources
// fm_sampler.cpp and fm_libsvm.cpp; exercises the libsvm reader (well-formed and malformed
// files), the randomSplit replay and its hash / RNG building blocks.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fm_hip.h"

namespace fmhip {
static std::string g_err;
void set_error(const std::string& m) { g_err = m; }
}  // namespace fmhip

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                    \
    }                                                             \
  } while (0)

static void write_file(const char* path, const char* text) {
  FILE* f = std::fopen(path, "wb");
  std::fputs(text, f);
  std::fclose(f);
}

static int read_all(const char* path, std::vector<double>& lab, std::vector<int64_t>& rp, std::vector<int32_t>& col,
                    std::vector<double>& val, int64_t& nf) {
  int64_t B = 0, N = 0;
  int rc = fm_read_libsvm(path, 0, 0, nullptr, nullptr, nullptr, nullptr, &B, &N, &nf);
  if (rc != FM_OK) return rc;
  lab.assign(B + 1, 0.0);
  rp.assign(B + 1, 0);
  col.assign(N + 1, 0);
  val.assign(N + 1, 0.0);
  return fm_read_libsvm(path, B + 1, N + 1, lab.data(), rp.data(), col.data(), val.data(), &B, &N, &nf);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  std::vector<double> lab, val;
  std::vector<int64_t> rp;
  std::vector<int32_t> col;
  int64_t nf = 0;
  const std::string good = dir + "/good.txt", bad = dir + "/bad.txt";
  write_file(good.c_str(), "# c\n\n 1 1:0.5 3:2  \n0\n-2.5 7:1e-3 9:4\n");
  CHECK(read_all(good.c_str(), lab, rp, col, val, nf) == FM_OK);
  CHECK(nf == 9 && rp[3] == 4 && col[0] == 0 && col[3] == 8 && lab[2] == -2.5);
  const char* bads[] = {"1 3:1 2:1\n", "1 0:1\n", "1 1:x\n", "x 1:1\n", "1 2\n", "1 99999999999:1\n", "1 :1\n", "1 1:\n"};
  for (const char* b : bads) {
    write_file(bad.c_str(), b);
    CHECK(read_all(bad.c_str(), lab, rp, col, val, nf) == FM_ERR_ARG);
  }
  int64_t B = 0, N = 0;
  CHECK(fm_read_libsvm((dir + "/missing.txt").c_str(), 0, 0, nullptr, nullptr, nullptr, nullptr, &B, &N, &nf) < 0);
  CHECK(read_all(good.c_str(), lab, rp, col, val, nf) == FM_OK);
  // too-small buffers are refused, not overrun
  CHECK(fm_read_libsvm(good.c_str(), 1, 1, lab.data(), rp.data(), col.data(), val.data(), &B, &N, &nf) == FM_ERR_ARG);

  // hashing / RNG building blocks: the SMHasher verification value of MurmurHash3_x86_32
  {
    std::vector<uint8_t> key(256);
    std::vector<uint32_t> hashes(256);
    for (int i = 0; i < 256; ++i) {
      key[i] = (uint8_t)i;
      hashes[i] = (uint32_t)fm_murmur3_bytes_hash(key.data(), i, 256 - i);
    }
    const uint32_t final_h =
        (uint32_t)fm_murmur3_bytes_hash(reinterpret_cast<const uint8_t*>(hashes.data()), 1024, 0);
    CHECK(final_h == 0xB0F57EE3u);
    std::vector<double> d(1000);
    CHECK(fm_xorshift_next_doubles(1234, 1000, d.data()) == FM_OK);
    for (double x : d) CHECK(x >= 0.0 && x < 1.0);
    (void)fm_xorshift_hash_seed(-7);
  }

  // randomSplit replay over two partitions of sparse + dense rows
  {
    const int n = 500;
    std::vector<int64_t> part_ptr = {0, 230, n};
    std::vector<double> label(n);
    std::vector<int8_t> vtype(n);
    std::vector<int32_t> vsize(n, 20);
    std::vector<int64_t> vptr(n + 1, 0);
    std::vector<int32_t> vidx;
    std::vector<double> vval;
    std::vector<int64_t> extra(n);
    for (int i = 0; i < n; ++i) {
      label[i] = (i * 7) % 3;
      vtype[i] = (i % 5 == 0) ? 1 : 0;
      extra[i] = i % 11;
      const int z = vtype[i] ? 20 : 1 + i % 6;
      for (int j = 0; j < z; ++j) {
        vidx.push_back(vtype[i] ? 0 : j * 3 + i % 3);  // sparse: ascending, < 20
        vval.push_back((i + j) % 4 * 0.5);
      }
      vptr[i + 1] = (int64_t)vidx.size();
    }
    std::vector<double> w = {0.3, 0.3, 0.4};
    std::vector<int32_t> split(n);
    std::vector<int64_t> sid(n), order(n);
    int rc = fm_random_split(2, part_ptr.data(), "LFI", label.data(), vtype.data(), vsize.data(), vptr.data(),
                             vidx.data(), vval.data(), extra.data(), 3, w.data(), 1234, split.data(), sid.data(),
                             order.data());
    CHECK(rc == FM_OK);
    int cnt[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
      CHECK(split[i] >= -1 && split[i] < 3);
      if (split[i] >= 0) ++cnt[split[i]];
    }
    CHECK(cnt[0] + cnt[1] + cnt[2] == n);  // weights sum to 1: every row lands in one split
  }
  std::printf("host sanitizer checks: %d failure(s)\n", fails);
  return fails ? 1 : 0;
}
