// CPU test driver for fmhip::HostPool (fm_spark_amd/csrc/fm_hostpool.h): every index runs once, an
// exception thrown by the job reaches the caller after the job has drained, and the pool serves the
// next job.  Built by tests/test_host_sanitizers.py under -fsanitize=thread and address.
#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "../../fm_spark_amd/csrc/fm_hostpool.h"

static int failures = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::printf("FAIL line %d: %s\n", __LINE__, #c);        \
      ++failures;                                             \
    }                                                         \
  } while (0)

int main() {
  fmhip::HostPool& pool = fmhip::HostPool::get();
  for (int rep = 0; rep < 50; ++rep) {
    // every index exactly once
    const int n = 1 + rep * 7;
    std::vector<std::atomic<int>> hits(n);
    for (auto& h : hits) h.store(0);
    pool.run(n, [&](int i) { hits[i].fetch_add(1); });
    for (int i = 0; i < n; ++i) CHECK(hits[i].load() == 1);
    // a throwing job: the exception reaches the caller, no index runs twice, the pool stays usable
    std::atomic<int> ran{0};
    bool caught = false;
    try {
      pool.run(64, [&](int i) {
        ran.fetch_add(1);
        if (i == rep % 64) throw std::runtime_error("job failed");
      });
    } catch (const std::runtime_error&) {
      caught = true;
    }
    CHECK(caught);
    CHECK(ran.load() >= 1 && ran.load() <= 64);
  }
  std::printf("%d failure(s), %d threads\n", failures, pool.threads());
  return failures ? 1 : 0;
}
