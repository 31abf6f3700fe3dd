// A persistent pool of host threads shared by the library's host passes (fm_capi.hip: fm_step's
// upload, fm_batch_from_rows; fm_sampler.cpp: fm_random_split's partitions).  Not part of the C-ABI.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace fmhip {

// A persistent pool of host threads (up to 16: the GPU box's CPU share per GPU; 8 measured the same
// in the fit loop) for the host passes of fm_step's upload, fm_batch_from_rows and fm_random_split:
// spawning the threads per call cost about as much as the work.  One job at a time (callers
// serialise on run_mu); the calling thread works too.
constexpr int kHostThreadsMax = 16;
class HostPool {
 public:
  static HostPool& get() {
    static HostPool p;
    return p;
  }
  int threads() const { return (int)workers_.size() + 1; }
  // f(i) for every i in [0, n).  An exception thrown by f is rethrown here (the first one caught)
  // once every index has been run or skipped and no worker still holds the job.
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    std::lock_guard<std::mutex> job_lk(run_mu_);
    if (n == 1 || workers_.empty()) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      njobs_ = n;
      next_.store(0);
      done_ = 0;
      err_ = nullptr;
      failed_.store(false);
      ++gen_;
    }
    cv_.notify_all();
    work(&f, n);
    std::exception_ptr err;
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return done_ == njobs_ && active_ == 0; });
      job_ = nullptr;
      err = err_;
    }
    if (err) std::rethrow_exception(err);
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  HostPool() {
    const int hw = std::max(1, (int)std::thread::hardware_concurrency());
    const int T = std::min(kHostThreadsMax, hw);
    for (int t = 1; t < T; ++t) workers_.emplace_back([this] { loop(); });
  }
  // indices of the current job until none is left; after the first exception the rest are skipped
  void work(const std::function<void(int)>* job, int n) {
    int mine = 0;
    for (int i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) {
      if (!failed_.load(std::memory_order_relaxed)) {
        try {
          (*job)(i);
        } catch (...) {
          std::lock_guard<std::mutex> lk(mu_);
          if (!err_) err_ = std::current_exception();
          failed_.store(true, std::memory_order_relaxed);
        }
      }
      ++mine;
    }
    if (mine) {
      std::lock_guard<std::mutex> lk(mu_);
      done_ += mine;
      if (done_ == njobs_) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      int n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (gen_ != seen && job_ != nullptr); });
        if (stop_) return;
        seen = gen_;
        job = job_;
        n = njobs_;
        ++active_;  // run() does not return (and f does not go out of scope) while a worker holds it
      }
      work(job, n);
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int njobs_ = 0, done_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  std::atomic<bool> failed_{false};
  std::exception_ptr err_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace fmhip
