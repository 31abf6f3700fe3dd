// Multi-GPU inside one fm_ctx: one host thread drives every rank of the job this process holds,
// and the exchanges between ranks run inside the library over RCCL (xGMI on one node).
//
// SURVEY §8(b) Threading: "Multi-GPU lives inside one context (one host thread)": the caller is
// the Spark driver, one JVM, so the multi-GPU step cannot need one process per GPU.  A context
// created with fm_config.parallel = FM_PARALLEL_SHARDED / FM_PARALLEL_REPLICATED holds n_gpus
// local ranks.  Each is an ordinary per-device fm_ctx (a "member": its share of the table, its
// streams and workspaces); this file sequences the member phases of fm_shard.hip / fm_capi.hip
// and moves the data between them.  The reference's shuffles it replaces:
//   sharded  : S1/S2 (entries ⋈ w, V by featureId, Model.scala:155-164) -> the entry all-to-all;
//              S3 (window by sampleId, :191) -> partial sums back to the requester;
//              S5/S6 (gradient groupBy + outer join, SGD.scala:148-166) -> S rows to the owner,
//              owner-local update (fm_shard.hip for the phases and the wire layout)
//   replicated: S5 -> one all-reduce of the per-slot gradient sums (fm_repl_grad / fm_repl_apply)
// A mini-batch handed to the context is split by rows, contiguously, over its local ranks; the
// iteration's miniBatchSize is the sum over every rank of the job (SGD.scala:124).
//
// Transports.  RCCL: grouped ncclSend/ncclRecv for the all-to-alls (every peer at once, so an
// all-to-all drives all 7 xGMI links of a GPU), ncclAllReduce / ncclAllGather for the gradient
// and the counts; one communicator per stream role (main: the iteration's critical path; side:
// the batch-only routing that runs one iteration ahead), each used in the same order on every
// rank.  COPY (one process only): device-to-device copies between the ranks' buffers, bracketed
// by event barriers across the ranks' streams; it also lets several ranks share one GPU, which
// RCCL refuses -- that is how the in-process tests run an 8-rank job on one MI355X.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <numeric>
#include <thread>
#include <mutex>
#include <functional>
#include <exception>
#include <condition_variable>

#include "fm_context.h"
#include "fm_plan.h"
#include "fm_device.h"

namespace fmhip {

#define FM_RCCL_CHECK(expr)                                                                  \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess)                                                                   \
      throw ::fmhip::Error{FM_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)}; \
  } while (0)

namespace {

// a member call through the C-ABI: its error (and message) becomes the group's
void mcheck(int rc, const char* what) {
  if (rc < 0) throw Error{rc, std::string(what) + ": " + fm_last_error()};
}

constexpr int kBlock = 256;

__global__ void k_slots_to_ids(const uint32_t* __restrict__ slot, int64_t n, uint32_t R, uint32_t shard,
                               uint32_t* __restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ids[i] = slot[i] * R + shard;
}

__global__ void k_add_f32(float* __restrict__ dst, const float* __restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

// COPY transport with every rank on one device: an all-to-all's blocks copied by one kernel launch
// (blockIdx.y = block) instead of one hipMemcpyAsync per (source, destination, segment) -- 128 host
// calls per all-to-all at R = 8, the COPY driver's host time (profiles/r06_host)
struct CopyDesc {
  const char* src;
  char* dst;
  uint64_t bytes;
};
constexpr int kMaxCopyDesc = 128;  // 3 KB of kernel arguments
struct CopyList {
  int n;
  CopyDesc d[kMaxCopyDesc];
};

__global__ void k_copy_list(CopyList cl) {
  const CopyDesc d = cl.d[blockIdx.y];
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
  if ((((uintptr_t)d.src | (uintptr_t)d.dst | d.bytes) & 15u) == 0) {
    const uint4* s = reinterpret_cast<const uint4*>(d.src);
    uint4* t = reinterpret_cast<uint4*>(d.dst);
    for (uint64_t i = tid; i < d.bytes / 16; i += nth) t[i] = s[i];
  } else {  // element sizes are multiples of 4 bytes
    const uint32_t* s = reinterpret_cast<const uint32_t*>(d.src);
    uint32_t* t = reinterpret_cast<uint32_t*>(d.dst);
    for (uint64_t i = tid; i < d.bytes / 4; i += nth) t[i] = s[i];
  }
}

inline unsigned grid_of(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 16));
}

}  // namespace

struct Rank {
  fm_ctx* m = nullptr;  // the member context (owned)
  int device = 0;
  int global = 0;
  ncclComm_t comm_main = nullptr, comm_side = nullptr, comm_x = nullptr;
  hipEvent_t ev_main = nullptr, ev_side = nullptr;  // COPY transport barriers
  DevBuf partials, part_in, s_send, s_recv;           // sharded wire buffers (main stream)
  DevBuf pc_out, pc_in, pred;                         // sharded predict: present counts, scores
  DevBuf grad, gtmp;                                  // replicated gradient buffer
  DevBuf xg_send, xg_recv;                            // counts all-gather (RCCL)
  Pinned xg_pin;
  // chunked partial exchange of the sharded step (R > 1): its own stream and communicator
  hipStream_t xstream = nullptr;
  hipEvent_t ev_x = nullptr, ev_fwd = nullptr, ev_xdone = nullptr;
  // lanes: 0 main stream, 1 side stream (batch-only work: route, entry exchange, owner preparation),
  // 2 the exchange stream.  Few streams on purpose: HIP maps a process's streams round-robin onto
  // GPU_MAX_HW_QUEUES hardware queues (4 by default), and two streams on one queue run in submission
  // order -- a route on a stream of its own shared the main stream's queue (profiles/r03_v3 kernel
  // trace: queue 4 for both) and waited behind the step
  hipStream_t stream(int lane) const { return lane == 2 ? xstream : lane ? m->side : m->stream; }
  hipEvent_t event(int lane) const { return lane == 2 ? ev_x : lane ? ev_side : ev_main; }
  // one communicator per stream, each used in the same order on every rank
  ncclComm_t comm(int lane) const { return lane == 2 ? comm_x : lane ? comm_side : comm_main; }
};
constexpr int kLaneMain = 0, kLaneSide = 1, kLaneXchg = 2;

struct GPart {
  fm_batch* b = nullptr;  // the member's batch (owned)
  int device = 0;
  int64_t rows = 0, row0 = 0, nnz = 0;
  DevBuf send_slot, send_ent, recv_slot, recv_ent;
  // what the owner reads: recv_*, or for a one-rank job its own send buffers (nothing to exchange)
  void* in_slot = nullptr;
  void* in_ent = nullptr;
  std::vector<int64_t> ent_out, pair_out, ent_in, pair_in;  // per global peer
};

struct GroupBatch {
  std::vector<GPart> parts;
  int64_t rows = 0, nnz = 0, global_rows = 0;
  bool prefetched = false;  // routed, exchanged and slot-sorted for its next step
  // sharded prepare, phase 1 done: routes and their count gather enqueued (side streams), the
  // counts on their way to cnt_pin; phase 2 (the host reads them, exchange, owner preparation)
  // runs at the context's next fm_batch_prepare or at this batch's step
  bool routed = false;
  Pinned cnt_pin;
  std::vector<hipEvent_t> ev_cnt;  // per local rank: its side-stream work of phase 1 is done
  Group* g = nullptr;              // the group while this batch is its pending phase 2
  // fm_batch_from_rows with this batch as the dataset: every local rank's full copy of it (member
  // batches on each rank's device, made at the first selection), from which each rank gathers its
  // share of a split's rows
  std::vector<fm_batch*> full;
  ~GroupBatch();
};

// Host workers of a multi-rank context: one thread per local rank beyond the first (the calling
// thread takes rank 0).  each(f) runs f(l) for every local rank at once and returns when all have
// returned; an exception thrown for any rank is rethrown afterwards (the lowest rank's).  The
// per-rank phases of an iteration (route, owner preparation, owner passes, combine, update) are
// enqueued this way: one thread enqueueing R ranks' kernels one after another costs R times one
// rank's host time per phase.  The C-ABI's contract is unchanged -- one caller thread at a time per
// context (its mutex); the workers only act inside one of that caller's calls, each on its own
// rank's member context, streams and communicators.
class RankWorkers {
 public:
  void start(int L) {
    for (int l = 1; l < L; ++l) threads_.emplace_back([this, l] { loop(l); });
  }
  void each(int L, const std::function<void(int)>& f) {
    if (threads_.empty() || L <= 1) {
      for (int l = 0; l < L; ++l) f(l);
      return;
    }
    std::vector<std::exception_ptr> err(L);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      err_ = &err;
      pending_ = L - 1;
      ++gen_;
    }
    cv_.notify_all();
    try {
      f(0);
    } catch (...) {
      err[0] = std::current_exception();
    }
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [&] { return pending_ == 0; });
      job_ = nullptr;
      err_ = nullptr;
    }
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }
  ~RankWorkers() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

 private:
  void loop(int l) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      std::vector<std::exception_ptr>* err;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
        err = err_;
      }
      try {
        (*f)(l);
      } catch (...) {
        (*err)[l] = std::current_exception();
      }
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  std::vector<std::exception_ptr>* err_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct Group {
  int mode = FM_PARALLEL_SHARDED;
  GroupBatch* pending = nullptr;  // the batch whose sharded prepare waits for its phase 2
  int L = 0, R = 0, nprocs = 1, prank = 0;
  int xchg = 4;  // chunks of the sharded partial exchange (fm_config.xchg_chunks)
  bool rccl = false;
  std::vector<Rank> ranks;
  std::unique_ptr<fm_batch> host_b[2];  // fm_step / fm_predict uploads, used in turn
  int hnext = 0;
  RankWorkers workers;  // per-rank host workers (L > 1)
  bool sharded() const { return mode == FM_PARALLEL_SHARDED; }
  // f(l) for every local rank, in parallel on the rank workers
  void each(const std::function<void(int)>& f) { workers.each(L, f); }
  ~Group() {
    if (pending) pending->g = nullptr;
    for (auto& h : host_b) h.reset();
    for (auto& r : ranks) {
      if (!r.m) continue;
      (void)hipSetDevice(r.device);
      (void)hipDeviceSynchronize();
      if (r.comm_x) (void)ncclCommDestroy(r.comm_x);
      if (r.comm_side) (void)ncclCommDestroy(r.comm_side);
      if (r.comm_main) (void)ncclCommDestroy(r.comm_main);
      for (DevBuf* d : {&r.partials, &r.part_in, &r.s_send, &r.s_recv, &r.pc_out, &r.pc_in, &r.pred, &r.grad, &r.gtmp,
                        &r.xg_send, &r.xg_recv})
        d->release();
      if (r.ev_main) (void)hipEventDestroy(r.ev_main);
      if (r.ev_side) (void)hipEventDestroy(r.ev_side);
      for (hipEvent_t e : {r.ev_x, r.ev_fwd, r.ev_xdone})
        if (e) (void)hipEventDestroy(e);
      if (r.xstream) (void)hipStreamDestroy(r.xstream);
    }
    for (auto& r : ranks)
      if (r.m) fm_destroy(r.m);
  }
};

GroupBatch::~GroupBatch() {
  if (g && g->pending == this) g->pending = nullptr;
  for (size_t l = 0; l < ev_cnt.size(); ++l) {
    (void)hipSetDevice(parts[l].device);
    (void)hipEventSynchronize(ev_cnt[l]);
    (void)hipEventDestroy(ev_cnt[l]);
  }
  for (auto& p : parts) {
    (void)hipSetDevice(p.device);
    for (DevBuf* d : {&p.send_slot, &p.send_ent, &p.recv_slot, &p.recv_ent}) d->release();
    if (p.b) fm_batch_destroy(p.b);
    p.b = nullptr;
  }
  for (fm_batch* f : full)
    if (f) fm_batch_destroy(f);
}

void GroupDeleter::operator()(Group* g) const { delete g; }
void GroupBatchDeleter::operator()(GroupBatch* g) const { delete g; }

namespace {

// run f with the member locked and its device current (internal, non-ABI member calls)
template <class F>
void on(Rank& r, F&& f) {
  std::lock_guard<std::mutex> lk(r.m->mu);
  FM_HIP_CHECK(hipSetDevice(r.device));
  f();
}

void ensure_on(int device, DevBuf& b, size_t bytes) {
  FM_HIP_CHECK(hipSetDevice(device));
  b.ensure(bytes + 16);
}

Group& grp(fm_ctx* ctx) { return *ctx->group; }

GroupBatch& gbatch(fm_ctx* ctx, fm_batch* b) {
  FM_REQUIRE(b != nullptr && b->owner == ctx && b->grp, "batch belongs to another context");
  return *b->grp;
}

// COPY transport: every rank's stream (side or main) waits for what every other rank's has queued
void barrier(Group& g, int side) {
  for (auto& r : g.ranks) {
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_HIP_CHECK(hipEventRecord(r.event(side), r.stream(side)));
  }
  for (auto& r : g.ranks) {
    FM_HIP_CHECK(hipSetDevice(r.device));
    for (auto& q : g.ranks)
      if (&q != &r) FM_HIP_CHECK(hipStreamWaitEvent(r.stream(side), q.event(side), 0));
  }
}

// One buffer pair of an all-to-all-v (element size esize; per local rank l, send[l] and recv[l]).
struct A2ASeg {
  const std::vector<const char*>& send;
  const std::vector<char*>& recv;
  size_t esize;
};
// Per local rank l and global peer p (in elements): send sc[l][p] from send[l] + so[l][p] to p, and
// receive rc[l][p] from p into recv[l] + ro[l][p].
struct A2APlan {
  std::vector<std::vector<int64_t>> so, sc, ro, rc;
  void add(plan::Plan&& p) {  // the next local rank's plan (fm_plan.h)
    so.push_back(std::move(p.so));
    sc.push_back(std::move(p.sc));
    ro.push_back(std::move(p.ro));
    rc.push_back(std::move(p.rc));
  }
};

// All-to-all-v of one or more segments with the same plan between the job's ranks, on `lane`;
// with RCCL every segment's sends and receives go in one group.
void a2a_plan(Group& g, int lane, const std::vector<A2ASeg>& segs, const A2APlan& pl) {
  if (g.rccl) {
    // the block a rank keeps for itself is a device copy on its own stream, not a send to itself
    // through RCCL's channel buffers
    for (const A2ASeg& s : segs) {
      for (int l = 0; l < g.L; ++l) {
        Rank& r = g.ranks[l];
        const int me = r.global;
        FM_REQUIRE(pl.sc[l][me] == pl.rc[l][me], "a2a: the self block differs between send and receive");
        const size_t bytes = (size_t)pl.sc[l][me] * s.esize;
        if (bytes) {
          FM_HIP_CHECK(hipSetDevice(r.device));
          FM_HIP_CHECK(hipMemcpyAsync(s.recv[l] + (size_t)pl.ro[l][me] * s.esize, s.send[l] + (size_t)pl.so[l][me] * s.esize,
                                      bytes, hipMemcpyDeviceToDevice, r.stream(lane)));
        }
      }
    }
    if (g.R == 1) return;
    FM_RCCL_CHECK(ncclGroupStart());
    for (const A2ASeg& s : segs) {
      for (int l = 0; l < g.L; ++l) {
        Rank& r = g.ranks[l];
        FM_HIP_CHECK(hipSetDevice(r.device));
        for (int p = 0; p < g.R; ++p) {
          if (p == r.global) continue;
          const size_t sb = (size_t)pl.sc[l][p] * s.esize, rb = (size_t)pl.rc[l][p] * s.esize;
          if (sb)
            FM_RCCL_CHECK(ncclSend(s.send[l] + (size_t)pl.so[l][p] * s.esize, sb, ncclChar, p, r.comm(lane), r.stream(lane)));
          if (rb)
            FM_RCCL_CHECK(ncclRecv(s.recv[l] + (size_t)pl.ro[l][p] * s.esize, rb, ncclChar, p, r.comm(lane), r.stream(lane)));
        }
      }
    }
    FM_RCCL_CHECK(ncclGroupEnd());
    return;
  }
  bool one_device = true;
  for (const Rank& r : g.ranks) one_device = one_device && r.device == g.ranks[0].device;
  if (one_device) {
    // rank 0's stream waits for every rank's, copies every block in one launch, every rank waits for it
    Rank& r0 = g.ranks[0];
    FM_HIP_CHECK(hipSetDevice(r0.device));
    for (int l = 1; l < g.L; ++l) {
      FM_HIP_CHECK(hipEventRecord(g.ranks[l].event(lane), g.ranks[l].stream(lane)));
      FM_HIP_CHECK(hipStreamWaitEvent(r0.stream(lane), g.ranks[l].event(lane), 0));
    }
    CopyList cl;
    cl.n = 0;
    uint64_t most = 0;
    auto flush = [&] {
      if (!cl.n) return;
      const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(1024, (most / 16 + 255) / 256));
      hipLaunchKernelGGL(k_copy_list, dim3(gx, (unsigned)cl.n), dim3(256), 0, r0.stream(lane), cl);
      FM_HIP_CHECK(hipGetLastError());
      cl.n = 0;
      most = 0;
    };
    for (const A2ASeg& s : segs)
      for (int l = 0; l < g.L; ++l)    // destination
        for (int q = 0; q < g.L; ++q) {  // source (one process: global rank = local rank)
          FM_REQUIRE(pl.sc[q][l] == pl.rc[l][q], "a2a: send and receive counts differ");
          const size_t bytes = (size_t)pl.rc[l][q] * s.esize;
          if (!bytes) continue;
          cl.d[cl.n++] = CopyDesc{s.send[q] + (size_t)pl.so[q][l] * s.esize, s.recv[l] + (size_t)pl.ro[l][q] * s.esize,
                                  (uint64_t)bytes};
          most = std::max<uint64_t>(most, bytes);
          if (cl.n == kMaxCopyDesc) flush();
        }
    flush();
    FM_HIP_CHECK(hipEventRecord(r0.event(lane), r0.stream(lane)));
    for (int l = 1; l < g.L; ++l) FM_HIP_CHECK(hipStreamWaitEvent(g.ranks[l].stream(lane), r0.event(lane), 0));
    return;
  }
  barrier(g, lane);
  for (const A2ASeg& s : segs) {
    for (int l = 0; l < g.L; ++l) {  // destination
      Rank& r = g.ranks[l];
      FM_HIP_CHECK(hipSetDevice(r.device));
      for (int q = 0; q < g.L; ++q) {  // source (one process: global rank = local rank)
        FM_REQUIRE(pl.sc[q][l] == pl.rc[l][q], "a2a: send and receive counts differ");
        const size_t bytes = (size_t)pl.rc[l][q] * s.esize;
        if (bytes)
          FM_HIP_CHECK(hipMemcpyAsync(s.recv[l] + (size_t)pl.ro[l][q] * s.esize, s.send[q] + (size_t)pl.so[q][l] * s.esize,
                                      bytes, hipMemcpyDefault, r.stream(lane)));
      }
    }
  }
  barrier(g, lane);
}

// The plan of a packed all-to-all-v: blocks peer-major in both buffers, out[l][p] / in[l][p] elements.
A2APlan packed_plan(Group& g, const std::vector<const int64_t*>& out, const std::vector<const int64_t*>& in) {
  A2APlan pl;
  for (int l = 0; l < g.L; ++l) pl.add(plan::packed(out[l], in[l], g.R));
  return pl;
}

void a2a_multi(Group& g, int lane, const std::vector<A2ASeg>& segs, const std::vector<const int64_t*>& out,
               const std::vector<const int64_t*>& in) {
  a2a_plan(g, lane, segs, packed_plan(g, out, in));
}

void a2a(Group& g, int lane, const std::vector<const char*>& send, const std::vector<char*>& recv,
         const std::vector<const int64_t*>& out, const std::vector<const int64_t*>& in, size_t esize) {
  a2a_multi(g, lane, {A2ASeg{send, recv, esize}}, out, in);
}

// Every rank's `width` int64 values -> all ranks' values on the host, rank-major [R][width].
std::vector<int64_t> allgather(Group& g, const std::vector<std::vector<int64_t>>& local, int width) {
  std::vector<int64_t> all((size_t)g.R * width, 0);
  if (!g.rccl) {
    for (int l = 0; l < g.L; ++l) std::copy(local[l].begin(), local[l].end(), all.begin() + (size_t)g.ranks[l].global * width);
    return all;
  }
  const size_t bs = sizeof(int64_t) * width, br = bs * g.R;
  for (int l = 0; l < g.L; ++l) {
    Rank& r = g.ranks[l];
    ensure_on(r.device, r.xg_send, bs);
    ensure_on(r.device, r.xg_recv, br);
    r.xg_pin.ensure(std::max(bs, br));
    std::memcpy(r.xg_pin.p, local[l].data(), bs);
    FM_HIP_CHECK(hipMemcpyAsync(r.xg_send.p, r.xg_pin.p, bs, hipMemcpyHostToDevice, r.stream(true)));
  }
  FM_RCCL_CHECK(ncclGroupStart());
  for (int l = 0; l < g.L; ++l) {
    Rank& r = g.ranks[l];
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_RCCL_CHECK(ncclAllGather(r.xg_send.p, r.xg_recv.p, width, ncclInt64, r.comm_side, r.stream(true)));
  }
  FM_RCCL_CHECK(ncclGroupEnd());
  Rank& r0 = g.ranks[0];
  FM_HIP_CHECK(hipSetDevice(r0.device));
  FM_HIP_CHECK(hipMemcpyAsync(r0.xg_pin.p, r0.xg_recv.p, br, hipMemcpyDeviceToHost, r0.stream(true)));
  for (auto& r : g.ranks) {
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_HIP_CHECK(hipStreamSynchronize(r.stream(true)));
  }
  std::memcpy(all.data(), r0.xg_pin.p, br);
  return all;
}

// Host time of a phase of the one-thread driver (enqueue only: nothing here waits for the GPU
// unless the phase says so), recorded with rank 0's profile as "host_<phase>" when profiling is on.
struct HostClock {
  fm_ctx* m;
  const char* name;
  std::chrono::steady_clock::time_point t0;
  HostClock(Group& g, const char* n)
      : m(g.ranks[0].m->prof ? g.ranks[0].m : nullptr), name(n), t0(std::chrono::steady_clock::now()) {}
  ~HostClock() {
    if (m) m->prof_host(name, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};

void drop_route(Group& g, GroupBatch& gb);

// Split a host CSR by rows over the local ranks and upload each part into its member batch.
void upload_parts(Group& g, const fm_csr* c, GroupBatch& gb, bool check_range) {
  FM_REQUIRE(c != nullptr, "null fm_csr");
  FM_REQUIRE(c->n_rows >= 0 && c->nnz >= 0, "negative n_rows / nnz");
  FM_REQUIRE(c->n_rows == 0 || (c->row_ptr && c->label), "null row_ptr / label");
  const int64_t B = c->n_rows;
  if (B > 0) {
    FM_REQUIRE(c->row_ptr[0] == 0 && c->row_ptr[B] == c->nnz, "row_ptr must run from 0 to nnz");
    for (int64_t i = 0; i < B; ++i) FM_REQUIRE(c->row_ptr[i] <= c->row_ptr[i + 1], "row_ptr must be non-decreasing");
  } else {
    FM_REQUIRE(c->nnz == 0, "nnz > 0 with n_rows == 0");
  }
  drop_route(g, gb);  // a routed plan of the old contents is dropped before its buffers are reused
  gb.parts.resize(g.L);
  gb.rows = B;
  gb.nnz = c->nnz;
  gb.prefetched = false;
  std::vector<int64_t> rp;
  std::vector<std::vector<int64_t>> rows(g.L, std::vector<int64_t>(1));
  for (int l = 0; l < g.L; ++l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    const int64_t r0 = B * l / g.L, r1 = B * (l + 1) / g.L;
    const int64_t e0 = B > 0 ? c->row_ptr[r0] : 0, e1 = B > 0 ? c->row_ptr[r1] : 0;
    rp.resize(r1 - r0 + 1);
    for (int64_t i = r0; i <= r1; ++i) rp[i - r0] = B > 0 ? c->row_ptr[i] - e0 : 0;
    fm_csr sub{};
    sub.n_rows = r1 - r0;
    sub.nnz = e1 - e0;
    sub.row_ptr = rp.data();
    sub.col = c->col ? c->col + e0 : nullptr;
    sub.val = c->val ? c->val + e0 : nullptr;
    sub.label = c->label ? c->label + r0 : nullptr;
    if (!p.b) p.b = new fm_batch();
    p.device = r.device;
    on(r, [&] { upload_batch(r.m, &sub, p.b, check_range); });
    p.b->host_rp.assign(rp.begin(), rp.end());  // fm_batch_from_rows sizes selections of it on the host
    p.rows = sub.n_rows;
    p.row0 = r0;
    p.nnz = sub.nnz;
    rows[l][0] = p.rows;
  }
  const std::vector<int64_t> all = allgather(g, rows, 1);
  gb.global_rows = std::accumulate(all.begin(), all.end(), int64_t(0));
}

// A new group batch (an fm_batch whose parts are member batches).
fm_batch* new_group_batch(fm_ctx* ctx) {
  std::unique_ptr<fm_batch> b(new fm_batch());
  b->owner = ctx;
  b->device = ctx->cfg.device;
  b->grp.reset(new GroupBatch());
  return b.release();
}

void sync_group_batch_view(fm_batch* b) {  // fm_batch_rows / fm_batch_nnz of the group batch
  b->dev.n_rows = b->grp->rows;
  b->dev.nnz = b->grp->nnz;
}

// Sharded prepare, phase 1: every local rank's route (fm_shard.hip phase 1) on its side stream,
// then the job's route counts (ctx->sh_tot: [R] pairs, [R] entries per rank) gathered and copied
// to the batch's pinned buffer, rank-major [R][2R]: RCCL all-gathers them on the side streams and
// local rank 0 copies them back, COPY copies each rank's.  Nothing waits on the host.
void launch_routes(Group& g, GroupBatch& gb) {
  const int R = g.R, L = g.L;
  const size_t row = sizeof(unsigned long long) * 2 * R;
  g.each([&](int l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    ensure_on(r.device, p.send_slot, sizeof(uint32_t) * p.nnz);
    ensure_on(r.device, p.send_ent, sizeof(uint2) * p.nnz);
    on(r, [&] { shard_route_launch(r.m, p.b, p.send_slot.p, p.send_ent.p, r.m->side); });
  });
  gb.cnt_pin.ensure(row * R);
  if ((int)gb.ev_cnt.size() != L) {
    gb.ev_cnt.assign(L, nullptr);
    for (int l = 0; l < L; ++l) {
      FM_HIP_CHECK(hipSetDevice(g.ranks[l].device));
      FM_HIP_CHECK(hipEventCreateWithFlags(&gb.ev_cnt[l], hipEventDisableTiming));
    }
  }
  if (g.rccl) {
    for (auto& r : g.ranks) ensure_on(r.device, r.xg_recv, row * R);
    FM_RCCL_CHECK(ncclGroupStart());
    for (auto& r : g.ranks) {
      FM_HIP_CHECK(hipSetDevice(r.device));
      FM_RCCL_CHECK(ncclAllGather(r.m->sh_tot.p, r.xg_recv.p, 2 * R, ncclUint64, r.comm_side, r.m->side));
    }
    FM_RCCL_CHECK(ncclGroupEnd());
    Rank& r0 = g.ranks[0];
    FM_HIP_CHECK(hipSetDevice(r0.device));
    FM_HIP_CHECK(hipMemcpyAsync(gb.cnt_pin.p, r0.xg_recv.p, row * R, hipMemcpyDeviceToHost, r0.m->side));
  } else {
    for (auto& r : g.ranks) {
      FM_HIP_CHECK(hipSetDevice(r.device));
      FM_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<char*>(gb.cnt_pin.p) + row * r.global, r.m->sh_tot.p, row,
                                  hipMemcpyDeviceToHost, r.m->side));
    }
  }
  for (int l = 0; l < L; ++l) {
    FM_HIP_CHECK(hipSetDevice(g.ranks[l].device));
    FM_HIP_CHECK(hipEventRecord(gb.ev_cnt[l], g.ranks[l].m->side));
  }
  gb.routed = true;
}

// A routed batch whose plan is dropped (re-uploaded, or routed again for a transform): its route
// work must be done before its buffers are reused.
void drop_route(Group& g, GroupBatch& gb) {
  if (!gb.routed) return;
  for (size_t l = 0; l < gb.ev_cnt.size(); ++l) {
    FM_HIP_CHECK(hipSetDevice(g.ranks[l].device));
    FM_HIP_CHECK(hipEventSynchronize(gb.ev_cnt[l]));
  }
  gb.routed = false;
  if (g.pending == &gb) g.pending = nullptr;
}

// Sharded prepare, phase 2 (fm_shard.hip phase 1b): the host reads the job's counts (the one host
// wait, for route work enqueued an iteration earlier), then on the side streams the entry exchange
// and every owner's pair table and slot order.
void finish_routes(Group& g, GroupBatch& gb) {
  const int R = g.R, L = g.L;
  {
    HostClock hc(g, "host_prepare_wait");  // the host waiting for the route counts (GPU time, not host work)
    for (int l = 0; l < L; ++l) {
      FM_HIP_CHECK(hipSetDevice(g.ranks[l].device));
      FM_HIP_CHECK(hipEventSynchronize(gb.ev_cnt[l]));
    }
  }
  if (g.pending == &gb) g.pending = nullptr;
  gb.routed = false;
  const unsigned long long* rc = reinterpret_cast<const unsigned long long*>(gb.cnt_pin.p);  // [source][pairs | entries]
  std::vector<const char*> ss(L), se(L);
  std::vector<char*> rs(L), re(L);
  std::vector<const int64_t*> out(L), in(L);
  g.each([&](int l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    std::vector<int64_t> counts(2 * R);
    on(r, [&] { shard_route_finish(r.m, p.b, rc + (size_t)r.global * 2 * R, counts.data()); });
    plan::RouteCounts c = plan::route_counts(rc, R, r.global);
    p.ent_out = std::move(c.ent_out);
    p.pair_out = std::move(c.pair_out);
    p.ent_in = std::move(c.ent_in);
    p.pair_in = std::move(c.pair_in);
    const int64_t n_in = std::accumulate(p.ent_in.begin(), p.ent_in.end(), int64_t(0));
    if (R > 1) {
      ensure_on(g.ranks[l].device, p.recv_slot, sizeof(uint32_t) * n_in);
      ensure_on(g.ranks[l].device, p.recv_ent, sizeof(uint2) * n_in);
    }
    p.in_slot = R > 1 ? p.recv_slot.p : p.send_slot.p;  // R = 1: the owner block is the send buffers' head
    p.in_ent = R > 1 ? p.recv_ent.p : p.send_ent.p;
    ss[l] = p.send_slot.as<char>();
    se[l] = p.send_ent.as<char>();
    rs[l] = p.recv_slot.as<char>();
    re[l] = p.recv_ent.as<char>();
    out[l] = p.ent_out.data();
    in[l] = p.ent_in.data();
  });
  if (R > 1) a2a_multi(g, true, {A2ASeg{ss, rs, sizeof(uint32_t)}, A2ASeg{se, re, sizeof(uint2)}}, out, in);
  g.each([&](int l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    const int64_t n_in = std::accumulate(p.ent_in.begin(), p.ent_in.end(), int64_t(0));
    mcheck(fm_shard_owner_prepare(r.m, p.b, p.in_slot, p.in_ent, n_in, p.ent_in.data(), p.pair_in.data()),
           "fm_shard_owner_prepare");
  });
  gb.prefetched = true;
}

// The batch-only phases of a sharded iteration, both halves (what the step needs if the caller
// did not prepare the batch).
void prefetch(Group& g, GroupBatch& gb) {
  if (gb.prefetched) return;
  if (!gb.routed) launch_routes(g, gb);
  finish_routes(g, gb);
}

// the pair buffers of one direction in the wire layout: [P][kp] fp32 vectors, then [P][2] fp32
// scalars -- two all-to-alls with the same pair counts
void a2a_pairs(Group& g, int kp, const std::vector<DevBuf*>& send, const std::vector<int64_t>& sendP,
               const std::vector<DevBuf*>& recv, const std::vector<int64_t>& recvP,
               const std::vector<const int64_t*>& out, const std::vector<const int64_t*>& in) {
  const int L = g.L;
  std::vector<const char*> sv(L), sc(L);
  std::vector<char*> rv(L), rc(L);
  for (int l = 0; l < L; ++l) {
    sv[l] = send[l]->as<char>();
    sc[l] = send[l]->as<char>() + sizeof(float) * sendP[l] * kp;
    rv[l] = recv[l]->as<char>();
    rc[l] = recv[l]->as<char>() + sizeof(float) * recvP[l] * kp;
  }
  a2a_multi(g, false, {A2ASeg{sv, rv, sizeof(float) * kp}, A2ASeg{sc, rc, sizeof(float) * 2}}, out, in);
}

// per-step stats rows of the members (loss, loss rows, distinct ids) at epoch index e -> the job's
void stats_row(Group& g, int64_t e, double* h) {
  h[0] = h[1] = h[2] = 0.0;
  const int nsum = g.rccl ? 1 : g.L;  // RCCL: the rows were all-reduced in place after the step
  for (int l = 0; l < nsum; ++l) {
    Rank& r = g.ranks[l];
    double v[3];
    on(r, [&] {
      FM_HIP_CHECK(hipMemcpyAsync(v, r.m->loss_hist.as<double>() + 3 * e, sizeof(v), hipMemcpyDeviceToHost, r.m->stream));
      FM_HIP_CHECK(hipStreamSynchronize(r.m->stream));
    });
    h[0] += v[0];
    h[1] += v[1];
    if (g.sharded() || l == 0) h[2] += v[2];  // replicated: every replica counts the same touched rows
  }
}

// RCCL: the step's stats rows summed over the job in place (loss and loss rows; sharded also the
// distinct ids, each owned by exactly one rank), on the main streams after the step
void reduce_stats(Group& g, int64_t e) {
  if (!g.rccl) return;
  FM_RCCL_CHECK(ncclGroupStart());
  for (auto& r : g.ranks) {
    FM_HIP_CHECK(hipSetDevice(r.device));
    double* row = r.m->loss_hist.as<double>() + 3 * e;
    FM_RCCL_CHECK(ncclAllReduce(row, row, g.sharded() ? 3 : 2, ncclFloat64, ncclSum, r.comm_main, r.m->stream));
  }
  FM_RCCL_CHECK(ncclGroupEnd());
}

void fill_out(Group& g, fm_ctx* ctx, int64_t e, int64_t global_rows, fm_step_out* out) {
  if (!out) return;
  double h[3];
  stats_row(g, e, h);
  out->loss_sum = h[0];
  out->n_loss_rows = (int64_t)h[1];
  out->n_unique = (int64_t)h[2];
  out->n_rows = global_rows;
}


// Chunks of the owners' partial pass whose exchange overlaps the next chunk's compute
// (fm_config.xchg_chunks, default 4; 1 = one pass, then one all-to-all).  Only with R > 1.
int xchg_chunks(const Group& g) {
  if (g.R <= 1 || g.R > kMaxChunkSources) return 1;
  return g.xchg;
}

void ensure_xchg(Group& g) {
  for (auto& r : g.ranks) {
    if (r.xstream) continue;
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_HIP_CHECK(hipStreamCreateWithFlags(&r.xstream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&r.ev_x, &r.ev_fwd, &r.ev_xdone}) FM_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
}

// The owners' partial pass in C chunks, each chunk's partial rows sent to their requesters on the
// exchange stream while the next chunk is computed.  Chunk c of the P pairs of a (owner, requester)
// block is [P c / C, P (c + 1) / C) on both sides (the owner's pair_in[p] = the requester's pair_out[o]).
void forward_exchange_chunked(Group& g, GroupBatch& gb, int kp, int C, const std::vector<int64_t>& Pin,
                              const std::vector<int64_t>& Pout) {
  const int L = g.L, R = g.R;
  ensure_xchg(g);
  std::vector<const char*> sv(L), sc(L);
  std::vector<char*> rv(L), rc(L);
  for (int l = 0; l < L; ++l) {
    Rank& r = g.ranks[l];
    sv[l] = r.partials.as<char>();
    sc[l] = r.partials.as<char>() + sizeof(float) * Pin[l] * kp;
    rv[l] = r.part_in.as<char>();
    rc[l] = r.part_in.as<char>() + sizeof(float) * Pout[l] * kp;
  }
  for (int c = 0; c < C; ++c) {
    A2APlan pl;
    for (int l = 0; l < L; ++l) pl.add(plan::chunk(gb.parts[l].pair_in.data(), gb.parts[l].pair_out.data(), R, c, C));
    g.each([&](int l) {
      Rank& r = g.ranks[l];
      on(r, [&] {
        shard_owner_partials(r.m, gb.parts[l].b, r.partials.p, nullptr, c, C);
        FM_HIP_CHECK(hipEventRecord(r.ev_fwd, r.m->stream));
        FM_HIP_CHECK(hipStreamWaitEvent(r.xstream, r.ev_fwd, 0));
      });
    });
    a2a_plan(g, kLaneXchg, {A2ASeg{sv, rv, sizeof(float) * kp}, A2ASeg{sc, rc, sizeof(float) * 2}}, pl);
  }
  for (auto& r : g.ranks) {  // the combine reads what the exchange stream received
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_HIP_CHECK(hipEventRecord(r.ev_xdone, r.xstream));
    FM_HIP_CHECK(hipStreamWaitEvent(r.m->stream, r.ev_xdone, 0));
  }
}

int step_sharded(fm_ctx* ctx, Group& g, GroupBatch& gb, int32_t t, double step_size, double reg_param,
                 fm_step_out* out) {
  const int L = g.L, kp = ctx->kp, W = kp + 2;
  prefetch(g, gb);
  std::vector<int64_t> Pin(L), Pout(L);
  std::vector<DevBuf*> parts(L), part_in(L), s_send(L), s_recv(L);
  std::vector<const int64_t*> pin(L), pout(L);
  for (int l = 0; l < L; ++l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    Pin[l] = std::accumulate(p.pair_in.begin(), p.pair_in.end(), int64_t(0));
    Pout[l] = std::accumulate(p.pair_out.begin(), p.pair_out.end(), int64_t(0));
    ensure_on(r.device, r.partials, sizeof(float) * Pin[l] * W);
    ensure_on(r.device, r.s_send, sizeof(float) * Pout[l] * W);
    if (g.R > 1) {  // a one-rank job keeps its pairs where they were written (below)
      ensure_on(r.device, r.s_recv, sizeof(float) * Pin[l] * W);
      ensure_on(r.device, r.part_in, sizeof(float) * Pout[l] * W);
    }
    parts[l] = &r.partials;
    part_in[l] = &r.part_in;
    s_send[l] = &r.s_send;
    s_recv[l] = &r.s_recv;
    pin[l] = p.pair_in.data();
    pout[l] = p.pair_out.data();
  }
  // R = 1: the owner's pairs are its own batch's, in the same order (Pin = Pout), so the combine
  // reads the partials where the owner pass wrote them and the update the S rows where the combine
  // wrote them -- no self copy (as the entries, finish_routes)
  const bool self = g.R == 1;
  for (int l = 0; self && l < L; ++l) FM_REQUIRE(Pin[l] == Pout[l], "one-rank job: pair counts differ");
  const int C = xchg_chunks(g);
  {
    HostClock hc(g, "host_forward_xchg");
    if (C > 1) {
      forward_exchange_chunked(g, gb, kp, C, Pin, Pout);
    } else {
      // owners: partial sums per received pair
      g.each([&](int l) {
        mcheck(fm_shard_owner_forward(g.ranks[l].m, gb.parts[l].b, g.ranks[l].partials.p), "fm_shard_owner_forward");
      });
      // back to the requesters (owner l -> requester p: the pair_in[l][p] pairs it got from p)
      if (!self) a2a_pairs(g, kp, parts, Pin, part_in, Pout, pin, pout);
    }
  }
  {
    HostClock hc(g, "host_combine");
    g.each([&](int l) {
      Rank& r = g.ranks[l];
      mcheck(fm_shard_combine(r.m, gb.parts[l].b, (self ? r.partials : r.part_in).p, r.s_send.p), "fm_shard_combine");
    });
  }
  // S rows to the owners
  if (!self) {
    HostClock hc(g, "host_s_xchg");
    a2a_pairs(g, kp, s_send, Pout, s_recv, Pin, pout, pin);
  }
  {
    HostClock hc(g, "host_update");
    g.each([&](int l) {
      Rank& r = g.ranks[l];
      mcheck(fm_shard_owner_update(r.m, gb.parts[l].b, (self ? r.s_send : r.s_recv).p, t, step_size, reg_param,
                                   gb.global_rows),
             "fm_shard_owner_update");
    });
  }
  gb.prefetched = false;
  const int64_t e = g.ranks[0].m->epoch - 1;
  HostClock hc(g, "host_stats");
  reduce_stats(g, e);
  ctx->epoch = (int32_t)(e + 1);
  fill_out(g, ctx, e, gb.global_rows, out);
  return FM_OK;
}

int step_replicated(fm_ctx* ctx, Group& g, GroupBatch& gb, int32_t t, double step_size, double reg_param,
                    fm_step_out* out) {
  const int L = g.L;
  const int64_t n = g.ranks[0].m->rows * (int64_t)(ctx->kp + 4);
  {
    HostClock hc(g, "host_grad");
    g.each([&](int l) {
      Rank& r = g.ranks[l];
      ensure_on(r.device, r.grad, sizeof(float) * n);
      mcheck(fm_repl_grad(r.m, gb.parts[l].b, r.grad.p), "fm_repl_grad");
    });
  }
  HostClock hc_ar(g, "host_allreduce_apply");
  if (g.rccl) {
    FM_RCCL_CHECK(ncclGroupStart());
    for (auto& r : g.ranks) {
      FM_HIP_CHECK(hipSetDevice(r.device));
      FM_RCCL_CHECK(ncclAllReduce(r.grad.p, r.grad.p, n, ncclFloat32, ncclSum, r.comm_main, r.m->stream));
    }
    FM_RCCL_CHECK(ncclGroupEnd());
  } else if (L > 1) {
    // rank order sum on rank 0, then rank 0's sum to every rank: every replica applies the same bytes
    barrier(g, false);
    Rank& r0 = g.ranks[0];
    ensure_on(r0.device, r0.gtmp, sizeof(float) * n);
    for (int l = 1; l < L; ++l) {
      FM_HIP_CHECK(hipSetDevice(r0.device));
      FM_HIP_CHECK(hipMemcpyAsync(r0.gtmp.p, g.ranks[l].grad.p, sizeof(float) * n, hipMemcpyDefault, r0.m->stream));
      hipLaunchKernelGGL(k_add_f32, dim3(grid_of(n)), dim3(kBlock), 0, r0.m->stream, r0.grad.as<float>(),
                         r0.gtmp.as<float>(), n);
      FM_HIP_CHECK(hipGetLastError());
    }
    for (int l = 1; l < L; ++l)
      FM_HIP_CHECK(hipMemcpyAsync(g.ranks[l].grad.p, r0.grad.p, sizeof(float) * n, hipMemcpyDefault, r0.m->stream));
    barrier(g, false);
  }
  g.each([&](int l) {
    mcheck(fm_repl_apply(g.ranks[l].m, g.ranks[l].grad.p, t, step_size, reg_param, gb.global_rows), "fm_repl_apply");
  });
  const int64_t e = g.ranks[0].m->epoch - 1;
  reduce_stats(g, e);
  ctx->epoch = (int32_t)(e + 1);
  fill_out(g, ctx, e, gb.global_rows, out);
  return FM_OK;
}

int step_group_batch(fm_ctx* ctx, GroupBatch& gb, int32_t t, double step_size, double reg_param, fm_step_out* out) {
  Group& g = grp(ctx);
  if (gb.global_rows == 0) {  // SGD.scala:126-128: every rank of the job skips together
    if (out) {
      out->loss_sum = 0.0;
      out->n_rows = out->n_loss_rows = out->n_unique = 0;
    }
    return FM_NOTHING_TO_DO;
  }
  FM_REQUIRE(t >= 1, "iteration index t must be >= 1");
  FM_REQUIRE(std::isfinite(step_size) && std::isfinite(reg_param), "non-finite step size / regParam");
  return g.sharded() ? step_sharded(ctx, g, gb, t, step_size, reg_param, out)
                     : step_replicated(ctx, g, gb, t, step_size, reg_param, out);
}

// FactorizationMachinesModel.transform over a sharded table: route (ids outside the model
// dropped) -> entries to the owners -> owner partial sums with present counts -> back ->
// predict epilogue per sample.  pred: host [gb.rows].
void predict_sharded(fm_ctx* ctx, Group& g, GroupBatch& gb, double lo, double hi, double* pred) {
  const int L = g.L, kp = ctx->kp, W = kp + 2;
  gb.prefetched = false;  // the route below replaces any pending training plan of this batch
  prefetch(g, gb);
  gb.prefetched = false;
  std::vector<int64_t> Pin(L), Pout(L);
  std::vector<DevBuf*> parts(L), part_in(L);
  std::vector<const int64_t*> pin(L), pout(L);
  std::vector<const char*> cs(L);
  std::vector<char*> cr(L);
  for (int l = 0; l < L; ++l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    Pin[l] = std::accumulate(p.pair_in.begin(), p.pair_in.end(), int64_t(0));
    Pout[l] = std::accumulate(p.pair_out.begin(), p.pair_out.end(), int64_t(0));
    ensure_on(r.device, r.partials, sizeof(float) * Pin[l] * W);
    ensure_on(r.device, r.part_in, sizeof(float) * Pout[l] * W);
    ensure_on(r.device, r.pc_out, sizeof(uint32_t) * Pin[l]);
    ensure_on(r.device, r.pc_in, sizeof(uint32_t) * Pout[l]);
    ensure_on(r.device, r.pred, sizeof(double) * p.rows);
    parts[l] = &r.partials;
    part_in[l] = &r.part_in;
    pin[l] = p.pair_in.data();
    pout[l] = p.pair_out.data();
    cs[l] = r.pc_out.as<char>();
    cr[l] = r.pc_in.as<char>();
    on(r, [&] { shard_owner_partials(r.m, p.b, r.partials.p, r.pc_out.as<uint32_t>()); });
  }
  a2a_pairs(g, kp, parts, Pin, part_in, Pout, pin, pout);
  a2a(g, false, cs, cr, pin, pout, sizeof(uint32_t));
  for (int l = 0; l < L; ++l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    on(r, [&] {
      shard_combine_predict(r.m, p.b, r.part_in.p, r.pc_in.as<uint32_t>(), lo, hi, r.pred.as<double>());
      if (p.rows > 0)
        FM_HIP_CHECK(hipMemcpyAsync(pred + p.row0, r.pred.p, sizeof(double) * p.rows, hipMemcpyDeviceToHost, r.m->stream));
    });
  }
  for (auto& r : g.ranks) on(r, [&] { FM_HIP_CHECK(hipStreamSynchronize(r.m->stream)); });
}

void predict_group_batch(fm_ctx* ctx, GroupBatch& gb, double lo, double hi, double* pred) {
  Group& g = grp(ctx);
  if (gb.rows == 0) return;
  FM_REQUIRE(pred != nullptr, "null argument");
  if (g.sharded()) {
    predict_sharded(ctx, g, gb, lo, hi, pred);
    return;
  }
  for (int l = 0; l < g.L; ++l)
    if (gb.parts[l].rows > 0)
      mcheck(fm_predict_batch(g.ranks[l].m, gb.parts[l].b, lo, hi, pred + gb.parts[l].row0), "fm_predict_batch");
}

fm_batch* host_slot(fm_ctx* ctx) {
  Group& g = grp(ctx);
  auto& h = g.host_b[g.hnext];
  g.hnext ^= 1;
  if (!h) h.reset(new_group_batch(ctx));
  return h.get();
}

}  // namespace

// ------------------------------------------------------------------------------ entry points
int group_create(const fm_config* cfg, fm_ctx** out) {
  FM_REQUIRE(cfg->parallel == FM_PARALLEL_SHARDED || cfg->parallel == FM_PARALLEL_REPLICATED, "bad parallel mode");
  FM_REQUIRE(cfg->n_gpus >= 1 && cfg->n_gpus <= FM_MAX_LOCAL, "n_gpus must be in [1, FM_MAX_LOCAL]");
  FM_REQUIRE(cfg->n_procs >= 1 && cfg->proc_rank >= 0 && cfg->proc_rank < cfg->n_procs, "bad n_procs / proc_rank");
  const int L = cfg->n_gpus, R = cfg->n_procs * cfg->n_gpus;
  FM_REQUIRE(cfg->parallel != FM_PARALLEL_SHARDED || R <= 64, "the sharded step supports at most 64 ranks");
  FM_REQUIRE(cfg->xchg_chunks >= 0 && cfg->xchg_chunks <= 64, "xchg_chunks must be in [0, 64]");
  bool repeat = false;
  for (int a = 0; a < L; ++a)
    for (int b = a + 1; b < L; ++b) repeat = repeat || cfg->devices[a] == cfg->devices[b];
  int transport = cfg->transport;
  if (transport == FM_TRANSPORT_AUTO) transport = (repeat && cfg->n_procs == 1) ? FM_TRANSPORT_COPY : FM_TRANSPORT_RCCL;
  FM_REQUIRE(transport == FM_TRANSPORT_RCCL || transport == FM_TRANSPORT_COPY, "bad transport");
  FM_REQUIRE(transport != FM_TRANSPORT_COPY || cfg->n_procs == 1, "the copy transport needs one process");
  FM_REQUIRE(transport != FM_TRANSPORT_RCCL || !repeat, "RCCL needs a distinct device per rank");
  std::unique_ptr<fm_ctx> c(new fm_ctx());
  c->cfg = *cfg;
  c->cfg.device = cfg->devices[0];
  c->kp = (cfg->k + 3) / 4 * 4;
  c->rows = 0;
  c->group.reset(new Group());
  Group& g = *c->group;
  g.mode = cfg->parallel;
  g.L = L;
  g.R = R;
  g.nprocs = cfg->n_procs;
  g.prank = cfg->proc_rank;
  g.rccl = transport == FM_TRANSPORT_RCCL;
  g.xchg = cfg->xchg_chunks > 0 ? cfg->xchg_chunks : 4;
  g.ranks.resize(L);
  for (int l = 0; l < L; ++l) {
    Rank& r = g.ranks[l];
    r.device = cfg->devices[l];
    r.global = cfg->proc_rank * L + l;
    fm_config mc = *cfg;
    mc.parallel = FM_PARALLEL_NONE;
    mc.n_gpus = 1;
    mc.device = r.device;
    mc.shard_index = g.sharded() ? r.global : 0;
    mc.shard_count = g.sharded() ? R : 1;
    // a replica's batches feed fm_repl_grad, which needs the whole sorted view (no singleton split)
    if (!g.sharded()) mc.fuse_single = FM_FUSE_OFF;
    mcheck(fm_create(&mc, &r.m), "fm_create (member)");
    FM_HIP_CHECK(hipSetDevice(r.device));
    FM_HIP_CHECK(hipEventCreateWithFlags(&r.ev_main, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventCreateWithFlags(&r.ev_side, hipEventDisableTiming));
  }
  for (auto& a : g.ranks)  // peer access between the distinct devices (copies, RCCL's P2P)
    for (auto& b : g.ranks)
      if (a.device != b.device) {
        FM_HIP_CHECK(hipSetDevice(a.device));
        const hipError_t e = hipDeviceEnablePeerAccess(b.device, 0);
        if (e != hipSuccess) (void)hipGetLastError();  // already enabled, or no P2P: copies stage
      }
  if (g.rccl) {
    ncclUniqueId id;
    static_assert(sizeof(id) == sizeof(cfg->comm_id), "ncclUniqueId is 128 bytes");
    if (cfg->n_procs == 1) FM_RCCL_CHECK(ncclGetUniqueId(&id));
    else std::memcpy(&id, cfg->comm_id, sizeof(id));
    FM_RCCL_CHECK(ncclGroupStart());
    for (auto& r : g.ranks) {
      FM_HIP_CHECK(hipSetDevice(r.device));
      FM_RCCL_CHECK(ncclCommInitRank(&r.comm_main, R, id, r.global));
    }
    FM_RCCL_CHECK(ncclGroupEnd());
    for (ncclComm_t Rank::*dst : {&Rank::comm_side, &Rank::comm_x}) {
      FM_RCCL_CHECK(ncclGroupStart());
      for (auto& r : g.ranks) {
        FM_HIP_CHECK(hipSetDevice(r.device));
        FM_RCCL_CHECK(ncclCommSplit(r.comm_main, 0, r.global, &(r.*dst), nullptr));
      }
      FM_RCCL_CHECK(ncclGroupEnd());
    }
  }
  g.workers.start(L);
  *out = c.release();
  return FM_OK;
}

fm_ctx* group_member0(fm_ctx* ctx) { return grp(ctx).ranks[0].m; }

int group_batch_create(fm_ctx* ctx, const fm_csr* csr, fm_batch** out) {
  FM_REQUIRE(out != nullptr, "null out");
  std::unique_ptr<fm_batch> b(new_group_batch(ctx));
  upload_parts(grp(ctx), csr, *b->grp, true);
  sync_group_batch_view(b.get());
  *out = b.release();
  return FM_OK;
}

namespace {

// Local rank l's full copy of the group batch dg (its parts copied from every rank's device), rows in
// the dataset's order: the source of that rank's fm_batch_from_rows gathers.  A dataset made by
// fm_batch_create_splits holds split s of the dataset as every rank's share of it (rank 0's rows of
// split s, then rank 1's, ...: group_batch_create_splits), so its copy is assembled split by split,
// rank by rank, and row i of the copy is row i of the caller's CSR.  Made once per dataset.
fm_batch* dataset_replica(Group& g, GroupBatch& dg, int l, const std::vector<int64_t>& split_rows) {
  if ((int)dg.full.size() != g.L) dg.full.assign(g.L, nullptr);
  if (dg.full[l]) return dg.full[l];
  Rank& r = g.ranks[l];
  std::unique_ptr<fm_batch> f(new fm_batch());
  f->owner = r.m;
  f->device = r.device;
  const int64_t B = dg.rows, N = dg.nnz;
  // the dataset's rows as segments {part, first row, end row} of the parts, in dataset order
  struct Seg {
    int part;
    int64_t a, z;
  };
  std::vector<Seg> segs;
  const int ns = split_rows.empty() ? 1 : (int)split_rows.size() - 1;
  for (int sp = 0; sp < ns; ++sp) {
    for (int q = 0; q < (int)dg.parts.size(); ++q) {
      const GPart& pq = dg.parts[q];
      FM_REQUIRE((int64_t)pq.b->host_rp.size() == pq.rows + 1, "group dataset part without its host row_ptr");
      if (split_rows.empty()) {
        segs.push_back({q, 0, pq.rows});
      } else {
        const std::vector<int64_t>& msr = pq.b->split_rows;
        FM_REQUIRE((int)msr.size() == ns + 1, "group dataset part without its split boundaries");
        segs.push_back({q, msr[sp], msr[sp + 1]});
      }
    }
  }
  std::vector<int64_t> rp;
  rp.reserve(B + 1);
  int64_t off = 0, mx = -1;
  for (const Seg& sg : segs) {
    const std::vector<int64_t>& hrp = dg.parts[sg.part].b->host_rp;
    for (int64_t i = sg.a; i < sg.z; ++i) rp.push_back(off + hrp[i] - hrp[sg.a]);
    off += hrp[sg.z] - hrp[sg.a];
  }
  for (const GPart& q : dg.parts) mx = std::max(mx, q.b->max_id);
  rp.push_back(off);
  FM_REQUIRE(off == N && (int64_t)rp.size() == B + 1, "group dataset parts do not add up");
  on(r, [&] {
    f->dev.n_rows = B;
    f->dev.nnz = N;
    f->max_id = mx;
    f->dev.row_ptr.ensure(sizeof(int64_t) * (B + 1));
    f->dev.col.ensure(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
    f->dev.xs.ensure(sizeof(float) * std::max<int64_t>(N, 4) + 16);
    f->dev.label.ensure(sizeof(double) * std::max<int64_t>(B, 4) + 16);
    FM_HIP_CHECK(hipMemcpy(f->dev.row_ptr.p, rp.data(), sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice));
    int64_t e = 0, row = 0;
    for (const Seg& sg : segs) {
      const GPart& q = dg.parts[sg.part];
      const int64_t e0 = q.b->host_rp[sg.a], ne = q.b->host_rp[sg.z] - e0, nr = sg.z - sg.a;
      if (ne > 0) {
        FM_HIP_CHECK(hipMemcpyPeer(f->dev.col.as<uint32_t>() + e, r.device, q.b->dev.col.as<uint32_t>() + e0, q.device,
                                   sizeof(uint32_t) * ne));
        FM_HIP_CHECK(hipMemcpyPeer(f->dev.xs.as<float>() + e, r.device, q.b->dev.xs.as<float>() + e0, q.device,
                                   sizeof(float) * ne));
      }
      if (nr > 0)
        FM_HIP_CHECK(hipMemcpyPeer(f->dev.label.as<double>() + row, r.device, q.b->dev.label.as<double>() + sg.a,
                                   q.device, sizeof(double) * nr));
      e += ne;
      row += nr;
    }
  });
  f->host_rp.swap(rp);
  dg.full[l] = f.release();
  return dg.full[l];
}

}  // namespace

int group_batch_from_rows(fm_ctx* ctx, const fm_batch* data, const int64_t* rows, int64_t n, fm_batch** out) {
  Group& g = grp(ctx);
  FM_REQUIRE(data != nullptr && data->owner == ctx && data->grp, "data belongs to another context");
  GroupBatch& dg = *const_cast<fm_batch*>(data)->grp;
  for (int64_t i = 0; i < n; ++i) FM_REQUIRE(rows[i] >= 0 && rows[i] < dg.rows, "row index out of [0, rows of data)");
  std::unique_ptr<fm_batch> fresh;
  fm_batch* b = *out;
  if (!b) {
    fresh.reset(new_group_batch(ctx));
    b = fresh.get();
  }
  FM_REQUIRE(b->owner == ctx && b->grp && b != data && b->split_rows.empty(),
             "out must be a batch of this context other than data");
  GroupBatch& gb = *b->grp;
  drop_route(g, gb);  // a routed plan of the old contents is dropped before its buffers are reused
  // a former dataset refilled as a selection: its per-rank full copies describe the old contents
  for (fm_batch* f : gb.full)
    if (f) fm_batch_destroy(f);
  gb.full.clear();
  gb.parts.resize(g.L);
  gb.prefetched = false;
  gb.rows = n;
  gb.nnz = 0;
  std::vector<std::vector<int64_t>> cnt(g.L, std::vector<int64_t>(1));
  for (int l = 0; l < g.L; ++l) {
    Rank& r = g.ranks[l];
    GPart& p = gb.parts[l];
    const int64_t r0 = n * l / g.L, r1 = n * (l + 1) / g.L;  // the split's rows by rows, as upload_parts
    fm_batch* src = dataset_replica(g, dg, l, data->split_rows);
    mcheck(fm_batch_from_rows(r.m, src, rows + r0, r1 - r0, &p.b), "fm_batch_from_rows");
    p.device = r.device;
    p.rows = r1 - r0;
    p.row0 = r0;
    p.nnz = fm_batch_nnz(p.b);
    gb.nnz += p.nnz;
    cnt[l][0] = p.rows;
  }
  // the global miniBatchSize: this process's rows, or every process's (one host wait for the counts)
  if (g.nprocs == 1) {
    gb.global_rows = n;
  } else {
    const std::vector<int64_t> all = allgather(g, cnt, 1);
    gb.global_rows = std::accumulate(all.begin(), all.end(), int64_t(0));
  }
  sync_group_batch_view(b);
  if (fresh) *out = fresh.release();
  return FM_OK;
}

// A dataset laid out split by split (fm_batch_create_splits): local rank l holds its share of every
// split -- the split's rows by rows over the local ranks, as a host CSR's are (upload_parts) -- as a
// member dataset with the same number of splits, so split s of the group dataset is every rank's
// split s (group_batch_split_view).
int group_batch_create_splits(fm_ctx* ctx, const fm_csr* c, int32_t n_splits, const int64_t* split_rows,
                              fm_batch** out) {
  Group& g = grp(ctx);
  FM_REQUIRE(c->n_rows >= 0 && c->nnz >= 0, "negative n_rows / nnz");
  FM_REQUIRE(c->n_rows == 0 || (c->row_ptr && c->label), "null row_ptr / label");
  FM_REQUIRE(c->nnz == 0 || (c->col && c->val), "null col / val");
  const int64_t B = c->n_rows;
  if (B > 0) {
    FM_REQUIRE(c->row_ptr[0] == 0 && c->row_ptr[B] == c->nnz, "row_ptr must run from 0 to nnz");
    for (int64_t i = 0; i < B; ++i) FM_REQUIRE(c->row_ptr[i] <= c->row_ptr[i + 1], "row_ptr must be non-decreasing");
  } else {
    FM_REQUIRE(c->nnz == 0, "nnz > 0 with n_rows == 0");
  }
  std::unique_ptr<fm_batch> b(new_group_batch(ctx));
  GroupBatch& gb = *b->grp;
  gb.parts.resize(g.L);
  gb.rows = B;
  gb.nnz = c->nnz;
  std::vector<std::vector<int64_t>> rows(g.L, std::vector<int64_t>(1));
  std::vector<int64_t> rp, msr;
  std::vector<int32_t> col;
  std::vector<double> val, lab;
  for (int l = 0; l < g.L; ++l) {
    rp.assign(1, 0);
    msr.assign(1, 0);
    col.clear();
    val.clear();
    lab.clear();
    for (int32_t s = 0; s < n_splits; ++s) {
      const int64_t ns = split_rows[s + 1] - split_rows[s];
      const int64_t a = split_rows[s] + ns * l / g.L, z = split_rows[s] + ns * (l + 1) / g.L;
      for (int64_t i = a; i < z; ++i) {
        lab.push_back(c->label[i]);
        col.insert(col.end(), c->col + c->row_ptr[i], c->col + c->row_ptr[i + 1]);
        val.insert(val.end(), c->val + c->row_ptr[i], c->val + c->row_ptr[i + 1]);
        rp.push_back((int64_t)col.size());
      }
      msr.push_back((int64_t)lab.size());
    }
    fm_csr sub{};
    sub.n_rows = (int64_t)lab.size();
    sub.nnz = (int64_t)col.size();
    sub.row_ptr = rp.data();
    sub.col = col.data();
    sub.val = val.data();
    sub.label = lab.data();
    GPart& p = gb.parts[l];
    mcheck(fm_batch_create_splits(g.ranks[l].m, &sub, n_splits, msr.data(), &p.b), "fm_batch_create_splits");
    p.device = g.ranks[l].device;
    p.rows = sub.n_rows;
    p.row0 = 0;  // its rows are not one range of the dataset (the dataset is not predicted as a whole)
    p.nnz = sub.nnz;
    rows[l][0] = p.rows;
  }
  const std::vector<int64_t> all = allgather(g, rows, 1);
  gb.global_rows = std::accumulate(all.begin(), all.end(), int64_t(0));
  b->split_rows.assign(split_rows, split_rows + n_splits + 1);
  sync_group_batch_view(b.get());
  *out = b.release();
  return FM_OK;
}

// Split s of a group dataset: every local rank's view of its own share (fm_batch_split_view); no copy.
int group_batch_split_view(fm_ctx* ctx, const fm_batch* data, int32_t split, fm_batch** out) {
  Group& g = grp(ctx);
  FM_REQUIRE(data->grp && !data->split_rows.empty(), "data must be a dataset made by fm_batch_create_splits");
  FM_REQUIRE(split >= 0 && split + 1 < (int32_t)data->split_rows.size(), "split index out of range");
  const GroupBatch& dg = *data->grp;
  std::unique_ptr<fm_batch> fresh;
  fm_batch* b = *out;
  if (!b) {
    fresh.reset(new_group_batch(ctx));
    b = fresh.get();
  }
  FM_REQUIRE(b->owner == ctx && b->grp && b != data && b->split_rows.empty(),
             "out must be a batch of this context other than data");
  GroupBatch& gb = *b->grp;
  drop_route(g, gb);  // a routed plan of the old contents is dropped before the parts change
  for (fm_batch* f : gb.full)
    if (f) fm_batch_destroy(f);
  gb.full.clear();
  gb.parts.resize(g.L);
  gb.prefetched = false;
  const int64_t n = data->split_rows[split + 1] - data->split_rows[split];
  gb.rows = n;
  gb.nnz = 0;
  std::vector<std::vector<int64_t>> cnt(g.L, std::vector<int64_t>(1));
  for (int l = 0; l < g.L; ++l) {
    GPart& p = gb.parts[l];
    mcheck(fm_batch_split_view(g.ranks[l].m, dg.parts[l].b, split, &p.b), "fm_batch_split_view");
    p.device = g.ranks[l].device;
    p.rows = fm_batch_rows(p.b);
    p.row0 = n * l / g.L;  // as group_batch_create_splits cut the split
    p.nnz = fm_batch_nnz(p.b);
    gb.nnz += p.nnz;
    cnt[l][0] = p.rows;
  }
  if (g.nprocs == 1) {
    gb.global_rows = n;
  } else {
    const std::vector<int64_t> all = allgather(g, cnt, 1);
    gb.global_rows = std::accumulate(all.begin(), all.end(), int64_t(0));
  }
  sync_group_batch_view(b);
  if (fresh) *out = fresh.release();
  return FM_OK;
}

int group_batch_prepare(fm_ctx* ctx, fm_batch* b) {
  Group& g = grp(ctx);
  GroupBatch& gb = gbatch(ctx, b);
  FM_REQUIRE(b->split_rows.empty(), "a dataset made by fm_batch_create_splits is prepared through its split views");
  if (g.sharded()) {
    // phase 2 of the batch prepared before this one (its routes ran beside the steps enqueued
    // since), then phase 1 of this one: the host waits only for route work an iteration old
    if (g.pending && g.pending != &gb) {
      HostClock hc(g, "host_prepare_finish");  // waits for route counts an iteration old
      finish_routes(g, *g.pending);
    }
    if (!gb.prefetched && !gb.routed) {
      HostClock hc(g, "host_prepare_route");
      launch_routes(g, gb);
      gb.g = &g;
      g.pending = &gb;
    }
  } else {
    for (int l = 0; l < g.L; ++l) mcheck(fm_batch_prepare(g.ranks[l].m, gb.parts[l].b), "fm_batch_prepare");
  }
  return FM_OK;
}

int group_step_batch(fm_ctx* ctx, fm_batch* b, int32_t t, double step_size, double reg_param, fm_step_out* out) {
  FM_REQUIRE(b == nullptr || b->split_rows.empty(),
             "a dataset made by fm_batch_create_splits is stepped through its split views");
  return step_group_batch(ctx, gbatch(ctx, b), t, step_size, reg_param, out);
}

int group_step(fm_ctx* ctx, const fm_csr* csr, int32_t t, double step_size, double reg_param, fm_step_out* out) {
  fm_batch* b = host_slot(ctx);
  upload_parts(grp(ctx), csr, *b->grp, true);
  sync_group_batch_view(b);
  return step_group_batch(ctx, *b->grp, t, step_size, reg_param, out);
}

int group_predict(fm_ctx* ctx, const fm_csr* csr, double lo, double hi, double* pred) {
  FM_REQUIRE(csr != nullptr && (csr->n_rows == 0 || pred), "null argument");
  fm_batch* b = host_slot(ctx);
  upload_parts(grp(ctx), csr, *b->grp, false);
  sync_group_batch_view(b);
  predict_group_batch(ctx, *b->grp, lo, hi, pred);
  return FM_OK;
}

int group_predict_batch(fm_ctx* ctx, fm_batch* b, double lo, double hi, double* pred) {
  FM_REQUIRE(b == nullptr || b->split_rows.empty(), "a dataset made by fm_batch_create_splits is predicted by split");
  predict_group_batch(ctx, gbatch(ctx, b), lo, hi, pred);
  return FM_OK;
}

int group_load_tables(fm_ctx* ctx, const int32_t* ids, int64_t n, const double* w, const double* V) {
  for (auto& r : grp(ctx).ranks) mcheck(fm_load_tables(r.m, ids, n, w, V), "fm_load_tables");
  return FM_OK;
}

int group_init_random(fm_ctx* ctx, const int32_t* ids, int64_t n, int64_t id_begin, int64_t id_end) {
  for (auto& r : grp(ctx).ranks) {
    if (ids) mcheck(fm_init_random(r.m, ids, n), "fm_init_random");
    else mcheck(fm_init_random_range(r.m, id_begin, id_end), "fm_init_random_range");
  }
  return FM_OK;
}

int group_init_from_batch(fm_ctx* ctx, fm_batch* b, int64_t* n_present) {
  Group& g = grp(ctx);
  GroupBatch& gb = gbatch(ctx, b);
  if (g.sharded() && !b->split_rows.empty()) {
    // a dataset laid out by splits: its entries' sample indices count from their split's first row,
    // so the owner routing runs split by split (the draw depends on (seed, id, factor) only).  Every
    // split is routed, also one with no entries in this process: the routing's exchanges are
    // collectives of the whole job, and another process may hold entries of that split
    fm_batch* v = nullptr;
    for (int32_t s = 0; s + 1 < (int32_t)b->split_rows.size(); ++s) {
      group_batch_split_view(ctx, b, s, &v);
      group_init_from_batch(ctx, v, nullptr);
    }
    if (v) {
      group_sync(ctx);
      fm_batch_destroy(v);
    }
    if (n_present) *n_present = group_num_present(ctx);
    return FM_OK;
  }
  if (g.sharded()) {
    // createInitialModel's distinct ids arrive at their owners through the step's own routing
    prefetch(g, gb);
    for (int l = 0; l < g.L; ++l) {
      Rank& r = g.ranks[l];
      GPart& p = gb.parts[l];
      const int64_t n_in = std::accumulate(p.ent_in.begin(), p.ent_in.end(), int64_t(0));
      if (n_in == 0) continue;
      on(r, [&] {
        FM_HIP_CHECK(hipStreamSynchronize(r.m->side));
        DevBuf ids;
        ids.ensure(sizeof(uint32_t) * n_in);
        hipLaunchKernelGGL(k_slots_to_ids, dim3(grid_of(n_in)), dim3(kBlock), 0, r.m->stream,
                           static_cast<const uint32_t*>(p.in_slot), n_in, (uint32_t)g.R, (uint32_t)r.global,
                           ids.as<uint32_t>());
        launch_init_entries(r.m->view(), ids.as<uint32_t>(), n_in, r.m->cfg.seed, r.m->cfg.init_sd, r.m->epoch,
                            r.m->cum_host.back(), r.m->stream);
        FM_HIP_CHECK(hipStreamSynchronize(r.m->stream));
        ids.release();
      });
    }
  } else {
    FM_REQUIRE(g.nprocs == 1, "replicated fm_init_from_batch needs one process (use fm_init_random_range)");
    // every replica draws every id of every part (the draw depends on (seed, id, factor) only)
    for (auto& r : g.ranks)
      for (auto& p : gb.parts) {
        if (p.nnz == 0) continue;
        on(r, [&] {
          DevBuf col;
          col.ensure(sizeof(uint32_t) * p.nnz);
          FM_HIP_CHECK(hipMemcpyAsync(col.p, p.b->dev.col.p, sizeof(uint32_t) * p.nnz, hipMemcpyDefault, r.m->stream));
          launch_init_entries(r.m->view(), col.as<uint32_t>(), p.nnz, r.m->cfg.seed, r.m->cfg.init_sd, r.m->epoch,
                              r.m->cum_host.back(), r.m->stream);
          FM_HIP_CHECK(hipStreamSynchronize(r.m->stream));
          col.release();
        });
      }
  }
  if (n_present) *n_present = group_num_present(ctx);
  return FM_OK;
}

int64_t group_num_present(fm_ctx* ctx) {
  Group& g = grp(ctx);
  int64_t tot = 0;
  for (int l = 0; l < (g.sharded() ? g.L : 1); ++l) {
    const int64_t n = fm_num_present(g.ranks[l].m);
    mcheck((int)std::min<int64_t>(n, 0), "fm_num_present");
    tot += n;
  }
  return tot;
}

int group_export_tables(fm_ctx* ctx, int32_t* ids, double* w, double* V, int64_t cap, int64_t* n) {
  Group& g = grp(ctx);
  FM_REQUIRE(n != nullptr && cap >= 0, "bad arguments");
  if (!g.sharded()) return fm_export_tables(g.ranks[0].m, ids, w, V, cap, n);
  const int k = ctx->cfg.k;
  std::vector<int64_t> cnt(g.L);
  int64_t tot = 0;
  for (int l = 0; l < g.L; ++l) {
    mcheck(fm_export_tables(g.ranks[l].m, nullptr, nullptr, nullptr, 0, &cnt[l]), "fm_export_tables");
    tot += cnt[l];
  }
  *n = tot;
  if (cap == 0) return FM_OK;
  FM_REQUIRE(cap >= tot && ids && w && V, "export buffers too small or null");
  std::vector<int32_t> ai(tot);
  std::vector<double> aw(tot), aV((size_t)tot * k);
  int64_t o = 0;
  for (int l = 0; l < g.L; ++l) {
    int64_t got = 0;
    if (cnt[l])
      mcheck(fm_export_tables(g.ranks[l].m, ai.data() + o, aw.data() + o, aV.data() + o * k, cnt[l], &got),
             "fm_export_tables");
    o += cnt[l];
  }
  std::vector<int64_t> ord(tot);
  std::iota(ord.begin(), ord.end(), int64_t(0));
  std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return ai[a] < ai[b]; });
  for (int64_t i = 0; i < tot; ++i) {
    ids[i] = ai[ord[i]];
    w[i] = aw[ord[i]];
    std::memcpy(V + i * k, aV.data() + ord[i] * k, sizeof(double) * k);
  }
  return FM_OK;
}

int group_export_rows(fm_ctx* ctx, const int32_t* ids, int64_t n, double* w, double* V, int8_t* present) {
  Group& g = grp(ctx);
  if (!g.sharded()) return fm_export_rows(g.ranks[0].m, ids, n, w, V, present);
  FM_REQUIRE(n >= 0, "negative n");
  if (n == 0) return FM_OK;
  FM_REQUIRE(ids && w && V && present, "null argument");
  const int k = ctx->cfg.k;
  std::vector<std::vector<int64_t>> pos(g.L);
  for (int64_t i = 0; i < n; ++i) {
    FM_REQUIRE(ids[i] >= 0 && ids[i] < ctx->cfg.num_features, "id out of [0, num_features)");
    const int owner = (int)(ids[i] % g.R);
    const int l = owner - g.prank * g.L;
    FM_REQUIRE(l >= 0 && l < g.L, "id owned by a rank of another process");
    pos[l].push_back(i);
  }
  for (int l = 0; l < g.L; ++l) {
    const int64_t m = (int64_t)pos[l].size();
    if (m == 0) continue;
    std::vector<int32_t> si(m);
    std::vector<double> sw(m), sV((size_t)m * k);
    std::vector<int8_t> sp(m);
    for (int64_t j = 0; j < m; ++j) si[j] = ids[pos[l][j]];
    mcheck(fm_export_rows(g.ranks[l].m, si.data(), m, sw.data(), sV.data(), sp.data()), "fm_export_rows");
    for (int64_t j = 0; j < m; ++j) {
      const int64_t i = pos[l][j];
      w[i] = sw[j];
      present[i] = sp[j];
      std::memcpy(V + i * k, sV.data() + j * k, sizeof(double) * k);
    }
  }
  return FM_OK;
}

int group_loss_history(fm_ctx* ctx, double* loss, int64_t cap, int64_t* n) {
  Group& g = grp(ctx);
  FM_REQUIRE(n != nullptr, "null n");
  *n = ctx->epoch;
  if (cap == 0 || ctx->epoch == 0) return FM_OK;
  FM_REQUIRE(loss != nullptr, "null loss buffer");
  const int64_t m = std::min<int64_t>(cap, ctx->epoch);
  for (int64_t e = 0; e < m; ++e) {
    double h[3];
    stats_row(g, e, h);
    loss[e] = h[0];
  }
  return FM_OK;
}

int group_last_stats(fm_ctx* ctx, double* loss_sum, int64_t* n_loss_rows, int64_t* n_unique) {
  FM_REQUIRE(loss_sum && n_loss_rows && n_unique, "null argument");
  FM_REQUIRE(ctx->epoch >= 1, "no step executed");
  double h[3];
  stats_row(grp(ctx), ctx->epoch - 1, h);
  *loss_sum = h[0];
  *n_loss_rows = (int64_t)h[1];
  *n_unique = (int64_t)h[2];
  return FM_OK;
}

int group_sync(fm_ctx* ctx) {
  for (auto& r : grp(ctx).ranks)
    on(r, [&] {
      FM_HIP_CHECK(hipStreamSynchronize(r.m->stream));
      FM_HIP_CHECK(hipStreamSynchronize(r.m->side));
      if (r.m->copy_stream) FM_HIP_CHECK(hipStreamSynchronize(r.m->copy_stream));
      if (r.xstream) FM_HIP_CHECK(hipStreamSynchronize(r.xstream));
    });
  return FM_OK;
}

int group_reserve(fm_ctx* ctx, int64_t max_rows, int64_t max_nnz) {
  Group& g = grp(ctx);
  for (auto& r : g.ranks) mcheck(fm_reserve(r.m, max_rows / g.L + 1, max_nnz), "fm_reserve");
  return FM_OK;
}

// op 0: enable(on) on every rank; 1: reset every rank; 2: read local rank 0's per-phase times
int group_profile(fm_ctx* ctx, int op, int32_t on_, char* names, int64_t names_cap, double* total_ms,
                  int64_t* launches, int64_t cap, int64_t* n) {
  Group& g = grp(ctx);
  if (op == 2) return fm_profile_read(g.ranks[0].m, names, names_cap, total_ms, launches, cap, n);
  for (auto& r : g.ranks) {
    if (op == 0) mcheck(fm_profile_enable(r.m, on_), "fm_profile_enable");
    else mcheck(fm_profile_reset(r.m), "fm_profile_reset");
  }
  return FM_OK;
}

}  // namespace fmhip

extern "C" int fm_comm_unique_id(uint8_t* id) {
  return fmhip::guarded_free([&]() -> int {
    FM_REQUIRE(id != nullptr, "null id");
    ncclUniqueId u;
    FM_RCCL_CHECK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return FM_OK;
  });
}
