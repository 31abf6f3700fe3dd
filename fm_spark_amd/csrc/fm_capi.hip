// C-ABI implementation of include/fm_hip.h: contexts, device tables, mini-batch upload,
// the step driver (forward -> sort -> segmented update) and the table import/export.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <thread>
#include <utility>

#include "fm_context.h"
#include "fm_hostpool.h"

namespace fmhip {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

void report_stale(hipError_t e) {
  if (e == hipSuccess) return;
  static std::mutex mu;
  static std::set<int> seen;
  std::lock_guard<std::mutex> lk(mu);
  if (seen.insert((int)e).second)
    fprintf(stderr, "[libfm_hip] cleared a stale HIP error left by an earlier call: %d %s\n", (int)e, hipGetErrorString(e));
}

void DevBuf::ensure(size_t n) {
  if (n <= bytes && p) return;
  // growing: work already queued on any stream may still read the old buffer (asynchronous
  // steps), so the device drains before it is freed
  if (p) FM_HIP_CHECK(hipDeviceSynchronize());
  release();
  if (n == 0) n = 16;
  FM_HIP_CHECK(hipMalloc(&p, n));
  bytes = n;
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

// How many contiguous chunks parallel_chunks cuts [0, n) into (one per pool thread, at least
// min_per_thread items each).
static int64_t chunk_count(int64_t n, int64_t min_per_thread) {
  return std::max<int64_t>(1, std::min<int64_t>(HostPool::get().threads(), n / std::max<int64_t>(min_per_thread, 1)));
}

// f(t, lo, hi) for chunk t = [n t / T, n (t + 1) / T) of T chunks, on the pool's threads.
template <class F>
static void parallel_chunks_t(int64_t n, int64_t T, F&& f) {
  if (T <= 1) {
    f(int64_t(0), int64_t(0), n);
    return;
  }
  const std::function<void(int)> job = [&](int t) { f((int64_t)t, n * t / T, n * (t + 1) / T); };
  HostPool::get().run((int)T, job);
}

// f(lo, hi) over [0, n) in contiguous chunks on the pool's threads; small ranges run inline.
template <class F>
static void parallel_chunks(int64_t n, int64_t min_per_thread, F&& f) {
  parallel_chunks_t(n, chunk_count(n, min_per_thread), [&](int64_t, int64_t lo, int64_t hi) { f(lo, hi); });
}

// Host CSR -> pinned staging [row_ptr int64 B+1][label f64 B][xoff int32 B][col u32 N][x f32 N]:
// values that round to 1.0f (one-hot / categorical fields) are not sent -- the id's bit 31 (free:
// ids are non-negative int32) marks an entry whose fp32 value follows in the x area, and xoff[i]
// is where row i's values start; each host thread packs its rows' values from its first entry's
// position on, and only those runs are copied -- so 4 B per unit entry and 8 B per other entry
// cross PCIe.  The device rebuilds each entry's sample index and value (k_explode) into the exploded
// {sample, x} entries of Model.scala:148-153.  Validated on the way; host threads write the
// staging directly.  check_range: ids must be owned by this context's table (training); otherwise
// any non-negative int32 id is accepted (predict drops unknown ids).
struct Staged {
  int64_t B = 0, N = 0, M = 0, max_id = -1, max_len = 0;
  size_t o_lab = 0, o_xoff = 0, o_col = 0, o_x = 0, bytes = 0;  // bytes: the image through col
  int nruns = 0;
  int64_t run_at[16] = {0}, run_n[16] = {0};  // packed value runs in the x area (floats)
};

static Staged stage_csr(fm_ctx* ctx, const fm_csr* c, bool check_range, Pinned& pin) {
  FM_REQUIRE(c != nullptr, "null fm_csr");
  FM_REQUIRE(c->n_rows >= 0 && c->nnz >= 0, "negative n_rows / nnz");
  FM_REQUIRE(c->n_rows < (int64_t(1) << 31), "n_rows must be < 2^31");
  FM_REQUIRE(c->nnz < (int64_t(1) << 31), "nnz must be < 2^31 per batch");
  FM_REQUIRE(c->n_rows == 0 || (c->row_ptr && c->label), "null row_ptr / label");
  FM_REQUIRE(c->nnz == 0 || (c->col && c->val), "null col / val");
  Staged g;
  const int64_t B = c->n_rows, N = c->nnz;
  g.B = B;
  g.N = N;
  if (B > 0) {
    FM_REQUIRE(c->row_ptr[0] == 0, "row_ptr[0] must be 0");
    FM_REQUIRE(c->row_ptr[B] == N, "row_ptr[n_rows] must equal nnz");
    for (int64_t i = 0; i < B; ++i) FM_REQUIRE(c->row_ptr[i] <= c->row_ptr[i + 1], "row_ptr must be non-decreasing");
  } else {
    FM_REQUIRE(N == 0, "nnz > 0 with n_rows == 0");
  }
  g.o_lab = sizeof(int64_t) * (B + 1);
  g.o_xoff = g.o_lab + sizeof(double) * B;
  g.o_col = (g.o_xoff + sizeof(int32_t) * B + 15) / 16 * 16;
  g.o_x = (g.o_col + sizeof(uint32_t) * N + 15) / 16 * 16;
  pin.ensure_slack(g.o_x + sizeof(float) * N + 16);  // M <= N
  char* base = reinterpret_cast<char*>(pin.p);
  int64_t* rp = reinterpret_cast<int64_t*>(base);
  double* lab = reinterpret_cast<double*>(base + g.o_lab);
  int32_t* xoff = reinterpret_cast<int32_t*>(base + g.o_xoff);
  uint32_t* col = reinterpret_cast<uint32_t*>(base + g.o_col);
  float* xs = reinterpret_cast<float*>(base + g.o_x);
  if (B > 0) std::memcpy(rp, c->row_ptr, sizeof(int64_t) * (B + 1));
  else rp[0] = 0;
  const int64_t F = ctx->cfg.num_features;
  std::atomic<int> bad{0};  // 1 negative id, 2 id >= num_features
  std::atomic<int64_t> mx{-1}, mlen{0};
  // one pass over row chunks: ids (bit 31 = a value follows), labels, the chunk's values packed
  // from its first entry's position on
  std::atomic<int> nrun{0};
  parallel_chunks(B, 4096, [&](int64_t r0, int64_t r1) {
    const int64_t x0 = B > 0 ? c->row_ptr[r0] : 0;
    int64_t lmx = -1, m = x0, llen = 0;
    int lbad = 0;
    for (int64_t i = r0; i < r1; ++i) {
      lab[i] = c->label[i];  // Double, as the reference's label column (SGD.scala:145-146)
      llen = std::max<int64_t>(llen, c->row_ptr[i + 1] - c->row_ptr[i]);
      xoff[i] = (int32_t)m;
      for (int64_t e = c->row_ptr[i]; e < c->row_ptr[i + 1]; ++e) {
        const int32_t id = c->col[e];
        if (id < 0) lbad |= 1;
        else if (check_range && id >= F) lbad |= 2;
        const float x = (float)c->val[e];
        const uint32_t valued = x != 1.0f;
        col[e] = (uint32_t)id | (valued << 31);
        xs[m] = x;  // branch-free: the slot is taken only by a value that is not 1
        m += valued;
        lmx = std::max<int64_t>(lmx, id);
      }
    }
    const int ri = nrun.fetch_add(1);
    g.run_at[ri] = x0;
    g.run_n[ri] = m - x0;
    if (lbad) bad.fetch_or(lbad);
    int64_t cur = mx.load();
    while (lmx > cur && !mx.compare_exchange_weak(cur, lmx)) {
    }
    cur = mlen.load();
    while (llen > cur && !mlen.compare_exchange_weak(cur, llen)) {
    }
  });
  FM_REQUIRE(!(bad.load() & 1), "negative feature id");
  FM_REQUIRE(!(bad.load() & 2), "feature id >= num_features");
  g.nruns = nrun.load();
  for (int r = 0; r < g.nruns; ++r) g.M += g.run_n[r];
  g.bytes = g.o_col + sizeof(uint32_t) * N;
  g.max_id = mx.load();
  g.max_len = mlen.load();
  return g;
}

// The fused step (fm_kernels.hip "Singleton rows") for batches this context prepares: a
// single-table context with kp <= 16; by default (FM_FUSE_DEFAULT) only for a table larger than
// the 256-MB Infinity Cache, where the update's re-read of the singleton rows goes to HBM -- a
// cache-resident table re-reads them on-die, and the split and tags would cost more than they save
// (c2 / c5: 0.245 / 0.273 ms per step fused against 0.184 / 0.208 unfused, profiles/r03_v1).
bool fuse_rule(const fm_ctx* ctx) {
  if (ctx->cfg.fuse_single == FM_FUSE_OFF || ctx->kp > 16) return false;
  const double table_bytes = (double)ctx->rows * ctx->stride * sizeof(float);
  return ctx->cfg.fuse_single == FM_FUSE_ON || table_bytes > 256.0 * 1024 * 1024;
}

static bool fuse_on(const fm_ctx* ctx) { return ctx->cfg.shard_count == 1 && fuse_rule(ctx); }

static bool batch_fits(const fm_batch* b, const Staged& g) {
  return b->dev.row_ptr.bytes >= sizeof(int64_t) * (g.B + 1) &&
         b->dev.col.bytes >= sizeof(uint32_t) * std::max<int64_t>(g.N, 4) + 16 &&
         b->dev.ent.bytes >= sizeof(uint32_t) * 2 * std::max<int64_t>(g.N, 4) + 16 &&
         b->dev.xs.bytes >= sizeof(float) * std::max<int64_t>(g.N, 4) + 16 &&
         b->dev.label.bytes >= sizeof(double) * std::max<int64_t>(g.B, 4) + 16 &&
         b->up.bytes >= g.o_x + sizeof(float) * g.N + 16;
}

// b's device buffers (grown, never shrunk) filled from the staging by one async copy on st (into
// b->up, the staging's device image), then col / label / row_ptr and the exploded entries are
// laid out from it by one kernel pass on st.
static void copy_staged(fm_ctx* ctx, const Staged& g, const Pinned& pin, fm_batch* b, hipStream_t st) {
  const int64_t B = g.B, N = g.N;
  b->owner = ctx;
  b->device = ctx->cfg.device;
  b->max_id = g.max_id;
  b->dev.n_rows = B;
  b->dev.nnz = N;
  b->dev.row_ptr.ensure_slack(sizeof(int64_t) * (B + 1));
  b->dev.col.ensure_slack(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
  b->dev.ent.ensure_slack(sizeof(uint32_t) * 2 * std::max<int64_t>(N, 4) + 16);
  b->dev.xs.ensure_slack(sizeof(float) * std::max<int64_t>(N, 4) + 16);
  b->dev.label.ensure_slack(sizeof(double) * std::max<int64_t>(B, 4) + 16);
  b->up.ensure_slack(g.o_x + sizeof(float) * N + 16);
  FM_HIP_CHECK(hipMemcpyAsync(b->up.p, pin.p, g.bytes, hipMemcpyHostToDevice, st));
  for (int r = 0; r < g.nruns; ++r)  // the packed value runs, each where its rows' xoff point
    if (g.run_n[r] > 0)
      FM_HIP_CHECK(hipMemcpyAsync(b->up.as<char>() + g.o_x + sizeof(float) * g.run_at[r],
                                  reinterpret_cast<const char*>(pin.p) + g.o_x + sizeof(float) * g.run_at[r],
                                  sizeof(float) * g.run_n[r], hipMemcpyHostToDevice, st));
  const char* up = b->up.as<char>();
  launch_explode(reinterpret_cast<const int64_t*>(up), reinterpret_cast<const double*>(up + g.o_lab),
                 reinterpret_cast<const int32_t*>(up + g.o_xoff), reinterpret_cast<const uint32_t*>(up + g.o_col),
                 reinterpret_cast<const float*>(up + g.o_x), B, N, b->dev.row_ptr.as<int64_t>(),
                 b->dev.label.as<double>(), b->dev.col.as<uint32_t>(), b->dev.ent.as<uint2>(), b->dev.xs.as<float>(), st);
}

// Synchronous upload (fm_batch_create, fm_predict, fm_loss_grad): staged in the context's
// pinned buffer, copied on the context's stream, returns after the copies.
void upload_batch(fm_ctx* ctx, const fm_csr* c, fm_batch* b, bool check_range) {
  FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));  // the staging / b may still feed queued work
  const Staged g = stage_csr(ctx, c, check_range, ctx->up_pin);
  copy_staged(ctx, g, ctx->up_pin, b, ctx->stream);
  FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
}

// The context's reusable batch for the synchronous host-buffer entry points (fm_predict,
// fm_loss_grad): its device buffers persist across calls.
fm_batch* host_batch(fm_ctx* ctx) {
  if (!ctx->host_batch) ctx->host_batch.reset(new fm_batch());
  return ctx->host_batch.get();
}

// A batch refilled by fm_batch_from_rows is written on the side stream: a reader on stream st waits
// for that (a no-op for batches that were never refilled).
void wait_built(const fm_batch* b, hipStream_t st) {
  if (b->built) FM_HIP_CHECK(hipStreamWaitEvent(st, b->built, 0));
}

void reserve_work(fm_ctx* ctx, int64_t B, int64_t N) {
  StepWork& w = ctx->work;
  w.S.ensure_slack(sizeof(float) * (size_t)std::max<int64_t>(B, 1) * s_rec_floats(ctx->kp));
  w.yl.ensure_slack(sizeof(float2) * (size_t)std::max<int64_t>(B, 1));
  w.sort.ensure(std::max<int64_t>(N, 1));
  const int64_t nranges = (N + 255) / 256;  // update waves (fm_kernels.hip, kWaveEnt)
  w.part.ensure_slack(sizeof(double) * (size_t)std::max<int64_t>(nranges, 1) * 2 * (ctx->kp + 2));
  w.ucnt.ensure_slack(sizeof(uint32_t) * (size_t)std::max<int64_t>((N + 1023) / 1024, 1));
  w.loss_part.ensure(sizeof(double) * 2 * 256 * 8);
}

}  // namespace fmhip

namespace {

// One fused step.  emit != nullptr (replicated mode, fm_repl_grad): the per-slot gradient sums
// are written to emit[rows][kp + 4] instead of being applied, and the epoch does not advance.
int step_impl(fm_ctx* ctx, fm_batch* b, int32_t t, double step_size, double reg_param, fm_step_out* out,
              float* emit = nullptr) {
  FM_REQUIRE(b != nullptr, "null batch");
  FM_REQUIRE(b->owner == ctx, "batch belongs to another context");
  FM_REQUIRE(ctx->cfg.shard_count == 1, "sharded contexts step through the fm_shard_* entry points");
  FM_REQUIRE(b->split_rows.empty(), "a dataset made by fm_batch_create_splits is stepped through its split views");
  if (emit) FM_HIP_CHECK(hipMemsetAsync(emit, 0, sizeof(float) * (size_t)ctx->rows * (ctx->kp + 4), ctx->stream));
  if (b->dev.n_rows == 0) return FM_NOTHING_TO_DO;  // SGD.scala:126-128
  FM_REQUIRE(t >= 1, "iteration index t must be >= 1");
  FM_REQUIRE(std::isfinite(step_size) && std::isfinite(reg_param), "non-finite step size / regParam");
  const int64_t B = b->dev.n_rows, N = b->dev.nnz;
  reserve_work(ctx, B, N);
  ctx->ensure_hist(ctx->epoch + 1);
  StepParams p;
  p.n_rows = B;
  p.eta = step_size / std::sqrt((double)t);  // SGD.scala:121
  p.lam = p.eta * reg_param;                 // SGD.scala:122
  p.m = (double)B;                           // miniBatchSize, SGD.scala:124
  p.scale_v = p.eta / (double)B;             // currentStepSize / miniBatchSize, SGD.scala:153
  p.epoch = ctx->epoch;
  p.cumE = ctx->cum_host.back();
  p.cum_next = p.cumE + p.lam;
  p.w0 = ctx->cfg.w0;
  const TableView T = ctx->view();
  wait_built(b, ctx->stream);
  int64_t nfwd = 0;
  const uint32_t* skeys = nullptr;
  const uint2* sents = nullptr;
  const bool prepared = b->prepared;
  const bool fused = prepared && b->split;  // the view holds the multi runs only (fm_batch_prepare)
  FM_REQUIRE(!(fused && emit), "a batch prepared for the fused step cannot feed fm_repl_grad");
  FM_REQUIRE(ctx->epoch < (1 << 29), "epoch count beyond the multi tags' range (2^29 steps)");
  if (prepared) {
    // sorted ahead of time by fm_batch_prepare on the side stream
    skeys = b->skeys.as<uint32_t>();
    sents = b->sents.as<uint2>();
  } else {
    // fork: the sort only reads the batch, so it runs on the side stream beside the forward
    FM_HIP_CHECK(hipEventRecord(ctx->ev_fork, ctx->stream));
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    hipEvent_t es = ctx->prof_begin(ctx->side);
    radix_sort_pairs64(ctx->work.sort, b->dev.col.as<uint32_t>(), b->dev.ent.as<uint2>(), N, bits_for(ctx->rows - 1),
                       ctx->side, &skeys, &sents);
    ctx->prof_end("sort", es, ctx->side);
    FM_HIP_CHECK(hipEventRecord(ctx->ev_join, ctx->side));
  }
  hipEvent_t e0 = nullptr;
  FwdOut fx{};
  if (fused) {
    // the batch's sorted view (fm_batch_prepare, a step ahead on the side stream) split here, on the
    // main stream: its runs of two or more entries into the multi view, each multi run's row tagged
    // with this step's epoch by the count pass as it finds the run (the split on the side stream with a
    // separate tag pass at the step measured 0.968-0.971 against 0.924-0.931 ms per c3 step, three
    // alternating reps, profiles/r04_i)
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->stream, b->ready, 0));
    e0 = ctx->prof_begin(ctx->stream);
    launch_split(b->fkeys.as<uint32_t>(), b->fents.as<uint2>(), N, ctx->split_work, b->skeys.as<uint32_t>(),
                 b->sents.as<uint2>(), b->split_n.as<int64_t>(), ctx->stream, T, p.epoch);
    ctx->prof_end("split", e0, ctx->stream);
    fx.fused = true;
  }
  e0 = ctx->prof_begin(ctx->stream);
  launch_forward(T, b->dev, ctx->work, p, ctx->stream, &nfwd, nullptr, fused ? &fx : nullptr);
  ctx->prof_end("forward", e0, ctx->stream);
  // (the prepared batch's wait moved before the forward, where its sort has long finished, measured
  // 0.170-0.173 against 0.167-0.168 ms at c2 and 0.191-0.192 against 0.187-0.190 at c5, three
  // alternating reps, profiles/r05_h/ab: not taken)
  if (!fused) FM_HIP_CHECK(hipStreamWaitEvent(ctx->stream, prepared ? b->ready : ctx->ev_join, 0));
  e0 = ctx->prof_begin(ctx->stream);
  double* stats = ctx->loss_hist.as<double>() + 3 * (int64_t)ctx->epoch;
  launch_segment_update(T, b->dev, ctx->work, p, skeys, sents, nfwd, stats, ctx->stream, emit,
                        fused ? b->split_n.as<int64_t>() : nullptr);
  // the shared sort workspace is read by the main stream only when the batch was sorted inline
  // (not prepared): only then must the next fm_batch_prepare's sort wait for this update
  if (!prepared) FM_HIP_CHECK(hipEventRecord(ctx->ev_upd_done, ctx->stream));
  // the last read of the batch (its next fm_batch_prepare or fm_batch_from_rows refill waits for it)
  if (b->last_use) FM_HIP_CHECK(hipEventRecord(b->last_use, ctx->stream));
  b->prepared = false;
  ctx->prof_end("update", e0, ctx->stream);
  if (emit) return FM_OK;
  ctx->epoch += 1;
  ctx->cum_host.push_back(p.cum_next);
  if (out) {
    ctx->pinned.ensure(64);
    FM_HIP_CHECK(hipMemcpyAsync(ctx->pinned.p, stats, sizeof(double) * 3, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const double* h = reinterpret_cast<const double*>(ctx->pinned.p);
    out->loss_sum = h[0];
    out->n_loss_rows = (int64_t)h[1];
    out->n_unique = (int64_t)h[2];
    out->n_rows = B;
  }
  return FM_OK;
}

}  // namespace

extern "C" {

const char* fm_last_error(void) { return g_last_error.c_str(); }

int fm_create(const fm_config* cfg, fm_ctx** out) {
  return guarded_free([&]() -> int {
    FM_REQUIRE(cfg && out, "null argument");
    if (cfg->parallel != FM_PARALLEL_NONE) return group_create(cfg, out);  // several ranks (fm_group.hip)
    FM_REQUIRE(cfg->num_features >= 1 && cfg->num_features <= (int64_t(1) << 31), "num_features must be in [1, 2^31]");
    FM_REQUIRE(cfg->k >= 1 && cfg->k <= 256, "dimFactorization must be in [1, 256]");
    FM_REQUIRE(cfg->shard_count >= 1 && cfg->shard_index >= 0 && cfg->shard_index < cfg->shard_count,
               "bad shard_index / shard_count");
    FM_REQUIRE(cfg->init_sd >= 0.0, "init_sd must be >= 0");
    FM_REQUIRE(cfg->fuse_single == FM_FUSE_DEFAULT || cfg->fuse_single == FM_FUSE_ON || cfg->fuse_single == FM_FUSE_OFF,
               "fuse_single must be FM_FUSE_DEFAULT, FM_FUSE_ON or FM_FUSE_OFF");
    int ndev = 0;
    FM_HIP_CHECK(hipGetDeviceCount(&ndev));
    FM_REQUIRE(cfg->device >= 0 && cfg->device < ndev, "device ordinal out of range");
    FM_HIP_CHECK(hipSetDevice(cfg->device));
    std::unique_ptr<fm_ctx> c(new fm_ctx());
    c->cfg = *cfg;
    c->kp = (cfg->k + 3) / 4 * 4;
    c->rows = (cfg->num_features - cfg->shard_index + cfg->shard_count - 1) / cfg->shard_count;
    // (the step's stream at high priority and the side stream at the lowest measured slower: c3
    // 0.984-0.996 against 0.946-0.951 ms)
    FM_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
    FM_HIP_CHECK(hipStreamCreateWithFlags(&c->side_own, hipStreamNonBlocking));
    c->side = c->side_own;
    FM_HIP_CHECK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventCreateWithFlags(&c->ev_upd_done, hipEventDisableTiming));
    FM_HIP_CHECK(hipEventRecord(c->ev_upd_done, c->stream));
    c->stride = record_stride(c->kp);
    c->rec.ensure(sizeof(float) * (size_t)std::max<int64_t>(c->rows, 1) * c->stride);
    c->ensure_hist(4096);
    launch_table_reset(c->view(), c->stream);
    FM_HIP_CHECK(hipStreamSynchronize(c->stream));
    *out = c.release();
    return FM_OK;
  });
}

void fm_destroy(fm_ctx* ctx) {
  if (!ctx) return;
  try {
    delete ctx;
  } catch (...) {
  }
}

int fm_set_stream(fm_ctx* ctx, void* s) {
  if (ctx && ctx->group) {  // a multi-GPU context: only with one local rank, whose streams these become
    if (ctx->cfg.n_gpus != 1) {
      set_error("fm_set_stream on a context with several local ranks");
      return FM_ERR_ARG;
    }
    return fm_set_stream(group_member0(ctx), s);
  }
  return guarded(ctx, [&]() -> int {
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (ctx->own_stream && ctx->stream) FM_HIP_CHECK(hipStreamDestroy(ctx->stream));
    // NULL selects the device's default (null) stream, which is what torch's default stream is
    ctx->stream = reinterpret_cast<hipStream_t>(s);
    ctx->own_stream = false;
    return FM_OK;
  });
}

int fm_set_side_stream(fm_ctx* ctx, void* s) {
  if (ctx && ctx->group) {  // a multi-GPU context: only with one local rank, whose streams these become
    if (ctx->cfg.n_gpus != 1) {
      set_error("fm_set_side_stream on a context with several local ranks");
      return FM_ERR_ARG;
    }
    return fm_set_side_stream(group_member0(ctx), s);
  }
  return guarded(ctx, [&]() -> int {
    FM_HIP_CHECK(hipStreamSynchronize(ctx->side));
    ctx->side = s ? reinterpret_cast<hipStream_t>(s) : ctx->side_own;
    return FM_OK;
  });
}

int fm_sync(fm_ctx* ctx) {
  return guarded(ctx, [&]() -> int {
    if (ctx->group) return group_sync(ctx);
    // every stream the context enqueues on: the step's, the side stream's preparations and the copy
    // stream's fm_batch_from_rows gathers (after this the caller may free a dataset it gathered from)
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->side));
    if (ctx->copy_stream) FM_HIP_CHECK(hipStreamSynchronize(ctx->copy_stream));
    return FM_OK;
  });
}

int fm_reserve(fm_ctx* ctx, int64_t max_rows, int64_t max_nnz) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(max_rows >= 0 && max_nnz >= 0, "negative reserve");
    if (ctx->group) return group_reserve(ctx, max_rows, max_nnz);
    reserve_work(ctx, max_rows, max_nnz);
    return FM_OK;
  });
}

int fm_load_tables(fm_ctx* ctx, const int32_t* ids, int64_t n, const double* w, const double* V) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0, "negative n");
    if (n == 0) return FM_OK;
    if (ctx->group) return group_load_tables(ctx, ids, n, w, V);
    FM_REQUIRE(ids && w && V, "null argument");
    for (int64_t i = 0; i < n; ++i)
      FM_REQUIRE(ids[i] >= 0 && ids[i] < ctx->cfg.num_features, "id out of [0, num_features)");
    DevBuf di, dw, dv;
    di.ensure(sizeof(int32_t) * n);
    dw.ensure(sizeof(double) * n);
    dv.ensure(sizeof(double) * n * ctx->cfg.k);
    FM_HIP_CHECK(hipMemcpy(di.p, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice));
    FM_HIP_CHECK(hipMemcpy(dw.p, w, sizeof(double) * n, hipMemcpyHostToDevice));
    FM_HIP_CHECK(hipMemcpy(dv.p, V, sizeof(double) * n * ctx->cfg.k, hipMemcpyHostToDevice));
    launch_load_rows(ctx->view(), di.as<int32_t>(), n, dw.as<double>(), dv.as<double>(), ctx->epoch,
                     ctx->cum_host.back(), ctx->stream);
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    di.release();
    dw.release();
    dv.release();
    return FM_OK;
  });
}

int fm_init_random(fm_ctx* ctx, const int32_t* ids, int64_t n) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0, "negative n");
    if (n == 0) return FM_OK;
    FM_REQUIRE(ids, "null ids");
    if (ctx->group) return group_init_random(ctx, ids, n, 0, 0);
    for (int64_t i = 0; i < n; ++i)
      FM_REQUIRE(ids[i] >= 0 && ids[i] < ctx->cfg.num_features, "id out of [0, num_features)");
    DevBuf di;
    di.ensure(sizeof(int32_t) * n);
    FM_HIP_CHECK(hipMemcpy(di.p, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice));
    launch_init_random(ctx->view(), di.as<int32_t>(), n, 0, ctx->cfg.seed, ctx->cfg.init_sd, ctx->epoch,
                       ctx->cum_host.back(), ctx->stream);
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    di.release();
    return FM_OK;
  });
}

int fm_init_random_range(fm_ctx* ctx, int64_t b, int64_t e) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b >= 0 && e >= b && e <= ctx->cfg.num_features, "bad id range");
    if (ctx->group) return group_init_random(ctx, nullptr, 0, b, e);
    launch_init_random(ctx->view(), nullptr, e - b, b, ctx->cfg.seed, ctx->cfg.init_sd, ctx->epoch,
                       ctx->cum_host.back(), ctx->stream);
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return FM_OK;
  });
}

int64_t fm_num_present(fm_ctx* ctx) {
  int64_t n = -1;
  int rc = guarded(ctx, [&]() -> int {
    if (ctx->group) {
      n = group_num_present(ctx);
      return FM_OK;
    }
    DevBuf d;
    d.ensure(sizeof(int64_t));
    launch_count_present(ctx->view(), d.as<int64_t>(), ctx->stream);
    FM_HIP_CHECK(hipMemcpyAsync(&n, d.p, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    d.release();
    return FM_OK;
  });
  return rc == FM_OK ? n : rc;
}

int64_t fm_epoch(fm_ctx* ctx) { return ctx ? ctx->epoch : -1; }

int fm_export_tables(fm_ctx* ctx, int32_t* ids, double* w, double* V, int64_t cap, int64_t* n) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n != nullptr && cap >= 0, "bad arguments");
    if (ctx->group) return group_export_tables(ctx, ids, w, V, cap, n);
    launch_flush(ctx->view(), ctx->epoch, ctx->cum_host.back(), ctx->stream);  // apply pending L1 to every row
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    const int k = ctx->cfg.k, kp = ctx->kp, S = ctx->stride;
    const int64_t chunk_rows = std::max<int64_t>(1, (int64_t(64) << 20) / (4 * S));
    std::vector<float> hv;
    int64_t cnt = 0, o = 0;
    const bool fill = cap > 0;
    for (int64_t r0 = 0; r0 < ctx->rows; r0 += chunk_rows) {
      const int64_t r1 = std::min(ctx->rows, r0 + chunk_rows);
      hv.resize((size_t)(r1 - r0) * S);
      FM_HIP_CHECK(hipMemcpy(hv.data(), ctx->rec.as<float>() + r0 * S, sizeof(float) * (r1 - r0) * S,
                             hipMemcpyDeviceToHost));
      for (int64_t i = r0; i < r1; ++i) {
        const float* row = hv.data() + (size_t)(i - r0) * S;
        RowHdr hd;
        std::memcpy(&hd, row + kp, sizeof(RowHdr));
        if (hd.t < 0) continue;
        ++cnt;
        if (!fill) continue;
        FM_REQUIRE(o < cap && ids && w && V, "export buffers too small or null");
        ids[o] = (int32_t)(i * ctx->cfg.shard_count + ctx->cfg.shard_index);
        w[o] = hd.w;
        for (int f = 0; f < k; ++f) V[o * k + f] = row[f];
        ++o;
      }
    }
    *n = cnt;
    return FM_OK;
  });
}

int fm_export_rows(fm_ctx* ctx, const int32_t* ids, int64_t n, double* w, double* V, int8_t* present) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0, "negative n");
    if (n == 0) return FM_OK;
    FM_REQUIRE(ids && w && V && present, "null argument");
    if (ctx->group) return group_export_rows(ctx, ids, n, w, V, present);
    const int R = ctx->cfg.shard_count;
    for (int64_t i = 0; i < n; ++i) {
      FM_REQUIRE(ids[i] >= 0 && ids[i] < ctx->cfg.num_features, "id out of [0, num_features)");
      FM_REQUIRE(ids[i] % R == ctx->cfg.shard_index, "id not owned by this shard");
    }
    const int k = ctx->cfg.k;
    DevBuf di, dw, dv, dp;
    di.ensure(sizeof(int32_t) * n);
    dw.ensure(sizeof(double) * n);
    dv.ensure(sizeof(double) * n * k);
    dp.ensure(sizeof(int8_t) * n);
    FM_HIP_CHECK(hipMemcpyAsync(di.p, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
    launch_gather_rows(ctx->view(), di.as<int32_t>(), n, ctx->cum_host.back(), dw.as<double>(), dv.as<double>(),
                       dp.as<int8_t>(), ctx->stream);
    FM_HIP_CHECK(hipMemcpyAsync(w, dw.p, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipMemcpyAsync(V, dv.p, sizeof(double) * n * k, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipMemcpyAsync(present, dp.p, sizeof(int8_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return FM_OK;
  });
}

int fm_batch_create(fm_ctx* ctx, const fm_csr* csr, fm_batch** out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(out != nullptr, "null out");
    if (ctx->group) return group_batch_create(ctx, csr, out);
    std::unique_ptr<fm_batch> b(new fm_batch());
    upload_batch(ctx, csr, b.get(), true);
    // kept for fm_batch_from_rows (a cached dataset's splits sized on the host)
    b->host_rp.assign(csr->row_ptr, csr->row_ptr + csr->n_rows + 1);
    *out = b.release();
    return FM_OK;
  });
}

void fm_batch_destroy(fm_batch* b) {
  if (!b) return;
  try {
    delete b;
  } catch (...) {
  }
}

int fm_batch_prepare(fm_ctx* ctx, fm_batch* b) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b != nullptr && b->owner == ctx, "batch belongs to another context");
    if (ctx->group) return group_batch_prepare(ctx, b);
    FM_REQUIRE(ctx->cfg.shard_count == 1, "fm_batch_prepare is for single-table contexts");
    FM_REQUIRE(b->split_rows.empty(), "a dataset made by fm_batch_create_splits is prepared through its split views");
    const int64_t N = b->dev.nnz;
    if (N == 0) return FM_OK;
    if (!b->ready) {
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->ready, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->last_use, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventRecord(b->last_use, ctx->stream));
    }
    b->skeys.ensure_slack(sizeof(uint32_t) * N);
    b->sents.ensure_slack(sizeof(uint2) * N);
    // the shared sort workspace and this batch's view may still be read by an enqueued step; a batch
    // refilled by fm_batch_from_rows is sorted once its gather is done
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->side, ctx->ev_upd_done, 0));
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->side, b->last_use, 0));
    wait_built(b, ctx->side);
    hipEvent_t es = ctx->prof_begin(ctx->side);
    const uint32_t* sk = nullptr;
    const uint2* sv = nullptr;
    b->split = fuse_on(ctx);
    const int kb = bits_for(ctx->rows - 1);
    const uint32_t* col = b->dev.col.as<uint32_t>();
    const uint2* ent = b->dev.ent.as<uint2>();
    if (b->split) {
      // the fused step's batch: the whole sorted view (fkeys / fents), which the step splits into the
      // multi view (skeys / sents, {their count, the number of singleton runs} in split_n)
      b->split_n.ensure(2 * sizeof(int64_t));
      b->fkeys.ensure_slack(sizeof(uint32_t) * N);
      b->fents.ensure_slack(sizeof(uint2) * N);
      radix_sort_pairs64(ctx->work.sort, col, ent, N, kb, ctx->side, &sk, &sv, b->fkeys.as<uint32_t>(),
                         b->fents.as<uint2>());
    } else {
      radix_sort_pairs64(ctx->work.sort, col, ent, N, kb, ctx->side, &sk, &sv, b->skeys.as<uint32_t>(),
                         b->sents.as<uint2>());
    }
    ctx->prof_end("sort", es, ctx->side);
    FM_HIP_CHECK(hipEventRecord(b->ready, ctx->side));
    b->prepared = true;
    return FM_OK;
  });
}

int fm_batch_from_rows(fm_ctx* ctx, const fm_batch* data, const int64_t* rows, int64_t n, fm_batch** out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(out != nullptr && data != nullptr, "null argument");
    FM_REQUIRE(data->owner == ctx, "data belongs to another context");
    FM_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "n out of range");
    FM_REQUIRE(n == 0 || rows != nullptr, "null rows");
    if (ctx->group) return group_batch_from_rows(ctx, data, rows, n, out);
    const int64_t Bd = data->dev.n_rows;
    FM_REQUIRE((int64_t)data->host_rp.size() == Bd + 1,
               "data must be a batch made by fm_batch_create");
    fm_batch* b = *out;
    std::unique_ptr<fm_batch> fresh;
    if (b == nullptr) {
      fresh.reset(new fm_batch());
      b = fresh.get();
      b->owner = ctx;
      b->device = ctx->cfg.device;
    } else {
      FM_REQUIRE(b->owner == ctx && b != data && !b->grp && b->split_rows.empty(),
                 "out must be a batch of this context other than data");
    }
    // a split view refilled as a selection: its borrowed pointers are dropped, its own buffers grown below
    b->detach_view();
    if (!b->ready) {
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->ready, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->last_use, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventRecord(b->last_use, ctx->stream));
    }
    if (!b->built) {
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->built, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->sel_copied, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventRecord(b->sel_copied, ctx->side));
    }
    // the staging {rows, row_ptr} of this batch's previous selection has been copied out
    FM_HIP_CHECK(hipEventSynchronize(b->sel_copied));
    const size_t img = sizeof(int64_t) * (2 * (size_t)n + 1);
    b->sel_pin.ensure_slack(img);
    int64_t* hrows = reinterpret_cast<int64_t*>(b->sel_pin.p);
    int64_t* rp = hrows + n;
    // the rows and their result row_ptr straight into the pinned staging, from the dataset's row_ptr
    // (validated on the way): random reads of the dataset's row_ptr, about 2 ms for 256K rows on one
    // thread -- longer than the GPU step -- so on the pool's threads, each chunk's running lengths,
    // then the chunks' offsets
    rp[0] = 0;
    const int64_t* hrp = data->host_rp.data();
    const int64_t T = chunk_count(n, 8192);
    std::vector<int64_t> tot(T + 1, 0);
    std::atomic<int> bad{0};
    parallel_chunks_t(n, T, [&](int64_t t, int64_t lo, int64_t hi) {
      int64_t acc = 0;
      for (int64_t i = lo; i < hi; ++i) {
        const int64_t r = rows[i];
        if (r < 0 || r >= Bd) {
          bad.store(1);
          return;
        }
        hrows[i] = r;
        acc += hrp[r + 1] - hrp[r];
        rp[i + 1] = acc;
      }
      tot[t + 1] = acc;
    });
    FM_REQUIRE(!bad.load(), "row index out of [0, rows of data)");
    for (int64_t t = 0; t < T; ++t) tot[t + 1] += tot[t];  // the chunks' offsets
    if (T > 1)
      parallel_chunks_t(n, T, [&](int64_t t, int64_t lo, int64_t hi) {
        const int64_t add = tot[t];
        if (add)
          for (int64_t i = lo; i < hi; ++i) rp[i + 1] += add;
      });
    const int64_t N = rp[n];
    FM_REQUIRE(N < (int64_t(1) << 31), "nnz must be < 2^31 per batch");
    // batch-only work on the copy stream, behind every queued step that reads this batch: the copy
    // of the next split overlaps the sort of the current one on the side stream (the sort waits
    // for `built`, fm_batch_prepare)
    if (!ctx->copy_stream) FM_HIP_CHECK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    hipStream_t gs = ctx->copy_stream;
    // the refill rewrites what queued work may still read: the last step of the batch (b->last_use,
    // recorded by the single-table step and by the sharded owner update on the main stream), the
    // sharded iteration's own last read (sh->last_use) and a preparation never stepped (its sort on the
    // side stream reads dev.col / dev.ent)
    FM_HIP_CHECK(hipStreamWaitEvent(gs, b->last_use, 0));
    if (b->sh && b->sh->last_use) FM_HIP_CHECK(hipStreamWaitEvent(gs, b->sh->last_use, 0));
    if (b->prepared && b->ready) FM_HIP_CHECK(hipStreamWaitEvent(gs, b->ready, 0));
    b->dev.n_rows = n;
    b->dev.nnz = N;
    b->max_id = data->max_id;
    b->dev.row_ptr.ensure_slack(sizeof(int64_t) * (n + 1));
    b->dev.col.ensure_slack(sizeof(uint32_t) * std::max<int64_t>(N, 4) + 16);
    b->dev.ent.ensure_slack(sizeof(uint32_t) * 2 * std::max<int64_t>(N, 4) + 16);
    b->dev.xs.ensure_slack(sizeof(float) * std::max<int64_t>(N, 4) + 16);
    b->dev.label.ensure_slack(sizeof(double) * std::max<int64_t>(n, 4) + 16);
    b->up.ensure_slack(img + 16);
    FM_HIP_CHECK(hipMemcpyAsync(b->up.p, b->sel_pin.p, img, hipMemcpyHostToDevice, gs));
    FM_HIP_CHECK(hipEventRecord(b->sel_copied, gs));
    if (n > 0) {
      const int64_t* up = b->up.as<int64_t>();
      launch_select_rows(data->dev, up, up + n, n, b->dev, gs);
    } else {
      FM_HIP_CHECK(hipMemcpyAsync(b->dev.row_ptr.p, b->up.as<int64_t>(), sizeof(int64_t), hipMemcpyDeviceToDevice, gs));
    }
    FM_HIP_CHECK(hipEventRecord(b->built, gs));
    b->prepared = false;  // a refilled batch is sorted again by its own fm_batch_prepare
    b->host_rp.clear();   // a selection is not itself a dataset (fm_batch_create's batches are)
    if (fresh) *out = fresh.release();
    return FM_OK;
  });
}

int fm_batch_create_splits(fm_ctx* ctx, const fm_csr* csr, int32_t n_splits, const int64_t* split_rows,
                           fm_batch** out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(out != nullptr && csr != nullptr, "null argument");
    FM_REQUIRE(n_splits >= 1 && split_rows != nullptr, "n_splits must be >= 1");
    FM_REQUIRE(split_rows[0] == 0 && split_rows[n_splits] == csr->n_rows, "split_rows must run from 0 to n_rows");
    for (int32_t i = 0; i < n_splits; ++i) FM_REQUIRE(split_rows[i] <= split_rows[i + 1], "split_rows must be non-decreasing");
    if (ctx->group) return group_batch_create_splits(ctx, csr, n_splits, split_rows, out);
    std::unique_ptr<fm_batch> b(new fm_batch());
    upload_batch(ctx, csr, b.get(), true);
    b->host_rp.assign(csr->row_ptr, csr->row_ptr + csr->n_rows + 1);
    b->split_rows.assign(split_rows, split_rows + n_splits + 1);
    DevBuf dsr;
    dsr.ensure(sizeof(int64_t) * (n_splits + 1));
    FM_HIP_CHECK(hipMemcpyAsync(dsr.p, split_rows, sizeof(int64_t) * (n_splits + 1), hipMemcpyHostToDevice, ctx->stream));
    b->split_rp.ensure(sizeof(int64_t) * (csr->n_rows + n_splits));
    launch_split_rebase(b->dev, dsr.as<int64_t>(), n_splits, b->split_rp.as<int64_t>(), ctx->stream);
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    dsr.release();
    *out = b.release();
    return FM_OK;
  });
}

int fm_batch_split_view(fm_ctx* ctx, const fm_batch* data, int32_t split, fm_batch** out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(out != nullptr && data != nullptr, "null argument");
    FM_REQUIRE(data->owner == ctx, "data belongs to another context");
    if (ctx->group) return group_batch_split_view(ctx, data, split, out);
    const int64_t ns = (int64_t)data->split_rows.size() - 1;
    FM_REQUIRE(ns >= 1, "data must be a dataset made by fm_batch_create_splits");
    FM_REQUIRE(split >= 0 && split < ns, "split index out of range");
    fm_batch* b = *out;
    std::unique_ptr<fm_batch> fresh;
    if (b == nullptr) {
      fresh.reset(new fm_batch());
      b = fresh.get();
      b->owner = ctx;
      b->device = ctx->cfg.device;
    } else {
      FM_REQUIRE(b->owner == ctx && b != data && !b->grp && b->split_rows.empty(),
                 "out must be a batch of this context other than data");
    }
    if (!b->view_of) {
      // an owning batch becomes a view: its own buffers are freed once no queued work reads them
      for (hipEvent_t e : {b->last_use, b->ready, b->built, b->sel_copied})
        if (e) FM_HIP_CHECK(hipEventSynchronize(e));
      for (DevBuf* d : {&b->dev.row_ptr, &b->dev.col, &b->dev.ent, &b->dev.xs, &b->dev.label, &b->up}) d->release();
    }
    if (!b->ready) {
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->ready, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventCreateWithFlags(&b->last_use, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventRecord(b->last_use, ctx->stream));
    }
    // the split's rows, entries and labels in place: pointers into data (no copy, no gather); the
    // step's reads of a view are ordered like any batch's (data was complete when it was created)
    const int64_t r0 = data->split_rows[split], r1 = data->split_rows[split + 1];
    const int64_t e0 = data->host_rp[r0], e1 = data->host_rp[r1];
    b->view_of = data;
    b->dev.n_rows = r1 - r0;
    b->dev.nnz = e1 - e0;
    b->dev.row_ptr.p = data->split_rp.as<int64_t>() + r0 + split;
    b->dev.row_ptr.bytes = sizeof(int64_t) * (r1 - r0 + 1);
    b->dev.col.p = data->dev.col.as<uint32_t>() + e0;
    b->dev.col.bytes = sizeof(uint32_t) * (e1 - e0);
    b->dev.ent.p = data->dev.ent.as<uint2>() + e0;
    b->dev.ent.bytes = sizeof(uint2) * (e1 - e0);
    b->dev.xs.p = data->dev.xs.as<float>() + e0;
    b->dev.xs.bytes = sizeof(float) * (e1 - e0);
    b->dev.label.p = data->dev.label.as<double>() + r0;
    b->dev.label.bytes = sizeof(double) * (r1 - r0);
    b->max_id = data->max_id;
    b->prepared = false;
    b->host_rp.clear();
    if (fresh) *out = fresh.release();
    return FM_OK;
  });
}

int32_t fm_fuse_active(fm_ctx* ctx) {
  if (!ctx) return -1;
  // a multi-GPU context never fuses: replicas feed fm_repl_grad the whole sorted view, and a sharded
  // owner's fused step measured slower than the unfused one at R = 8 and at world 1
  if (ctx->group) return 0;
  return fuse_on(ctx) ? 1 : 0;
}

int64_t fm_batch_rows(const fm_batch* b) { return b ? b->dev.n_rows : -1; }
int64_t fm_batch_nnz(const fm_batch* b) { return b ? b->dev.nnz : -1; }

int fm_step_batch(fm_ctx* ctx, fm_batch* batch, int32_t t, double step_size, double reg_param,
                  fm_step_out* out) {
  return guarded(ctx, [&]() -> int {
    if (ctx->group) return group_step_batch(ctx, batch, t, step_size, reg_param, out);
    return step_impl(ctx, batch, t, step_size, reg_param, out);
  });
}

int fm_step(fm_ctx* ctx, const fm_csr* csr, int32_t t, double step_size, double reg_param, fm_step_out* out) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(csr != nullptr, "null batch");
    if (csr->n_rows == 0) {
      if (out) {
        out->loss_sum = 0.0;
        out->n_rows = 0;
        out->n_loss_rows = 0;
        out->n_unique = 0;
      }
      if (!ctx->group) return FM_NOTHING_TO_DO;  // a group's other processes may hold rows: they agree below
    }
    if (ctx->group) return group_step(ctx, csr, t, step_size, reg_param, out);
    // two upload slots used in turn: while the device runs step i from one slot, the host explodes
    // batch i + 1 into the other slot's pinned staging and its copies queue on the copy stream
    HostSlot& h = ctx->hslot[ctx->hnext];
    ctx->hnext ^= 1;
    if (!h.batch) {
      h.batch.reset(new fm_batch());
      FM_HIP_CHECK(hipEventCreateWithFlags(&h.copied, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventCreateWithFlags(&h.consumed, hipEventDisableTiming));
      FM_HIP_CHECK(hipEventRecord(h.copied, ctx->stream));
      FM_HIP_CHECK(hipEventRecord(h.consumed, ctx->stream));
    }
    if (!ctx->copy_stream) FM_HIP_CHECK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    FM_HIP_CHECK(hipEventSynchronize(h.copied));  // the slot's staging has been copied out
    const Staged g = stage_csr(ctx, csr, true, h.pin);
    if (!batch_fits(h.batch.get(), g)) FM_HIP_CHECK(hipEventSynchronize(h.consumed));  // before reallocating
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->copy_stream, h.consumed, 0));  // the slot's last step read it
    copy_staged(ctx, g, h.pin, h.batch.get(), ctx->copy_stream);
    FM_HIP_CHECK(hipEventRecord(h.copied, ctx->copy_stream));
    FM_HIP_CHECK(hipStreamWaitEvent(ctx->stream, h.copied, 0));
    const int rc = step_impl(ctx, h.batch.get(), t, step_size, reg_param, out);  // out == NULL: no host sync
    FM_HIP_CHECK(hipEventRecord(h.consumed, ctx->stream));
    return rc;
  });
}

int fm_loss_history(fm_ctx* ctx, double* loss, int64_t cap, int64_t* n) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n != nullptr, "null n");
    if (ctx->group) return group_loss_history(ctx, loss, cap, n);
    *n = ctx->epoch;
    if (cap == 0 || ctx->epoch == 0) return FM_OK;
    FM_REQUIRE(loss != nullptr, "null loss buffer");
    const int64_t m = std::min<int64_t>(cap, ctx->epoch);
    std::vector<double> h(3 * m);
    FM_HIP_CHECK(hipMemcpyAsync(h.data(), ctx->loss_hist.p, sizeof(double) * 3 * m, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (int64_t i = 0; i < m; ++i) loss[i] = h[3 * i];
    return FM_OK;
  });
}

int fm_predict(fm_ctx* ctx, const fm_csr* csr, double lo, double hi, double* pred) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(csr != nullptr && (csr->n_rows == 0 || pred), "null argument");
    if (ctx->group) return group_predict(ctx, csr, lo, hi, pred);
    if (csr->n_rows == 0) return FM_OK;
    fm_batch* b = host_batch(ctx);
    upload_batch(ctx, csr, b, false);
    DevBuf dp;
    dp.ensure(sizeof(double) * csr->n_rows);
    launch_predict(ctx->view(), b->dev, ctx->cum_host.back(), ctx->cfg.w0, lo, hi, dp.as<double>(), ctx->stream);
    FM_HIP_CHECK(hipMemcpyAsync(pred, dp.p, sizeof(double) * csr->n_rows, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    dp.release();
    return FM_OK;
  });
}

int fm_predict_batch(fm_ctx* ctx, fm_batch* b, double lo, double hi, double* pred) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b != nullptr && b->owner == ctx, "batch belongs to another context");
    if (ctx->group) return group_predict_batch(ctx, b, lo, hi, pred);
    const int64_t B = b->dev.n_rows;
    FM_REQUIRE(B == 0 || pred, "null argument");
    if (B == 0) return FM_OK;
    DevBuf dp;
    dp.ensure(sizeof(double) * B);
    wait_built(b, ctx->stream);
    hipEvent_t e0 = ctx->prof_begin(ctx->stream);
    launch_predict(ctx->view(), b->dev, ctx->cum_host.back(), ctx->cfg.w0, lo, hi, dp.as<double>(), ctx->stream);
    ctx->prof_end("predict", e0, ctx->stream);
    FM_HIP_CHECK(hipMemcpyAsync(pred, dp.p, sizeof(double) * B, hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    dp.release();
    return FM_OK;
  });
}

int fm_init_from_batch(fm_ctx* ctx, fm_batch* b, int64_t* n_present) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(b != nullptr && b->owner == ctx, "batch belongs to another context");
    if (ctx->group) return group_init_from_batch(ctx, b, n_present);
    wait_built(b, ctx->stream);
    launch_init_entries(ctx->view(), b->dev.col.as<uint32_t>(), b->dev.nnz, ctx->cfg.seed, ctx->cfg.init_sd, ctx->epoch,
                        ctx->cum_host.back(), ctx->stream);
    if (n_present) {
      DevBuf d;
      d.ensure(sizeof(int64_t));
      launch_count_present(ctx->view(), d.as<int64_t>(), ctx->stream);
      FM_HIP_CHECK(hipMemcpyAsync(n_present, d.p, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
      FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
      d.release();
    } else {
      FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    }
    return FM_OK;
  });
}

static int loss_grad_impl(fm_ctx* ctx, const fm_csr* csr, double fill_sd, uint64_t seed, double* pred, double* loss,
                          double* dw, double* dv) {
  if (ctx && ctx->group) {
    // a replicated group's replicas are identical: member 0 answers, with the group locked so that
    // no group step is caught between a member's fm_repl_grad and fm_repl_apply
    return guarded(ctx, [&]() -> int {
      FM_REQUIRE(ctx->cfg.parallel == FM_PARALLEL_REPLICATED,
                 "fm_loss_grad needs the whole table (a replicated or single-table context)");
      return loss_grad_impl(group_member0(ctx), csr, fill_sd, seed, pred, loss, dw, dv);
    });
  }
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(ctx->cfg.shard_count == 1, "fm_loss_grad needs the whole table (shard_count == 1)");
    FM_REQUIRE(csr != nullptr, "null argument");
    if (csr->n_rows == 0 || csr->nnz == 0) return FM_OK;
    fm_batch* b = host_batch(ctx);
    // the fill covers ids the table cannot hold too (ids >= num_features, the left outer join)
    upload_batch(ctx, csr, b, fill_sd <= 0.0);
    const int64_t N = csr->nnz;
    const int k = ctx->cfg.k;
    DevBuf dpred, dloss, ddw, ddv, dabs;
    dpred.ensure(sizeof(double) * N);
    dloss.ensure(sizeof(double) * N);
    ddw.ensure(sizeof(double) * N);
    ddv.ensure(sizeof(double) * N * k);
    dabs.ensure(sizeof(int32_t));
    FM_HIP_CHECK(hipMemsetAsync(dabs.p, 0, sizeof(int32_t), ctx->stream));
    launch_loss_grad(ctx->view(), b->dev, ctx->cum_host.back(), ctx->cfg.w0, dpred.as<double>(), dloss.as<double>(),
                     ddw.as<double>(), ddv.as<double>(), dabs.as<int32_t>(), ctx->stream, fill_sd, seed);
    int32_t absent = 0;
    FM_HIP_CHECK(hipMemcpyAsync(&absent, dabs.p, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    FM_REQUIRE(fill_sd > 0.0 || absent == 0, "batch references feature ids absent from the model");
    if (pred) FM_HIP_CHECK(hipMemcpy(pred, dpred.p, sizeof(double) * N, hipMemcpyDeviceToHost));
    if (loss) FM_HIP_CHECK(hipMemcpy(loss, dloss.p, sizeof(double) * N, hipMemcpyDeviceToHost));
    if (dw) FM_HIP_CHECK(hipMemcpy(dw, ddw.p, sizeof(double) * N, hipMemcpyDeviceToHost));
    if (dv) FM_HIP_CHECK(hipMemcpy(dv, ddv.p, sizeof(double) * N * k, hipMemcpyDeviceToHost));
    return FM_OK;
  });
}

int fm_loss_grad(fm_ctx* ctx, const fm_csr* csr, double* pred, double* loss, double* dw, double* dv) {
  return loss_grad_impl(ctx, csr, 0.0, 0, pred, loss, dw, dv);
}

int fm_calc_loss_grad(fm_ctx* ctx, const fm_csr* csr, double initial_sd, uint64_t seed, double* pred, double* loss,
                      double* dw, double* dv) {
  if (!(initial_sd > 0.0) || !std::isfinite(initial_sd)) {
    set_error("requirement failed: initSd (initial Standard Deviation) must be > 0.0");
    return FM_ERR_ARG;
  }
  return loss_grad_impl(ctx, csr, initial_sd, seed, pred, loss, dw, dv);
}

int fm_vector_sum_by_key(fm_ctx* ctx, const int32_t* keys, int64_t n, const double* vecs, int32_t k,
                         int32_t* out_keys, double* out_sums, int64_t* n_out) {
  if (ctx && ctx->group)  // on member 0's device, with the group locked
    return guarded(ctx, [&]() -> int {
      return fm_vector_sum_by_key(group_member0(ctx), keys, n, vecs, k, out_keys, out_sums, n_out);
    });
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n >= 0 && k >= 1 && n_out, "bad arguments");
    *n_out = 0;
    if (n == 0) return FM_OK;
    FM_REQUIRE(keys && vecs && out_keys && out_sums, "null argument");
    int64_t mx = 0;
    for (int64_t i = 0; i < n; ++i) {
      FM_REQUIRE(keys[i] >= 0, "negative key");
      mx = std::max<int64_t>(mx, keys[i]);
    }
    DevBuf dk, dvec, dok, dos, drun, dn;
    SortWork sw;
    dk.ensure(sizeof(uint32_t) * n);
    dvec.ensure(sizeof(double) * n * k);
    dok.ensure(sizeof(int32_t) * n);
    dos.ensure(sizeof(double) * n * k);
    drun.ensure(sizeof(uint32_t) * n);
    dn.ensure(sizeof(int64_t));
    FM_HIP_CHECK(hipMemcpy(dk.p, keys, sizeof(int32_t) * n, hipMemcpyHostToDevice));
    FM_HIP_CHECK(hipMemcpy(dvec.p, vecs, sizeof(double) * n * k, hipMemcpyHostToDevice));
    const uint32_t *sk = nullptr, *sv = nullptr;
    radix_sort_pairs(sw, dk.as<uint32_t>(), nullptr, n, bits_for(mx), ctx->stream, &sk, &sv);
    launch_segment_sum(sk, sv, n, dvec.as<double>(), k, drun.as<uint32_t>(), dok.as<int32_t>(), dos.as<double>(),
                       dn.as<int64_t>(), ctx->stream);
    int64_t nu = 0;
    FM_HIP_CHECK(hipMemcpyAsync(&nu, dn.p, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    FM_HIP_CHECK(hipMemcpy(out_keys, dok.p, sizeof(int32_t) * nu, hipMemcpyDeviceToHost));
    FM_HIP_CHECK(hipMemcpy(out_sums, dos.p, sizeof(double) * nu * k, hipMemcpyDeviceToHost));
    *n_out = nu;
    DevBuf* bufs[] = {&dk, &dvec, &dok, &dos, &drun, &dn, &sw.keys_a, &sw.keys_b, &sw.vals_a, &sw.vals_b,
                      &sw.counts, &sw.digit_tot};
    for (auto* bb : bufs) bb->release();
    return FM_OK;
  });
}

int fm_profile_enable(fm_ctx* ctx, int32_t on) {
  return guarded(ctx, [&]() -> int {
    if (ctx->group) return group_profile(ctx, 0, on, nullptr, 0, nullptr, nullptr, 0, nullptr);
    ctx->prof = on != 0;
    return FM_OK;
  });
}

int fm_profile_reset(fm_ctx* ctx) {
  return guarded(ctx, [&]() -> int {
    if (ctx->group) return group_profile(ctx, 1, 0, nullptr, 0, nullptr, nullptr, 0, nullptr);
    ctx->resolve_profile();
    ctx->prof_acc.clear();
    ctx->prof_order.clear();
    return FM_OK;
  });
}

int fm_profile_read(fm_ctx* ctx, char* names, int64_t names_cap, double* total_ms, int64_t* launches, int64_t cap,
                    int64_t* n) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(n != nullptr, "null n");
    if (ctx->group) return group_profile(ctx, 2, 0, names, names_cap, total_ms, launches, cap, n);
    ctx->resolve_profile();
    *n = (int64_t)ctx->prof_order.size();
    std::string joined;
    int64_t i = 0;
    for (const auto& nm : ctx->prof_order) {
      if (i < cap) {
        if (total_ms) total_ms[i] = ctx->prof_acc[nm].ms;
        if (launches) launches[i] = ctx->prof_acc[nm].n;
      }
      if (!joined.empty()) joined += "\n";
      joined += nm;
      ++i;
    }
    if (names && names_cap > 0) {
      const size_t m = std::min<size_t>((size_t)names_cap - 1, joined.size());
      std::memcpy(names, joined.data(), m);
      names[m] = '\0';
    }
    return FM_OK;
  });
}

int fm_repl_grad(fm_ctx* ctx, fm_batch* batch, void* grad) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(!ctx->group, "a multi-GPU context runs its replicated step itself (fm_step / fm_step_batch)");
    FM_REQUIRE(grad != nullptr, "null gradient buffer");
    FM_REQUIRE(!ctx->repl_pending, "fm_repl_apply must follow fm_repl_grad");
    ctx->ensure_hist(ctx->epoch + 1);
    double* stats = ctx->loss_hist.as<double>() + 3 * (int64_t)ctx->epoch;
    FM_HIP_CHECK(hipMemsetAsync(stats, 0, sizeof(double) * 3, ctx->stream));
    const int rc = step_impl(ctx, batch, 1, 0.0, 0.0, nullptr, reinterpret_cast<float*>(grad));
    ctx->repl_pending = true;
    return rc;
  });
}

int fm_repl_apply(fm_ctx* ctx, const void* grad, int32_t t, double step_size, double reg_param,
                  int64_t global_rows) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(!ctx->group, "a multi-GPU context runs its replicated step itself (fm_step / fm_step_batch)");
    FM_REQUIRE(ctx->repl_pending, "fm_repl_grad must run first");
    FM_REQUIRE(global_rows >= 0, "negative global_rows");
    ctx->repl_pending = false;
    if (global_rows == 0) return FM_NOTHING_TO_DO;  // SGD.scala:126-128 (every rank skips)
    FM_REQUIRE(grad != nullptr, "null gradient buffer");
    FM_REQUIRE(t >= 1, "iteration index t must be >= 1");
    FM_REQUIRE(std::isfinite(step_size) && std::isfinite(reg_param), "non-finite step size / regParam");
    StepParams p{};
    p.n_rows = global_rows;
    p.eta = step_size / std::sqrt((double)t);  // SGD.scala:121
    p.lam = p.eta * reg_param;                 // SGD.scala:122
    p.m = (double)global_rows;                 // global miniBatchSize
    p.scale_v = p.eta / (double)global_rows;
    p.epoch = ctx->epoch;
    p.cumE = ctx->cum_host.back();
    p.cum_next = p.cumE + p.lam;
    p.w0 = ctx->cfg.w0;
    ctx->ensure_hist(ctx->epoch + 1);
    ctx->repl_cnt.ensure(sizeof(uint32_t) * kReplApplyBlocks);
    hipEvent_t e0 = ctx->prof_begin(ctx->stream);
    double* stats = ctx->loss_hist.as<double>() + 3 * (int64_t)ctx->epoch;
    launch_repl_apply(ctx->view(), reinterpret_cast<const float*>(grad), p, ctx->repl_cnt.as<uint32_t>(), stats + 2,
                      ctx->stream);
    ctx->prof_end("apply", e0, ctx->stream);
    ctx->epoch += 1;
    ctx->cum_host.push_back(p.cum_next);
    return FM_OK;
  });
}

int fm_last_stats(fm_ctx* ctx, double* loss_sum, int64_t* n_loss_rows, int64_t* n_unique) {
  return guarded(ctx, [&]() -> int {
    FM_REQUIRE(loss_sum && n_loss_rows && n_unique, "null argument");
    if (ctx->group) return group_last_stats(ctx, loss_sum, n_loss_rows, n_unique);
    FM_REQUIRE(ctx->epoch >= 1, "no step executed");
    double h[3];
    FM_HIP_CHECK(hipMemcpyAsync(h, ctx->loss_hist.as<double>() + 3 * (int64_t)(ctx->epoch - 1), sizeof(h),
                                hipMemcpyDeviceToHost, ctx->stream));
    FM_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    *loss_sum = h[0];
    *n_loss_rows = (int64_t)h[1];
    *n_unique = (int64_t)h[2];
    return FM_OK;
  });
}

}  // extern "C"
