// The context and batch objects behind the opaque C handles (shared by fm_capi.hip and
// fm_shard.hip).  Not part of the C-ABI.
#pragma once

#include <map>
#include <memory>
#include <utility>

#include "fm_internal.h"

namespace fmhip {

// Pinned host staging for small device->host reads.
struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t n) {
    if (n <= bytes && p) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    FM_HIP_CHECK(hipHostMalloc(&p, n, hipHostMallocDefault));
    bytes = n;
  }
  void ensure_slack(size_t n) {
    if (n > bytes || !p) ensure(n + n / 8 + 4096);
  }
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
};

// One upload slot of fm_step's host-buffer path: pinned staging + device batch, with the events
// that say when the staging may be rewritten and when the batch may be refilled.
struct HostSlot {
  std::unique_ptr<fm_batch> batch;
  Pinned pin;
  hipEvent_t copied = nullptr;    // copy stream: the staging's copies are done
  hipEvent_t consumed = nullptr;  // main stream: the step that read the batch is done
};

struct ProfEntry {
  double ms = 0.0;
  int64_t n = 0;
};

// Per-batch state of the row-sharded step (fm_shard.hip).  Everything a sharded iteration
// derives from the batch alone (the owner routing, the received entries' pair table and their
// slot order) is produced ahead of the iteration on the side stream and kept here, so the next
// batch's preparation overlaps the current iteration.
struct ShardBatchState {
  // requester: fm_shard_route -> fm_shard_combine
  DevBuf pairidx;                  // [B][R] int32 pair index of (sample, owner), -1 if none
  std::vector<int64_t> pairs_out;  // pairs sent to each owner
  int64_t route_nnz = -1;
  DevBuf poff;                     // [R+1] int64 owner blocks of the partial / S rows
  int64_t loss_blocks = 0;
  hipEvent_t fwd_e0 = nullptr;  // owner_forward profile start (chunked passes)
  bool combined = false;
  // owner: fm_shard_owner_prepare -> fm_shard_owner_forward -> fm_shard_owner_update
  bool prepared = false;
  const uint32_t* recv_slot = nullptr;  // caller's buffers, valid until owner_forward completes
  const uint2* recv_ent = nullptr;
  int64_t n = 0, P = 0;
  Pinned pin_off;
  DevBuf src_off;            // [R+1] int64 source offsets of the received entries, then [R+1] pair offsets
  DevBuf pair_ptr;           // [P+1] int64 entry offsets of the pairs
  DevBuf skeys, sents;       // received entries sorted by slot: slots / {pair, x bits}
  hipEvent_t ready_fwd = nullptr;  // side stream: pair table done
  hipEvent_t ready_upd = nullptr;  // side stream: slot sort done
  hipEvent_t last_use = nullptr;   // main stream: the iteration's update has read everything
  void release(int device) {
    (void)hipSetDevice(device);
    for (hipEvent_t e : {ready_fwd, ready_upd, last_use})
      if (e) (void)hipEventSynchronize(e);
    for (hipEvent_t e : {ready_fwd, ready_upd, last_use})
      if (e) (void)hipEventDestroy(e);
    ready_fwd = ready_upd = last_use = nullptr;
    for (DevBuf* b : {&pairidx, &poff, &src_off, &pair_ptr, &skeys, &sents}) b->release();
  }
};

// Multi-GPU context state (fm_group.hip): the ranks one fm_ctx drives, and a group batch's
// per-rank parts.
struct Group;
struct GroupBatch;
struct GroupDeleter {
  void operator()(Group* g) const;
};
struct GroupBatchDeleter {
  void operator()(GroupBatch* g) const;
};

}  // namespace fmhip

using namespace fmhip;

struct fm_batch {
  fm_ctx* owner = nullptr;
  int device = 0;
  BatchDev dev;
  int64_t max_id = -1;
  DevBuf up;  // device image of the host staging (fm_capi.hip copy_staged)
  // feature-major view produced by fm_batch_prepare (consumed once by the next step): the whole
  // sorted view in skeys / sents, or -- split = true, the fused step -- the whole sorted view in
  // fkeys / fents, which the step splits into the runs of two or more entries (skeys / sents) with
  // split_n = {their count, the number of singleton runs} on the device (fm_kernels.hip)
  DevBuf skeys, sents;
  DevBuf fkeys, fents;
  DevBuf split_n;
  bool split = false;
  hipEvent_t ready = nullptr;     // recorded on the side stream after the prepared sort
  hipEvent_t last_use = nullptr;  // recorded on the main stream after a step read the batch
  bool prepared = false;
  // fm_batch_from_rows: the host copy of row_ptr that sizes a selection of this batch's rows without
  // a device read (kept by fm_batch_create and fm_batch_from_rows), the selection's pinned staging
  // {rows, row_ptr} and its events (copy stream: staging copied out; the batch's rows written --
  // every reader of dev on another stream waits for `built`)
  std::vector<int64_t> host_rp;
  Pinned sel_pin;
  hipEvent_t sel_copied = nullptr, built = nullptr;
  // fm_batch_create_splits: the dataset's split boundaries (row offsets [n_splits + 1]) and every
  // split's own row_ptr rebased to its first entry (split_rp, [rows + n_splits]: split s at
  // split_rows[s] + s); its entries' sample indices are relative to their split's first row, so the
  // dataset itself is never stepped -- its splits are, through views
  std::vector<int64_t> split_rows;
  DevBuf split_rp;
  // fm_batch_split_view: dev's buffers point into view_of's (borrowed: never grown, never freed here)
  const fm_batch* view_of = nullptr;
  // a view's borrowed pointers dropped (before the batch frees or grows its own)
  void detach_view() {
    if (!view_of) return;
    for (DevBuf* d : {&dev.row_ptr, &dev.col, &dev.ent, &dev.xs, &dev.label}) {
      d->p = nullptr;
      d->bytes = 0;
    }
    view_of = nullptr;
  }
  std::unique_ptr<ShardBatchState> sh;  // sharded contexts only
  std::unique_ptr<GroupBatch, GroupBatchDeleter> grp;  // a multi-GPU context's batch: its per-rank parts
  ~fm_batch() {
    grp.reset();
    (void)hipSetDevice(device);
    if (sh) sh->release(device);
    for (hipEvent_t e : {ready, last_use, sel_copied, built})
      if (e) (void)hipEventSynchronize(e);
    for (hipEvent_t e : {ready, last_use, sel_copied, built})
      if (e) (void)hipEventDestroy(e);
    detach_view();
    split_rp.release();
    skeys.release();
    sents.release();
    fkeys.release();
    fents.release();
    split_n.release();
    up.release();
    dev.row_ptr.release();
    dev.col.release();
    dev.ent.release();
    dev.xs.release();
    dev.label.release();
  }
};

struct fm_ctx {
  std::mutex mu;
  fm_config cfg{};
  std::unique_ptr<Group, GroupDeleter> group;  // non-null: this context drives several ranks (fm_group.hip)
  int32_t kp = 0;
  int64_t rows = 0;  // local rows
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipStream_t side = nullptr;  // the entry sort runs here, overlapped with the forward
  hipStream_t side_own = nullptr;  // the context's own side stream (fm_set_side_stream may replace side)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_upd_done = nullptr;  // last main-stream read of the shared sort workspace (an inline-sorted step)
  DevBuf rec;  // [rows * stride] float records (V row + header)
  int32_t stride = 0;
  std::vector<double> cum_host{0.0};  // cum[e] = sum of lambda over executed steps 1..e
  int32_t epoch = 0;
  DevBuf loss_hist;  // [hist_cap][3] double {loss, n_loss, n_unique}
  int64_t hist_cap = 0;
  StepWork work;
  Pinned pinned;
  Pinned up_pin;                         // host CSR upload staging (upload_batch)
  std::unique_ptr<fm_batch> host_batch;  // reused by fm_predict / fm_loss_grad
  HostSlot hslot[2];                     // fm_step's double-buffered uploads
  int hnext = 0;
  hipStream_t copy_stream = nullptr;     // their host -> device copies
  // profiling
  bool prof = false;
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> free_events;
  std::map<std::string, ProfEntry> prof_acc;
  std::vector<std::string> prof_order;
  // sharded step scratch (fm_shard.hip): used only on the side stream by fm_shard_route and
  // fm_shard_owner_prepare (the per-batch results live in fm_batch::sh)
  DevBuf sh_okey;      // [N] owner of each entry (partition sort keys)
  DevBuf sh_mask;      // [B] uint64 owners present in each sample
  DevBuf sh_tcnt;      // [R][tiles] pair counts -> exclusive offsets
  DevBuf sh_tot;       // [R] pairs per owner, then [R] entries per owner (uint64)
  DevBuf sh_pay;       // [N] uint2 route payload {pair index within the owner's block, x bits}
  DevBuf sh_skey;      // [N] owner-partitioned route keys
  DevBuf sh_ent2;      // [n] uint2 {pair, x bits}: the slot sort's payload
  SortWork side_sort;  // radix sort workspace of the side stream
  SortWork route_sort;  // the route's owner partition (fm_shard_route)
  // the split of an LSD-sorted view into its multi runs: only the single-table fused step runs it, at
  // the step (main stream, step_impl), so one stream uses the workspace
  SplitWork split_work;
  Pinned side_pinned;  // route counts (device -> host)
  // replicated step state (fm_repl_*)
  DevBuf repl_cnt;            // touched-row counts per apply block (uint32)
  bool repl_pending = false;  // fm_repl_grad ran, fm_repl_apply not yet

  TableView view() const {
    TableView T;
    T.rec = rec.as<float>();
    T.rows = rows;
    T.stride = stride;
    T.k = cfg.k;
    T.kp = kp;
    T.shard_count = cfg.shard_count;
    T.shard_index = cfg.shard_index;
    return T;
  }

  hipEvent_t get_event() {
    if (!free_events.empty()) {
      hipEvent_t e = free_events.back();
      free_events.pop_back();
      return e;
    }
    hipEvent_t e;
    FM_HIP_CHECK(hipEventCreate(&e));
    return e;
  }

  // RAII-free helpers: begin() records a start event, end() the stop event for `name`.
  hipEvent_t prof_begin(hipStream_t s) {
    if (!prof) return nullptr;
    hipEvent_t e = get_event();
    FM_HIP_CHECK(hipEventRecord(e, s));
    return e;
  }
  void prof_end(const char* name, hipEvent_t e0, hipStream_t s) {
    if (!prof || !e0) return;
    hipEvent_t e1 = get_event();
    FM_HIP_CHECK(hipEventRecord(e1, s));
    pending.push_back({name, {e0, e1}});
    if (pending.size() > 4096) resolve_profile();
  }
  // host time of a phase (the multi-GPU driver's enqueue, fm_group.hip), beside the device phases
  void prof_host(const char* name, double ms) {
    if (!prof) return;
    auto it = prof_acc.find(name);
    if (it == prof_acc.end()) {
      prof_order.push_back(name);
      it = prof_acc.emplace(name, ProfEntry{}).first;
    }
    it->second.ms += ms;
    it->second.n += 1;
  }
  void resolve_profile() {
    if (pending.empty()) return;
    FM_HIP_CHECK(hipStreamSynchronize(stream));
    FM_HIP_CHECK(hipStreamSynchronize(side));
    for (auto& pe : pending) {
      float ms = 0.f;
      FM_HIP_CHECK(hipEventElapsedTime(&ms, pe.second.first, pe.second.second));
      auto it = prof_acc.find(pe.first);
      if (it == prof_acc.end()) {
        prof_order.push_back(pe.first);
        it = prof_acc.emplace(pe.first, ProfEntry{}).first;
      }
      it->second.ms += ms;
      it->second.n += 1;
      free_events.push_back(pe.second.first);
      free_events.push_back(pe.second.second);
    }
    pending.clear();
  }

  void ensure_hist(int64_t need) {
    if (need <= hist_cap) return;
    int64_t c = std::max<int64_t>(4096, hist_cap);
    while (c < need) c *= 2;
    FM_HIP_CHECK(hipStreamSynchronize(stream));
    DevBuf nb;
    nb.ensure(sizeof(double) * 3 * c);
    FM_HIP_CHECK(hipMemset(nb.p, 0, sizeof(double) * 3 * c));
    if (hist_cap > 0)
      FM_HIP_CHECK(hipMemcpy(nb.p, loss_hist.p, sizeof(double) * 3 * hist_cap, hipMemcpyDeviceToDevice));
    loss_hist.release();
    loss_hist = nb;
    nb.p = nullptr;
    hist_cap = c;
  }

  ~fm_ctx() {
    group.reset();
    (void)hipSetDevice(cfg.device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    for (auto& h : hslot) {
      if (h.copied) (void)hipEventDestroy(h.copied);
      if (h.consumed) (void)hipEventDestroy(h.consumed);
    }
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    for (auto& pe : pending) {
      (void)hipEventDestroy(pe.second.first);
      (void)hipEventDestroy(pe.second.second);
    }
    for (auto e : free_events) (void)hipEventDestroy(e);
    if (side) (void)hipStreamSynchronize(side);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (ev_upd_done) (void)hipEventDestroy(ev_upd_done);
    if (side_own) (void)hipStreamSynchronize(side_own);
    if (side_own) (void)hipStreamDestroy(side_own);
    rec.release();
    loss_hist.release();
    DevBuf* bufs[] = {&work.S, &work.yl, &work.loss_part, &work.part, &work.ucnt,
                      &work.sort.keys_a, &work.sort.keys_b, &work.sort.vals_a, &work.sort.vals_b,
                      &work.sort.counts, &work.sort.digit_tot, &side_sort.keys_a, &side_sort.keys_b,
                      &side_sort.vals_a, &side_sort.vals_b, &side_sort.counts, &side_sort.digit_tot,
                      &route_sort.keys_a, &route_sort.keys_b, &route_sort.vals_a, &route_sort.vals_b,
                      &route_sort.counts, &route_sort.digit_tot,
                      &sh_okey, &sh_mask, &sh_tcnt, &sh_tot, &sh_pay, &sh_skey, &sh_ent2, &repl_cnt,
                      &split_work.cnt, &split_work.off};
    for (auto* b : bufs) b->release();
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }
};


namespace fmhip {
void report_stale(hipError_t e);  // fm_capi.hip

template <class F>
int guarded(fm_ctx* ctx, F&& f) {
  if (!ctx) {
    set_error("null fm_ctx");
    return FM_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  // the caller's current device is restored on the way out (torch and other contexts keep theirs)
  int prev_dev = -1;
  if (hipGetDevice(&prev_dev) != hipSuccess) prev_dev = -1;
  struct Restore {
    int d;
    ~Restore() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore{prev_dev};
  try {
    // a sticky error left by an earlier call whose status was ignored (a destructor's event waits)
    // belongs to no launch of this call: reported on stderr once per code, then cleared, so that the
    // launch checks below see their own launches only
    report_stale(hipGetLastError());
    FM_HIP_CHECK(hipSetDevice(ctx->cfg.device));
    return f();
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed");
    return FM_ERR_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return FM_ERR_HIP;
  } catch (...) {
    set_error("unknown error");
    return FM_ERR_HIP;
  }
}

template <class F>
int guarded_free(F&& f) {
  try {
    return f();
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed");
    return FM_ERR_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return FM_ERR_HIP;
  } catch (...) {
    set_error("unknown error");
    return FM_ERR_HIP;
  }
}

inline int bits_for(int64_t max_value) {
  int b = 1;
  while (b < 63 && (int64_t(1) << b) <= max_value) ++b;
  return b;
}

// shared host helpers (fm_capi.hip)
// the fused step's rule (fm_config.fuse_single, kp <= 16, tables above 256 MB unless FUSE_ON) for the
// single table
bool fuse_rule(const fm_ctx* ctx);
// stream st waits until a batch refilled by fm_batch_from_rows has been gathered (copy stream)
void wait_built(const fm_batch* b, hipStream_t st);
void upload_batch(fm_ctx* ctx, const fm_csr* c, fm_batch* b, bool check_range);
void reserve_work(fm_ctx* ctx, int64_t B, int64_t N);

// the sharded route (fm_shard_route) in two halves, for fm_group.hip: enqueue (counts stay in
// ctx->sh_tot on the device), then digest the host copy of those counts ([R] pairs, [R] entries)
// (on stream st: the group routes on a stream of its own, so the route does not queue behind the
// previous batch's owner preparation on the side stream)
void shard_route_launch(fm_ctx* ctx, fm_batch* b, void* send_slot, void* send_ent, hipStream_t st);
void shard_route_finish(fm_ctx* ctx, fm_batch* b, const unsigned long long* hc, int64_t* counts);
// sharded predict building blocks (fm_shard.hip), called by fm_group.hip with the member locked:
// the owner partial pass with the per-pair count of present rows (Model.scala:103-112 inner
// joins: absent ids contribute nothing), and the requester's predict epilogue
// (Model.scala:78-86, 127-132): w0 for a row without a learned feature, else clamp.
// chunk c of C (C > 1): only the chunk's pairs of every source (FwdOut::ch_*), for an exchange that
// sends each chunk while the next is computed; the profile event covers the last chunk
void shard_owner_partials(fm_ctx* ctx, fm_batch* b, void* partials_out, uint32_t* present_out, int chunk = 0,
                          int chunks = 1);
void shard_combine_predict(fm_ctx* ctx, fm_batch* b, const void* partials_in, const uint32_t* present_in,
                           double lo, double hi, double* pred_dev);

// multi-GPU contexts (fm_group.hip); each runs inside the group context's guarded()
int group_create(const fm_config* cfg, fm_ctx** out);
int group_batch_create(fm_ctx* ctx, const fm_csr* csr, fm_batch** out);
int group_batch_prepare(fm_ctx* ctx, fm_batch* b);
int group_batch_from_rows(fm_ctx* ctx, const fm_batch* data, const int64_t* rows, int64_t n, fm_batch** out);
int group_batch_create_splits(fm_ctx* ctx, const fm_csr* csr, int32_t n_splits, const int64_t* split_rows,
                              fm_batch** out);
int group_batch_split_view(fm_ctx* ctx, const fm_batch* data, int32_t split, fm_batch** out);
int group_step(fm_ctx* ctx, const fm_csr* csr, int32_t t, double step_size, double reg_param, fm_step_out* out);
int group_step_batch(fm_ctx* ctx, fm_batch* b, int32_t t, double step_size, double reg_param, fm_step_out* out);
int group_predict(fm_ctx* ctx, const fm_csr* csr, double lo, double hi, double* pred);
int group_predict_batch(fm_ctx* ctx, fm_batch* b, double lo, double hi, double* pred);
int group_load_tables(fm_ctx* ctx, const int32_t* ids, int64_t n, const double* w, const double* V);
int group_init_random(fm_ctx* ctx, const int32_t* ids, int64_t n, int64_t id_begin, int64_t id_end);
int group_init_from_batch(fm_ctx* ctx, fm_batch* b, int64_t* n_present);
int group_export_tables(fm_ctx* ctx, int32_t* ids, double* w, double* V, int64_t cap, int64_t* n);
int group_export_rows(fm_ctx* ctx, const int32_t* ids, int64_t n, double* w, double* V, int8_t* present);
int64_t group_num_present(fm_ctx* ctx);
int group_loss_history(fm_ctx* ctx, double* loss, int64_t cap, int64_t* n);
int group_last_stats(fm_ctx* ctx, double* loss_sum, int64_t* n_loss_rows, int64_t* n_unique);
int group_sync(fm_ctx* ctx);
int group_reserve(fm_ctx* ctx, int64_t max_rows, int64_t max_nnz);
int group_profile(fm_ctx* ctx, int op, int32_t on, char* names, int64_t names_cap, double* total_ms,
                  int64_t* launches, int64_t cap, int64_t* n);
fm_ctx* group_member0(fm_ctx* ctx);

}  // namespace fmhip
