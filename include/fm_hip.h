/*
 * fm_hip.h — C-ABI of the MI355X factorization-machine SGD hot path.
 *
 * This is the drop-in seam for Rainbowboys/fm_spark.  The reference has no FFI of its
 * own: the hot path is the fold body of FactorizationMachinesSGD.runMiniBatchSGD
 * (src/main/scala/org/apache/spark/ml/fm/FactorizationMachinesSGD.scala:116-211) plus the
 * DataFrame plan it builds through FactorizationMachinesModel.calcLossGrad
 * (FactorizationMachinesModel.scala:135-234).  Each entry point below names the reference
 * code it replaces.  A JNI binding for the Scala side is sketched in INTEGRATION.md.
 *
 * Conventions
 *   - plain C types only; every pointer argument is caller-owned and only borrowed for
 *     the duration of the call (host pointers unless the name says _device);
 *   - return codes: FM_OK (0) success, FM_NOTHING_TO_DO (1) an empty mini-batch
 *     (FactorizationMachinesSGD.scala:126-128), negative = error; the message is available
 *     from fm_last_error() on the calling thread.  No C++ exception, abort or exit crosses
 *     this boundary;
 *   - one fm_ctx owns one device's tables, or -- fm_config.parallel != FM_PARALLEL_NONE -- every
 *     rank of a multi-GPU job that this process drives: n_gpus devices from ONE host thread, the
 *     table row-sharded (or replicated) across them, the exchanges done inside the library over
 *     RCCL (xGMI), as SURVEY §8(b) Threading asks of the Spark driver.  Calls on one context are
 *     serialised by an internal mutex; independent contexts may run concurrently
 *     (CrossValidator keeps several models alive at once).
 *   - arithmetic: tables are fp32 on the device, accumulations fp64; inputs/outputs fp64.
 */
#ifndef FM_HIP_H
#define FM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FM_OK 0
#define FM_NOTHING_TO_DO 1
#define FM_ERR_ARG (-1)
#define FM_ERR_OOM (-2)
#define FM_ERR_HIP (-3)
#define FM_ERR_RCCL (-4)
#define FM_ERR_STATE (-5)

#define FM_PARALLEL_NONE 0       /* this context is one table (or one manual shard, shard_index/count) */
#define FM_PARALLEL_SHARDED 1    /* rows sharded by id % R over the job's R ranks, owner-computes */
#define FM_PARALLEL_REPLICATED 2 /* every rank holds the whole table; gradient all-reduce */
#define FM_TRANSPORT_AUTO 0      /* RCCL, unless a device repeats in devices[] (then COPY) */
#define FM_TRANSPORT_RCCL 1      /* RCCL send/recv and all-reduce over xGMI */
#define FM_TRANSPORT_COPY 2      /* one process only: device-to-device copies between the ranks */
#define FM_MAX_LOCAL 16
#define FM_FUSE_DEFAULT 0 /* fm_config.fuse_single: the library's choice (tables above 256 MB) */
#define FM_FUSE_ON 1
#define FM_FUSE_OFF (-1)

typedef struct fm_ctx fm_ctx;
typedef struct fm_batch fm_batch;

/* Model hyper-parameters fixed at creation.
 * num_features : feature ids are int32 in [0, num_features) (README.md:7 "<= Int.MaxValue").
 * k            : dimFactorization (FactorizationMachines.scala:26, >= 1).
 * w0           : globalBias (FactorizationMachinesModel.scala:45); fit always uses 0.0
 *                (FactorizationMachinesSGD.scala:246).
 * init_sd/seed : createInitialModel's N(0, initialSd^2) draw (FactorizationMachinesSGD.scala:234-241),
 *                made deterministic (the reference's draw is unseeded).
 * shard_index/shard_count : (parallel == FM_PARALLEL_NONE) row sharding by feature hash for a
 *                caller that drives the fm_shard_* phases itself; this context owns the ids with
 *                id % shard_count == shard_index (shard_count 1 = whole table).
 * parallel     : FM_PARALLEL_SHARDED / _REPLICATED: this context drives n_gpus local ranks
 *                (devices[0..n_gpus)) of a job of R = n_procs * n_gpus ranks; global rank of local
 *                rank l = proc_rank * n_gpus + l (every process uses the same n_gpus).  Mini-batches
 *                given to it are split by rows, contiguously, over the local ranks; the global
 *                miniBatchSize is the sum over all ranks (SGD.scala:124).  Replaces the shuffles
 *                S1/S2/S5/S6 of SURVEY §2b (Model.scala:155-164, SGD.scala:148-166).
 * transport    : how the ranks exchange (FM_TRANSPORT_*).  n_procs > 1 needs RCCL and comm_id:
 *                process 0 calls fm_comm_unique_id and hands the 128 bytes to the others by any
 *                channel (Spark broadcast, torch.distributed, a file).
 *                RCCL with R > 1 ranks has not run on hardware yet (every test box had one
 *                MI355X): the R > 1 protocol is verified through the COPY transport only.
 * fuse_single  : FM_FUSE_ON: a batch prepared by fm_batch_prepare on a single-table context with
 *                k <= 16 takes the fused step -- the forward updates every row whose feature has one
 *                entry in the batch, the segmented update only the rest (the same table as the
 *                unfused step within fp64 summation order); FM_FUSE_DEFAULT (0): the same, for tables
 *                larger than the 256-MB Infinity Cache; FM_FUSE_OFF: never.  Multi-GPU contexts
 *                never fuse (a sharded owner's fused step measured slower than the unfused one at
 *                R = 8 and at world 1).
 * xchg_chunks  : sharded step with R > 1: the owners' partial pass runs in this many chunks, each
 *                sent while the next is computed (0 = the default, 4; 1 = one pass then one
 *                all-to-all; at most 64).  Every process of a job must pass the same value.
 * Zero-initialise the struct: every field's 0 is its default. */
typedef struct fm_config {
  int64_t num_features;
  int32_t k;
  int32_t device;
  uint64_t seed;
  double init_sd;
  double w0;
  int32_t shard_index;
  int32_t shard_count;
  int32_t parallel;
  int32_t n_gpus;
  int32_t devices[FM_MAX_LOCAL];
  int32_t transport;
  int32_t n_procs;
  int32_t proc_rank;
  uint8_t comm_id[128];
  int32_t fuse_single;
  int32_t xchg_chunks;
} fm_config;

/* One mini-batch in CSR form: the result of explode(udfVecToMap(features))
 * (FactorizationMachinesModel.scala:148-153, 244-250).  Row i holds the active entries
 * of sample i (explicit zeros kept, one entry per index).  n_rows counts every sampled
 * row, including rows without active entries: it is miniBatchSize (SGD.scala:124). */
typedef struct fm_csr {
  int64_t n_rows;
  int64_t nnz;
  const int64_t* row_ptr; /* [n_rows + 1], row_ptr[0] == 0 */
  const int32_t* col;     /* [nnz] feature ids */
  const double* val;      /* [nnz] feature values */
  const double* label;    /* [n_rows] */
} fm_csr;

/* What one SGD iteration reports (SGD.scala:134-139 logs lossSum). */
typedef struct fm_step_out {
  double loss_sum;      /* sum over samples with >= 1 active entry of (yhat - y)^2 */
  int64_t n_rows;       /* miniBatchSize m */
  int64_t n_loss_rows;  /* samples contributing to loss_sum */
  int64_t n_unique;     /* distinct feature ids touched (U) */
} fm_step_out;

/* ---- context --------------------------------------------------------------------- */
/* Replaces: new FactorizationMachinesModel(uid, k, globalBias, ...) (Model.scala:43-48).
 * A multi-GPU context (parallel != FM_PARALLEL_NONE) accepts every entry point below except the
 * manual fm_shard_* / fm_repl_* phases, fm_set_stream / fm_set_side_stream (unless n_gpus == 1)
 * and fm_loss_grad / fm_calc_loss_grad on a sharded table (FM_ERR_ARG: the per-entry outputs
 * need every owner's rows on one device; replicated contexts answer them); the table entry points
 * act on the rows this process's ranks
 * hold (all rows when n_procs == 1). */
int fm_create(const fm_config* cfg, fm_ctx** out);
/* RCCL unique id for a job of several processes (ncclGetUniqueId), 128 bytes into id. */
int fm_comm_unique_id(uint8_t* id);
void fm_destroy(fm_ctx* ctx);
const char* fm_last_error(void);
/* Launch on an externally owned HIP stream (hipStream_t passed as void*); NULL = the device's
 * default (null) stream.  A new context launches on a non-blocking stream of its own. */
int fm_set_stream(fm_ctx* ctx, void* hip_stream);
/* The context's side stream (hipStream_t as void*), on which batch-only work runs ahead of its
 * step: fm_batch_prepare, fm_shard_route, fm_shard_owner_prepare.  NULL = the context's own
 * non-blocking side stream (the default). */
int fm_set_side_stream(fm_ctx* ctx, void* hip_stream);
/* Wait for everything the context has enqueued: its step stream, its side stream (preparations) and
 * its copy stream (fm_step uploads, fm_batch_from_rows gathers); a multi-GPU context, every rank's. */
int fm_sync(fm_ctx* ctx);
/* Pre-size the per-step workspace so no step allocates. */
int fm_reserve(fm_ctx* ctx, int64_t max_rows, int64_t max_nnz);

/* ---- tables (C9: Strength / FactorizedInteraction, Model.scala:275-289) ------------ */
/* Inject rows (id, w, V[k]) and mark them present: the M0 injection point. */
int fm_load_tables(fm_ctx* ctx, const int32_t* ids, int64_t n, const double* w, const double* V);
/* createInitialModel (SGD.scala:218-252): w, V ~ N(0, init_sd^2) for the given ids,
 * counter-based (seed, id, factor) so the draw is independent of order and shard. */
int fm_init_random(fm_ctx* ctx, const int32_t* ids, int64_t n);
/* Same for every id in [id_begin, id_end) (ids this shard does not own are skipped). */
int fm_init_random_range(fm_ctx* ctx, int64_t id_begin, int64_t id_end);
/* createInitialModel over a device-resident dataset (SGD.scala:224-241: the distinct active ids of
 * the data, then the random draw): every id of the batch's entries that this context owns and
 * that is absent gets the same draw as fm_init_random; present rows are kept.  Runs on the device
 * over the entries (the draw depends on (seed, id, factor) only, so no distinct pass is needed).
 * *n_present (may be NULL) receives the number of present rows afterwards. */
int fm_init_from_batch(fm_ctx* ctx, fm_batch* data, int64_t* n_present);
/* Export every present row owned by this context, ascending id, after applying the
 * pending L1 shrink.  cap = capacity in rows; *n receives the number of present rows
 * (call with cap 0 to size).  V is row-major [n][k]. */
int fm_export_tables(fm_ctx* ctx, int32_t* ids, double* w, double* V, int64_t cap, int64_t* n);
/* The rows of the given ids (each owned by this context) as they stand now, pending L1 shrink
 * applied, without exporting the whole table (the model Datasets queried by id: at F = Int.MaxValue
 * a full export is 2^31 rows).  present[i] = 1 for a present row, else 0 and a zero row.  V is
 * row-major [n][k]. */
int fm_export_rows(fm_ctx* ctx, const int32_t* ids, int64_t n, double* w, double* V, int8_t* present);
int64_t fm_num_present(fm_ctx* ctx);
/* Number of executed (non-empty) SGD steps. */
int64_t fm_epoch(fm_ctx* ctx);

/* ---- mini-batches --------------------------------------------------------------------- */
/* Copy a CSR batch into device memory once (validated: ids in range, row_ptr monotone). */
int fm_batch_create(fm_ctx* ctx, const fm_csr* csr, fm_batch** out);
void fm_batch_destroy(fm_batch* b);
/* Sort the batch's entries by feature (the grouping the gradient reduction consumes) ahead
 * of its step, on the context's side stream, so the sort overlaps whatever the previous step
 * still runs (input prefetch).  The prepared order is consumed by the next fm_step_batch on
 * this batch; a batch that was not prepared is sorted inside its step.  Stream-ordered, no
 * host synchronisation. */
int fm_batch_prepare(fm_ctx* ctx, fm_batch* batch);
/* The mini-batch of the given rows of a device-resident dataset, built on the device: row i of the
 * result is row rows[i] of data (any order, repeats allowed), with its label.  Replaces the split
 * of the cached training data that each SGD iteration consumes -- dfData.cache() and
 * dfData.randomSplit(...) (FactorizationMachinesSGD.scala:93, 111-112): the dataset crosses PCIe
 * once (fm_batch_create), each split is a row list (fm_random_split) gathered on the device.
 * data: a batch of this context made by fm_batch_create (the library keeps its row_ptr on the host
 * too, so the result is sized without a device read; the host pass runs on a pool of host threads).  *out == NULL: a new
 * batch is created; otherwise *out (a batch of this context, not data) is refilled in place.  The
 * gather runs on the context's copy stream behind every queued step, preparation and sharded
 * iteration that reads *out, and the host returns once it is enqueued (rows is copied); steps,
 * fm_batch_prepare, fm_predict_batch and fm_init_from_batch on the result are ordered after it.
 * data must stay alive until the gather has run: fm_sync waits for the context's step, side and
 * copy streams.  A multi-GPU context splits the selected rows contiguously over its local ranks,
 * as fm_batch_create splits a host CSR; each rank gathers its share from its own copy of the
 * dataset (made on its device from the dataset's parts at the first selection). */
int fm_batch_from_rows(fm_ctx* ctx, const fm_batch* data, const int64_t* rows, int64_t n, fm_batch** out);
/* A training dataset laid out split after split, made resident once: the rows of csr are the
 * randomSplit splits of the cached dfData concatenated in iteration order (FactorizationMachinesSGD
 * .scala:93, 111-112), split s = rows [split_rows[s], split_rows[s + 1]) (split_rows [n_splits + 1],
 * from 0 to n_rows; a last split may hold the rows no iteration samples), each split's rows in the
 * order its mini-batch takes them.  Each split is then a mini-batch in place: fm_batch_split_view
 * hands it to fm_batch_prepare / fm_step_batch with no copy and no gather (fm_batch_from_rows stays
 * for row lists that are not laid out beforehand).  The dataset itself is not stepped or prepared
 * (FM_ERR_ARG; its entries count their sample from their split's first row); fm_init_from_batch
 * (createInitialModel over every row) and fm_batch_from_rows (row i = row i of csr) accept it.  A
 * multi-GPU context cuts every split by rows over its local ranks, as it cuts a host CSR.  Synchronous (returns when the
 * dataset is on the device). */
int fm_batch_create_splits(fm_ctx* ctx, const fm_csr* csr, int32_t n_splits, const int64_t* split_rows,
                           fm_batch** out);
/* Split `split` of a dataset made by fm_batch_create_splits as a mini-batch: its rows, entries and
 * labels where they lie in data (borrowed -- data must outlive the view and every step queued on
 * it).  *out == NULL: a new batch; otherwise *out is re-pointed in place.  Re-pointing a view is
 * host-only, no device work, so a loop re-points the batch it has just stepped while that step still
 * runs (its next fm_batch_prepare waits for it).  The first conversion of a batch that owns device
 * buffers (one made by fm_batch_create or fm_batch_from_rows) into a view blocks: it waits for the
 * batch's queued work, then frees its buffers. */
int fm_batch_split_view(fm_ctx* ctx, const fm_batch* data, int32_t split, fm_batch** out);
/* 1 if a batch prepared by fm_batch_prepare on this context takes the fused step (fm_config.fuse_single
 * and the library's rule: a single-table context, k <= 16, table above 256 MB unless FM_FUSE_ON;
 * multi-GPU contexts never fuse), else 0; -1 for a null context. */
int32_t fm_fuse_active(fm_ctx* ctx);
int64_t fm_batch_rows(const fm_batch* b);
int64_t fm_batch_nnz(const fm_batch* b);

/* ---- the hot path ------------------------------------------------------------------- */
/* One mini-batch SGD iteration = the foldLeft body, SGD.scala:116-211:
 *   eta = step_size / sqrt(t); lambda = eta * reg_param (SGD.scala:121-122)
 *   forward + loss                      (Model.scala:148-233; SGD.scala:134-138)
 *   per-feature gradient sums           (SGD.scala:142-155; note SURVEY P1: g_w = x*yhat - y)
 *   w -= (sum g_w / m) * eta; V -= (sum g_V) * (eta / m)      (SGD.scala:150-154,171-175)
 *   soft-threshold S_lambda on EVERY present row              (SGD.scala:177-181)
 * t is the 1-based iteration index (tuple._2 + 1, SGD.scala:119).  Returns
 * FM_NOTHING_TO_DO for n_rows == 0 without touching the model (SGD.scala:126-128).
 * fm_step takes the host batch (borrowed for the call only: it is exploded into pinned staging
 * by host threads, then copied asynchronously); fm_step_batch uses a device-resident batch.
 * With out == NULL both only enqueue (no host synchronisation; losses are kept on the device,
 * see fm_loss_history): consecutive fm_step calls then overlap the next batch's host work and
 * copies with the current step (two upload slots used in turn). */
int fm_step(fm_ctx* ctx, const fm_csr* batch, int32_t t, double step_size, double reg_param,
            fm_step_out* out);
int fm_step_batch(fm_ctx* ctx, fm_batch* batch, int32_t t, double step_size,
                  double reg_param, fm_step_out* out);
/* Per-step loss sums of every executed step so far (SGD.scala:139 log line). */
int fm_loss_history(fm_ctx* ctx, double* loss, int64_t cap, int64_t* n);

/* ---- inference & diagnostics ------------------------------------------------------- */
/* FactorizationMachinesModel.transform/predict (Model.scala:69-133): ids absent from the
 * model (or >= num_features) are dropped (inner joins, :103-112); a row with no learned
 * feature gets w0 unclamped (na.fill, :86); otherwise clamp(yhat, min_label, max_label)
 * (:129-132).  Pass -inf/+inf for the unclamped score. */
int fm_predict(fm_ctx* ctx, const fm_csr* csr, double min_label, double max_label, double* pred);
/* The same on a device-resident batch (fm_batch_create): transform over a cached DataFrame
 * without re-uploading it.  pred is a host buffer of fm_batch_rows(batch) doubles. */
int fm_predict_batch(fm_ctx* ctx, fm_batch* batch, double min_label, double max_label, double* pred);
/* calcLossGrad (Model.scala:135-234), per active entry e in CSR order:
 * pred[e] = yhat of its row (unclamped), loss[e] = (yhat - y)^2, delta_w[e] = x,
 * delta_v[e*k + f] = vfxiSum_f * x - (v_f * x) * x.  Any output may be NULL.
 * Ids absent from the model are an error here (the reference fills them with an
 * unseeded random draw, Model.scala:170-171, which is never reached from fit). */
int fm_loss_grad(fm_ctx* ctx, const fm_csr* csr, double* pred, double* loss, double* delta_w,
                 double* delta_v);
/* calcLossGrad(dfSampleIndexed, initialSd) with the reference's fill for ids the model lacks
 * (Model.scala:144-146, 170-171: coalesce(strength, randn() * initialSd) and udfInitVec() per
 * joined row): every entry whose id is absent (or >= num_features) gets its own w and v drawn
 * from N(0, initial_sd^2) -- keyed by (seed, entry index in CSR order, column), so a call is
 * reproducible where the reference's draws are unseeded.  initial_sd must be > 0 (:136).
 * Refused on a row-sharded multi-GPU context (see fm_create). */
int fm_calc_loss_grad(fm_ctx* ctx, const fm_csr* csr, double initial_sd, uint64_t seed, double* pred,
                      double* loss, double* delta_w, double* delta_v);
/* VectorSum UDAF + groupBy (FactorizationMachines.scala:45-81): for every distinct key,
 * the element-wise fp64 sum of its k-vectors in input order.  Output ascending by key;
 * *n_out = number of distinct keys (<= n).  Runs the device sort + segmented reduction. */
int fm_vector_sum_by_key(fm_ctx* ctx, const int32_t* keys, int64_t n, const double* vecs,
                         int32_t k, int32_t* out_keys, double* out_sums, int64_t* n_out);

/* Per-kernel device time of the last fm_step_batch calls, measured with HIP events on the
 * launch stream when enabled (names: "forward", "sort", "update", ...). */
int fm_profile_enable(fm_ctx* ctx, int32_t on);
/* Writes up to cap entries: names as a '\n'-joined string into names (size names_cap),
 * total milliseconds and launch counts per kernel; *n = number of kernels. */
int fm_profile_read(fm_ctx* ctx, char* names, int64_t names_cap, double* total_ms,
                    int64_t* launches, int64_t cap, int64_t* n);
int fm_profile_reset(fm_ctx* ctx);

/* ---- input format: Spark 2.1 `libsvm` data source (data/sample.txt, config c1) ------------ */
/* MLUtils.parseLibSVMFile semantics: trimmed lines, '#'-lines and empty lines skipped, one-based
 * strictly ascending indices (stored 0-based), numFeatures = max last index + 1 (an empty row
 * counts as index 0).  Call with cap_rows = cap_nnz = 0 to size: *n_rows, *nnz, *num_features
 * are always filled; then again with buffers label[n_rows], row_ptr[n_rows + 1], col[nnz],
 * val[nnz].  A malformed line is an FM_ERR_ARG with the line in fm_last_error(). */
int fm_read_libsvm(const char* path, int64_t cap_rows, int64_t cap_nnz, double* label, int64_t* row_ptr,
                   int32_t* col, double* val, int64_t* n_rows, int64_t* nnz, int64_t* num_features);

/* ---- mini-batch sampler: Dataset.randomSplit replay (SGD.scala:111-112) --------------- */
/* Host-side replay of Spark 2.1.0 randomSplit(weights, seed) on a cached DataFrame whose
 * rows are given partition by partition (part_ptr[n_parts+1]).  Each partition is sorted
 * ascending by all columns in schema order (column_order: 'L' label double, 'F' features
 * vector, 'I' int64 column extra[] ; sampleId is appended last), then split i keeps the
 * rows whose XORShiftRandom(seed + partition).nextDouble() falls in
 * [cumw[i], cumw[i+1]).  Features: vec_type (0 sparse, 1 dense), vec_size,
 * vec_ptr[n+1], vec_idx (sparse only; ignored for dense), vec_val.
 * Outputs: split_of[n] (-1 = in no split), sample_id[n] = (partition << 33) + row index
 * (monotonically_increasing_id, Model.scala:268-272), order[n] = row indices in sorted
 * (per-partition) order.  Partitions are sorted and sampled in parallel on the library's host
 * thread pool (each writes only its own rows; the result does not depend on the thread count);
 * an allocation failure is FM_ERR_OOM. */
int fm_random_split(int32_t n_parts, const int64_t* part_ptr, const char* column_order,
                    const double* label, const int8_t* vec_type, const int32_t* vec_size,
                    const int64_t* vec_ptr, const int32_t* vec_idx, const double* vec_val,
                    const int64_t* extra, int32_t n_weights, const double* weights,
                    int64_t seed, int32_t* split_of, int64_t* sample_id, int64_t* order);
/* The building blocks, exported for the parity tests. */
int64_t fm_xorshift_hash_seed(int64_t seed);
int32_t fm_murmur3_bytes_hash(const uint8_t* data, int64_t len, int32_t seed);
/* n successive nextDouble() of XORShiftRandom(seed). */
int fm_xorshift_next_doubles(int64_t seed, int64_t n, double* out);

/* ---- row-sharded multi-GPU step (owner-computes) -----------------------------------------
 * One context per rank (fm_config.shard_index / shard_count = rank / R, R <= 64; the owner of
 * feature id is id % R, its local slot id / R).  The caller exchanges the device buffers
 * between phases with all-to-all (RCCL over xGMI; fm_spark_amd/distributed.py).  Replaces the
 * feature-keyed shuffles S1/S2/S5/S6 and the per-sample window of the reference plan
 * (Model.scala:155-164, :191, SGD.scala:148-166).
 * A "pair" is (sample of a source rank, owner holding some of its entries).  Wire buffers are fp32
 * structures of arrays over P pairs, kp + 2 fp32 words per pair (kp = roundup(k, 4)):
 *   partials = [P][kp] sum v*x, then [P][2] {sum v^2 x^2, sum w*x}
 *   S        = [P][kp] vfxiSum, then [P][2] {r, yhat}  (the residual r = yhat - y is formed in fp64
 *              from the fp64 label, as the reference's Double column, SGD.scala:145-146, and rounded
 *              once; the owner forms g_w = x*yhat - y as (x - 1)*yhat + r)
 * so the exchange is two all-to-alls per direction (the vector section, the scalar section).
 * Every phase is keyed by `batch`, this rank's mini-batch of the iteration; its state lives with
 * the batch.  Phases 1 and 1b depend on the batch alone and run on the side stream
 * (fm_set_side_stream), so the next iteration's routing, entry exchange and slot sort overlap the
 * current iteration; phases 2-4 run on the main stream and wait for them through events.
 * Phase 1 (requester): partition the batch's entries by owner, CSR order kept, into
 * send_slot (uint32 local slots, N) and send_ent ({index of the entry's (sample, owner) pair
 * among this rank's pairs to that owner, x bits}, N) -- device buffers of the batch's nnz.
 * counts[0..R) = entries to each owner, counts[R..2R) = pairs to each owner.
 * Synchronises the side stream (not the main stream). */
int fm_shard_route(fm_ctx* ctx, fm_batch* batch, void* send_slot, void* send_ent, int64_t* counts);
/* Phase 1b (owner): the n received entries (source-rank major: src_entries[r] from rank r, which
 * sent src_pairs[r] pairs) -> their pair table and their order by slot (stable: source rank,
 * then CSR order), kept with `batch`.  No host synchronisation.  recv_slot / recv_ent must stay
 * valid until the main stream has run fm_shard_owner_forward of this batch. */
int fm_shard_owner_prepare(fm_ctx* ctx, fm_batch* batch, const void* recv_slot, const void* recv_ent,
                           int64_t n, const int64_t* src_entries, const int64_t* src_pairs);
/* Phase 2 (owner): partials_out[sum src_pairs] (source-major, sample order): per received pair
 * the partial forward sums over the entries this rank owns, lazy L1 caught up on read. */
int fm_shard_owner_forward(fm_ctx* ctx, fm_batch* batch, void* partials_out);
/* Phase 3 (requester): the partials received from the owners (owner-major, counts[R + o] rows
 * from owner o) -> per sample S, yhat and the loss; s_send gets the S rows in the same layout. */
int fm_shard_combine(fm_ctx* ctx, fm_batch* batch, const void* partials_in, void* s_send);
/* Phase 4 (owner): the S rows received for its pairs (same order as its partials) -> per-slot
 * gradient sums over the slot-sorted entries, update + L1 with global miniBatchSize global_rows
 * (the sum of every rank's rows).  Returns FM_NOTHING_TO_DO when global_rows == 0 (every rank
 * skips, SGD.scala:126-128). */
int fm_shard_owner_update(fm_ctx* ctx, fm_batch* batch, const void* s_recv, int32_t t, double step_size,
                          double reg_param, int64_t global_rows);

/* ---- replicated multi-GPU step (small tables) --------------------------------------------
 * Every rank holds the whole table (shard_count = 1, same seed / same loaded tables) and steps
 * its own rows of the global mini-batch.
 * Phase 1: forward, sort and per-slot gradient sums of this rank's batch into the device
 * buffer grad[num_features][kp + 4] fp32 = [sum g_V (kp) | sum g_w | touched | 0] (zeroed
 * first; an empty batch contributes zeros and returns FM_NOTHING_TO_DO).
 * The caller all-reduces grad (sum; RCCL over xGMI), then
 * Phase 2: the update + L1 of SGD.scala:150-181 on every touched row with global miniBatchSize
 * global_rows; identical on every rank, so the replicas stay identical.  Returns
 * FM_NOTHING_TO_DO when global_rows == 0. */
int fm_repl_grad(fm_ctx* ctx, fm_batch* batch, void* grad);
int fm_repl_apply(fm_ctx* ctx, const void* grad, int32_t t, double step_size, double reg_param,
                  int64_t global_rows);

/* Statistics of the last step on this context: loss sum and loss rows of its samples, distinct
 * ids (sharded: those this rank owns; replicated: touched rows of the whole step).  Multi-GPU
 * callers all-reduce the first two (SGD.scala:134-139). */
int fm_last_stats(fm_ctx* ctx, double* loss_sum, int64_t* n_loss_rows, int64_t* n_unique);

#ifdef __cplusplus
}
#endif

#endif /* FM_HIP_H */
