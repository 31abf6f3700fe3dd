#!/usr/bin/env python3
"""FM mini-batch SGD throughput on MI355X (BASELINE.json metric: train samples/s at k=16).

One "step" = one fm_step over one device-resident synthetic mini-batch: forward + loss,
stable sort of the entries by feature, segmented gradient reduction and the fused
update + L1 over the model tables.  Workload (default) = config c3 of BASELINE.json:
100M hashed features, k = 16, 256K rows per mini-batch (per GPU), 39 active entries per
row (Criteo-shaped synthetic data); stepSize 0.1, regParam 1e-6.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

N = 1 runs the single-table path (fused step: the forward updates the rows whose feature has one
entry in the batch).  N > 1 row-shards the table (owner = id mod N; --parallel replicated keeps a
whole table per GPU) and exchanges entries / partial sums / S rows with RCCL all-to-all inside
libfm_hip (weak scaling: every rank steps its own 256K-row batch each iteration).  Without a
launcher, --gpus N drives N GPUs from this one process through one multi-GPU fm_ctx (the Spark
driver's path); under torch.distributed.run each process drives its own GPU.  Asking for more GPUs
than are visible exits non-zero.  Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# HIP maps a process's streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by default);
# two streams on one queue run in submission order, so the library's main, side and exchange streams
# must not share one with each other or with torch's ("Hardware queues").  Set before
# anything initialises HIP.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (num_features, k, rows per batch, zipf_s, description)
    "c2": (1_000_000, 8, 65_536, 1.05, "synthetic Criteo-shaped 1M features, 39 nnz/row, k=8, batch 64K"),
    "c3": (100_000_000, 16, 262_144, 1.05, "synthetic hashed 100M features, 39 nnz/row, k=16, batch 256K"),
    "c4": (2_147_483_647, 32, 262_144, 1.05, "Int.MaxValue features, 39 nnz/row, k=32, batch 256K"),
    # c5: the CrossValidator config's step (one grid point: k = 16; regression labels); hot rows
    "c5": (1_000_000, 16, 65_536, 1.2, "Zipf(1.2) hashed 1M features, 39 nnz/row, k=16, batch 64K, regression"),
}
STEP_SIZE = 0.1
REG_PARAM = 1e-6
INIT_SD = 0.01
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--batches", type=int, default=4, help="distinct resident mini-batches cycled through")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-steps", type=int, default=2)
    p.add_argument("--profile-kernels", type=int, default=1, help="HIP-event timing of each kernel phase")
    p.add_argument("--profile-every", type=int, default=4,
                   help="time the kernel phases of every n-th timed step (HIP events cost ~2 %% of a c3 step, "
                        "~12 %% of a c5 step when every step carries them)")
    p.add_argument("--features", type=int, default=0, help="override num_features (experiments)")
    p.add_argument("--k", type=int, default=0, help="override k (experiments)")
    p.add_argument("--rows", type=int, default=0, help="override rows per batch (experiments)")
    p.add_argument("--zipf", type=float, default=0.0, help="override the Zipf exponent (c5's hot rows: 1.2)")
    p.add_argument("--force-sharded", action="store_true",
                   help="N = 1: run the multi-GPU group context (RCCL, one rank) instead of the single table")
    p.add_argument("--parallel", default="auto", choices=["auto", "sharded", "replicated"],
                   help="multi-GPU table layout: row-sharded by id %% R or replicated with a gradient all-reduce "
                        "(auto: replicated for c2, else sharded); given explicitly at N = 1 it implies the group path")
    p.add_argument("--no-prefetch", action="store_true",
                   help="sort each batch inside its own step instead of during the previous step")
    p.add_argument("--host-path", action="store_true",
                   help="single table: time fm_step with the host CSR each call (PCIe-inclusive, as a JNI "
                        "caller sees it) instead of device-resident batches; reported, never the headline")
    p.add_argument("--prefetch-depth", type=int, default=0,
                   help="how many steps ahead a batch is prepared: sorted on the side stream, or "
                        "sharded, routed (and its entries exchanged and slot-sorted) on the side streams; 0 = 1 for "
                        "the single table (c3, 20-step runs: 0.990-0.997 against 1.000-1.004 ms for 2, 1.017-1.024 for "
                        "3; profiles/r03_v15/depth), 2 for a group (two-phase prepare: each route gets a step)")
    p.add_argument("--copy-ranks", type=int, default=0,
                   help="measurement only: run an R-rank group job on GPU 0 (COPY transport), e.g. to time the "
                        "one host thread's per-iteration enqueue at R = 8; the line is not a multi-GPU result")
    p.add_argument("--fuse", default="auto", choices=["auto", "on", "off"],
                   help="single table, k <= 16: the fused step (the forward updates the rows whose feature has one "
                        "entry in the batch; fm_config.fuse_single): auto = the library's default (tables larger "
                        "than the 256-MB Infinity Cache), on, off")
    p.add_argument("--trainer", default="lib", choices=["lib", "torch"],
                   help="N > 1: 'lib' = the multi-GPU fm_ctx, every exchange inside libfm_hip over RCCL (the "
                        "C-ABI path); 'torch' (torch.distributed.run only) = the torch.distributed test harness "
                        "(fm_spark_amd/distributed.py) driving the fm_shard_* phases")
    p.add_argument("--fit-iters", type=int, default=16,
                   help="N = 1: after the timed region, run the estimator's resident mini-batch loop "
                        "(fm_spark_amd.ml.run_minibatch_sgd_resident, what FactorizationMachinesSGD.fit runs after its "
                        "randomSplit replay) over a resident synthetic dataset of this many batches' rows, split by "
                        "the randomSplit replay into as many iterations, for fit_ms_per_iter; 0 = skip")
    p.add_argument("--host-path-steps", type=int, default=12,
                   help="N = 1: after the timed region, time this many fm_step calls with the host CSR "
                        "(PCIe-inclusive, what a JNI caller gets) for host_path_ms_per_step; 0 = skip")
    return p.parse_args()


def median_step_ms(events):
    """Median of the per-step device times between consecutive step-start events (BASELINE.md:
    median over >= 20 steps); the events sit on the stream the steps are launched on."""
    d = [events[i].elapsed_time(events[i + 1]) for i in range(len(events) - 1)]
    return float(np.median(d)) if d else None


XGMI_LINK_GBS = 153.0  # per direction per link (MI355X: 7 links to the 7 peers of an 8-GPU node)


def exchange_bytes(b, R, r, kp):
    """Per iteration, what rank r sends over xGMI for its own batch b in the sharded step
    (include/fm_hip.h wire formats): its entries to remote owners (4 B slot + 8 B {pair, x}), the
    S rows back to them ((kp + 4) words per remote pair); as an owner it returns a partial row per
    pair it received (about the same count by symmetry of the hashed ids)."""
    ids = b.col.astype(np.int64)
    owner = ids % R
    sample = np.repeat(np.arange(b.n_rows, dtype=np.int64), np.diff(b.row_ptr))
    pairs = np.unique(sample * R + owner)
    ent_remote = int(np.count_nonzero(owner != r))
    pair_remote = int(np.count_nonzero(pairs % R != r))
    row = (kp + 4) * 4
    return {"entries_B": 12 * ent_remote, "s_rows_B": row * pair_remote, "partials_B": row * pair_remote,
            "remote_entries": ent_remote, "remote_pairs": pair_remote}


def host_path_leg(ctx, host_batches, t, steps, torch):
    """fm_step with a host CSR every call (staged, copied over PCIe, exploded on the device, then
    the step): the rate a JNI caller sees.  Two warm-up calls, then `steps` timed calls, each
    bracketed by events on the context's stream; returns (median ms, mean ms, next t)."""
    from fm_spark_amd._native import CSRHost

    hosts = [CSRHost(b.row_ptr, b.col, b.val, b.label) for b in host_batches]
    st = torch.cuda.current_stream()
    for i in range(2):
        t += 1
        ctx.step(hosts[i % len(hosts)], t, STEP_SIZE, REG_PARAM, sync=False)
    ctx.sync()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i].record(st)
        t += 1
        ctx.step(hosts[i % len(hosts)], t, STEP_SIZE, REG_PARAM, sync=False)
    evs[steps].record(st)
    ctx.sync()
    torch.cuda.synchronize()
    mean = 1000.0 * (time.perf_counter() - t0) / steps
    return median_step_ms(evs), mean, t


def fit_leg(ctx, F, B, zipf_s, lab, iters, parts=16):
    """The estimator's mini-batch loop on a resident dataset (what FactorizationMachinesSGD.fit runs
    after its randomSplit replay, fm_spark_amd/ml.py run_minibatch_sgd_splits): a synthetic dataset
    of `iters` x B rows in `parts` partitions, split by the randomSplit replay into `iters` splits of
    about B rows (randomSplit normalises the weights: each split gets 1/iters of the rows, :111-112),
    is uploaded once laid out split after split (dfData.cache(), SGD.scala:93; fm_batch_create_splits),
    and the loop -- each split stepped in place through a view, sorted on the side stream while the
    previous one steps -- runs twice: once to grow the views' sort buffers and the step workspace
    (kept for the second), once timed (host clock around the whole loop, the final sync included:
    the pipeline's fill -- the first split's sort, nothing to overlap -- counts against it)."""
    from fm_spark_amd._native import CSRHost
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.ml import _select_csr, run_minibatch_sgd_splits
    from fm_spark_amd.sampler import random_split_csr

    t0 = time.perf_counter()
    ds = concat_batches([synthetic_batch(B, F, batch_index=7000 + i, zipf_s=zipf_s, **lab) for i in range(iters)])
    n = ds.n_rows
    sizes = [n * (i + 1) // parts - n * i // parts for i in range(parts)]
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    split_of, _, order = random_split_csr(sizes, ds.label, ds.row_ptr, ds.col, ds.val, F, [0.1] * iters, 1234)
    t_sampler = time.perf_counter() - t0
    t0 = time.perf_counter()
    splits = [order[split_of[order] == i] for i in range(iters)]
    rest = order[split_of[order] < 0]
    lay = _select_csr(ds.row_ptr, ds.col, ds.val, ds.label, np.concatenate(splits + [rest]).astype(np.int64))
    split_rows = np.concatenate([[0], np.cumsum([len(r) for r in splits] + [len(rest)])])
    t_layout = time.perf_counter() - t0
    t0 = time.perf_counter()
    data = ctx.batch_splits(lay, split_rows)
    ctx.sync()
    t_upload = time.perf_counter() - t0
    bufs = [None, None]  # the two views used in turn, kept across the loops
    run_minibatch_sgd_splits(ctx, data, STEP_SIZE, REG_PARAM, n_iter=iters, bufs=bufs)  # untimed: buffers grown
    half = iters // 2
    t0 = time.perf_counter()
    run_minibatch_sgd_splits(ctx, data, STEP_SIZE, REG_PARAM, n_iter=half, bufs=bufs)
    dt_half = time.perf_counter() - t0
    t0 = time.perf_counter()
    losses = run_minibatch_sgd_splits(ctx, data, STEP_SIZE, REG_PARAM, n_iter=iters, bufs=bufs)
    dt = time.perf_counter() - t0
    for b in bufs:
        b.close()
    data.close()
    rows = [len(r) for r in splits]
    return {"fit_ms_per_iter": 1e3 * dt / iters, "iterations": iters, "rows_per_iter_mean": float(np.mean(rows)),
            "fit_ms_per_iter_steady": 1e3 * (dt - dt_half) / (iters - half) if iters > half else None,
            "samples_per_s": float(np.sum(rows)) / dt, "dataset_rows": n, "partitions": parts,
            "finite_losses": bool(np.all(np.isfinite(losses))),
            "setup_s": {"generate": t_gen, "random_split": t_sampler, "layout": t_layout, "upload_once": t_upload,
                        "random_split_threads": sampler_threads()},
            "what": "FactorizationMachinesSGD.fit's mini-batch loop on the resident dataset laid out split after "
                    "split (fm_batch_create_splits): each randomSplit split stepped in place through a view "
                    "(fm_batch_split_view: no copy, no gather) and sorted on the side stream while the previous split "
                    "steps; host clock over the whole loop incl. the pipeline fill (fit_ms_per_iter), and the loop over "
                    "all splits minus the loop over the first half, per iteration (fit_ms_per_iter_steady: the fill "
                    "cancels)"}


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def sampler_threads():
    # fm_random_split's partitions run on the library's host pool: min(16, hardware threads)
    return min(16, os.cpu_count() or 1)


def algorithmic_bytes(F, k, B, z, U):
    """A = 8z + 12 + 4z(k+1) + 8(k+1) U/B bytes per sample, split by kernel."""
    fwd = B * (8 * z + 12 + 4 * z * (k + 1))  # CSR col+val, row_ptr+label, gather of w+V
    upd = 8 * (k + 1) * U  # read + write of every touched row
    return fwd, upd


# HIP kernels behind each timed phase (the "update" phase is the segmented update + its combine)
PHASE_KERNELS = {"forward": ["k_forward"], "update": ["k_segment_update", "k_segment_combine"],
                 "owner_forward": ["k_forward"], "owner_update": ["k_segment_update", "k_segment_combine"]}


def pmc_traffic(F, k, B, phase, fused=False, world=1):
    """HBM bytes per launch of `phase` from the committed rocprofv3 PMC passes of this workload
    (profiles/pmc_*.json, made by tools/pmc.sh + tools/pmc_to_json.py with the calibrated
    FETCH_SIZE/WRITE_SIZE corrections; "fused" says which step variant the passes measured, "mode"
    whether the single-table step or the sharded owner phases).  None when no pass of this exact
    workload and variant is committed."""
    mode = "sharded" if phase.startswith("owner_") else "single"
    for f, d in _pmc_files(F, k, B, fused, mode, world):
        ks = d.get("kernels", {})
        names = PHASE_KERNELS.get(phase, [])
        if names and all("traffic_bytes" in ks.get(n, {}) for n in names):
            return sum(ks[n]["traffic_bytes"] for n in names), os.path.relpath(f, ROOT) + " (" + d.get("build", "") + ")"
    return None, None


# Random-line request ceiling of the L2 (TCC_HIT + TCC_MISS per second) on MI355X, measured by
# tools/gather_bench.hip with the same counters (profiles/r04_gather): the rate random 64/128-B row
# gathers saturate at, whatever bytes each request carries.  The gather-bound kernels are judged
# against it as well as against HBM bytes.
L2_REQ_CEILING_GPS = L2_REQ_UNIFORM_GPS = None
C3_SKELETON = None  # the fused forward's memory skeleton replayed on c3's own stream: {ms, l2_requests, ...}
try:
    with open(os.path.join(ROOT, "profiles", "gather_ceiling.json")) as _fh:
        _gc = json.load(_fh)
    L2_REQ_CEILING_GPS = float(_gc["l2_requests_per_s"]) / 1e9          # best variant (40 % hot rows)
    L2_REQ_UNIFORM_GPS = float(_gc["uniform_l2_requests_per_s"]) / 1e9  # uniformly random rows
    C3_SKELETON = (_gc.get("c3_stream") or {}).get("variants", {}).get("gather<8,5,32,3>")
except (OSError, ValueError, KeyError, TypeError):
    pass


def _pmc_files(F, k, B, fused, mode, world, group=None):
    """The committed PMC files of this workload; with `group` ("lsd"), those counted
    with that grouping sort first, then those that do not say."""
    import glob

    hits = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("num_features"), d.get("k"), d.get("batch_rows"), bool(d.get("fused", False)),
                d.get("mode", "single"), d.get("world", 1)) == (F, k, B, fused, mode, world):
            g = d.get("grouping")
            if group is None or g in (None, group):
                hits.append((g is None, f, d))
    for _, f, d in sorted(hits, key=lambda h: h[0]):
        yield f, d


def _requests(kc):
    c = kc.get("counters", {})
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        return c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
    return None


def pmc_requests(F, k, B, phase, fused=False, world=1):
    """L2 requests (TCC_HIT + TCC_MISS) per launch of `phase` from the committed PMC passes, or None."""
    mode = "sharded" if phase.startswith("owner_") else "single"
    for f, d in _pmc_files(F, k, B, fused, mode, world):
        ks = d.get("kernels", {})
        names = PHASE_KERNELS.get(phase, [])
        vals = [_requests(ks.get(n, {})) for n in names]
        if names and all(v is not None for v in vals):
            return sum(vals), os.path.relpath(f, ROOT)
    return None, None


def requests_roof(req, seconds):
    """The request-rate side of the roofline: L2 requests per second against the measured random-line
    ceiling (L2_REQ_CEILING_GPS)."""
    if not req or not seconds:
        return None
    rate = req / seconds / 1e9
    return {"l2_requests": req, "achieved_G_per_s": rate, "ceiling_G_per_s": L2_REQ_CEILING_GPS,
            "frac": rate / L2_REQ_CEILING_GPS if L2_REQ_CEILING_GPS else None,
            "uniform_random_G_per_s": L2_REQ_UNIFORM_GPS,
            "frac_of_uniform": rate / L2_REQ_UNIFORM_GPS if L2_REQ_UNIFORM_GPS else None,
            "ceiling_source": "profiles/gather_ceiling.json (tools/gather_ceiling.hip, TCC_HIT + TCC_MISS per second: "
                              "the best variant, 40 % of the gathers on 1000 hot rows; and uniformly random rows)"}


def sort_passes(num_rows):
    """Digit passes of the feature-slot radix sort (fm_sort.hip digit_bits: at most 10-bit digits,
    spread evenly, never narrower than 9 bits)."""
    kb = max(1, int(num_rows - 1).bit_length())
    p = -(-kb // 10)
    rb = max(9, -(-kb // p))
    return -(-kb // rb)


def step_kernels(F, fused):
    """Launches per single-table step of each kernel (fm_capi.hip step_impl / fm_batch_prepare,
    fm_sort.hip): the forward, update and combine; count / chunk scan / chunk top / scatter per
    digit pass of the LSD sort (+ the split kernels at the step, which tag the multi rows, fused)."""
    ps = {"k_forward": 1, "k_segment_update": 1, "k_segment_combine": 1}
    passes = sort_passes(F)
    if fused:  # the split at the step, its count pass writing the multi tags
        ps.update({"k_split_count": 1, "k_split_scan": 1, "k_split_scatter": 1})
    ps.update({"k_radix_count": passes, "k_radix_chunk_scan": passes, "k_radix_chunk_top": passes,
               "k_radix_scatter": passes})
    return ps


def step_traffic(F, k, B, fused):
    """Counted HBM bytes and L2 requests of one whole single-table step: every kernel's per-launch
    figures in the committed PMC passes of this workload times its launches per step (the file's
    "per_step" map when it has one, else step_kernels).  None unless every kernel of the step was
    counted."""
    per_step = step_kernels(F, fused)
    for f, d in _pmc_files(F, k, B, fused, "single", 1, "lsd"):
        ks = d.get("kernels", {})
        ps = d.get("per_step", per_step)
        if all("traffic_bytes" in ks.get(kn, {}) for kn in ps):
            req = [_requests(ks[kn]) for kn in ps]
            return (sum(ks[kn]["traffic_bytes"] * c for kn, c in ps.items()),
                    sum(r * c for r, c in zip(req, ps.values())) if all(r is not None for r in req) else None,
                    os.path.relpath(f, ROOT) + " (" + d.get("build", "") + ")")
    return None, None, None


def cpu_baseline(cfg, batch, steps):
    """The fp64 C restatement (oracle/fm_oracle.c, OpenMP) timed on this host's cores on a
    bounded sample of the same workload: `steps` mini-batch steps over the full table."""
    import ctypes as C

    from oracle import oracle_c

    F, k, B, _, _ = cfg
    lib = oracle_c.load()
    threads = oracle_c.threads(lib)
    m = oracle_c.create(lib, F, k)
    try:
        t0 = time.perf_counter()
        lib.oracle_init_random(m, 12345, INIT_SD, 0, F)
        t_init = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i in range(steps):
            oracle_c.step(lib, m, batch, i + 1, STEP_SIZE, REG_PARAM)
        dt = time.perf_counter() - t0
    finally:
        lib.oracle_destroy(m)
    return {
        "value": steps * B / dt,
        "unit": "samples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{steps} mini-batch steps x {B} rows on the full F={F} k={k} table (fp64, eager L1 over "
                  f"every row as the reference; init {t_init:.1f}s excluded), oracle/fm_oracle.c",
    }


class PlanError(SystemExit):
    """An impossible request: bench.py exits non-zero with this message instead of measuring
    something other than what was asked (never a silent downgrade to fewer GPUs)."""


NNZ_PER_ROW = 39  # the synthetic Criteo-shaped rows (fm_spark_amd/data.py N_FIELDS)


def auto_parallel(F, k, B, z, R):
    """The layout whose per-rank exchange is smaller at R ranks ("c2 at N = 8"): the
    replicated step all-reduces a dense F x (kp + 4) fp32 buffer (a ring moves 2 (R - 1) / R of it per
    rank), the sharded step sends every (sample, owner) pair's partial sums and S row, kp + 2 fp32
    each way (a sample's z ids meet R (1 - (1 - 1/R)^z) owners on average; (R - 1) / R of them
    remote).  c2 (1M x k = 8, 64K rows) at R = 8: 84 MB against 42 MB per rank: sharded; a 100K-row
    table: 8.4 MB against 42 MB: replicated."""
    if R <= 1:
        return "sharded"
    kp = (k + 3) // 4 * 4
    dense = 2.0 * (R - 1) / R * F * (kp + 4) * 4
    owners = R * (1.0 - (1.0 - 1.0 / R) ** z)
    pairs = 2.0 * B * owners * (kp + 2) * 4 * (R - 1) / R
    return "replicated" if dense < pairs else "sharded"


def plan_run(args, env, n_visible):
    """How this invocation runs, from the arguments, the launcher's environment and the number of
    visible GPUs (torch.cuda.device_count(), which does not initialise the GPU):

      single : one GPU, one single-table fm_ctx (N = 1, the default)
      group  : ONE process drives N GPUs through one multi-GPU fm_ctx (fm_config.n_gpus = N,
               RCCL inside libfm_hip: what INTEGRATION.md's createMulti gives a Spark driver); also
               N = 1 with --force-sharded / --parallel (the group protocol on one rank)
      procs  : torch.distributed.run started one process per GPU (WORLD_SIZE = N); each holds a
               one-GPU group context of an N-rank job (fm_config.n_procs = N)

    parallel: "sharded" (rows owned by id % R) or "replicated" (every rank the whole table,
    gradient all-reduce); "auto" = auto_parallel's choice for the config at N ranks."""
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local_rank = int(env.get("LOCAL_RANK", "0"))
    n_ranks = max(world, args.gpus, args.copy_ranks, 1)
    F, k, B = CONFIGS[args.config][:3]
    par = args.parallel if args.parallel != "auto" else auto_parallel(F, k, B, NNZ_PER_ROW, n_ranks)
    if args.gpus < 1:
        raise PlanError("--gpus must be >= 1")
    if world > 1:
        if args.gpus != world:
            raise PlanError(f"--gpus {args.gpus} under a launcher with WORLD_SIZE={world}: they must agree")
        if n_visible < local_rank + 1:
            raise PlanError(f"LOCAL_RANK={local_rank} but only {n_visible} GPU(s) visible")
        return {"mode": "procs", "world": world, "rank": rank, "local_rank": local_rank, "n_local": 1,
                "parallel": par, "devices": [local_rank]}
    if args.gpus > 1:
        if n_visible < args.gpus:
            raise PlanError(f"--gpus {args.gpus} needs {args.gpus} visible GPUs in this process, {n_visible} visible; "
                            f"nothing was measured")
        if args.trainer != "lib":
            raise PlanError("--trainer torch needs torch.distributed.run (one process per GPU)")
        return {"mode": "group", "world": args.gpus, "rank": 0, "local_rank": 0, "n_local": args.gpus,
                "parallel": par, "devices": list(range(args.gpus))}
    if n_visible < 1:
        raise PlanError("no GPU visible")
    if args.copy_ranks > 1:
        # measurement only: an R-rank job on this one GPU (COPY transport: device copies between the
        # ranks' buffers), e.g. the one host thread's enqueue and prepare cost at R = 8
        return {"mode": "group", "world": args.copy_ranks, "rank": 0, "local_rank": 0, "n_local": args.copy_ranks,
                "parallel": par, "devices": [0] * args.copy_ranks}
    if args.force_sharded or args.parallel != "auto":
        return {"mode": "group", "world": 1, "rank": 0, "local_rank": 0, "n_local": 1, "parallel": par,
                "devices": [0]}
    return {"mode": "single", "world": 1, "rank": 0, "local_rank": 0, "n_local": 1, "parallel": None,
            "devices": [0]}


def batch_ids(b):
    """(U, singleton share) of a host batch: its distinct feature ids -- the rows a step updates, what
    the device reports as n_unique -- and the share of them with exactly one entry (the rows the fused
    step updates in its forward)."""
    _, c = np.unique(b.col, return_counts=True)
    return len(c), float(np.count_nonzero(c == 1)) / max(len(c), 1)


def concat_batches(parts):
    """Row-concatenation of CSR batches (the per-rank batches a one-process group context splits
    back by rows, contiguously)."""
    from fm_spark_amd.data import Batch

    if len(parts) == 1:
        return parts[0]
    offs = np.cumsum([0] + [p.nnz for p in parts])
    row_ptr = np.concatenate([parts[0].row_ptr[:1]] + [p.row_ptr[1:] + o for p, o in zip(parts, offs[:-1])])
    return Batch(row_ptr=row_ptr.astype(np.int64), col=np.concatenate([p.col for p in parts]),
                 val=np.concatenate([p.val for p in parts]), label=np.concatenate([p.label for p in parts]))


class ProfileSampler:
    """Per-phase HIP-event timing (fm_profile_*) on every n-th timed step only: each phase's start
    and stop events sit on its launch stream inside the timed region, and the kernels' average
    durations come from the sampled launches (batches cycle, so every batch is sampled)."""

    def __init__(self, ctx, args):
        self.ctx, self.on = ctx, False
        self.every = max(1, args.profile_every) if args.profile_kernels else 0

    def __call__(self, i):
        want = self.every > 0 and i % self.every == 0
        if want != self.on:
            self.ctx.profile_enable(want)
            self.on = want

    def off(self):
        if self.on:
            self.ctx.profile_enable(False)
            self.on = False


def main():
    args = parse()
    import torch

    pl = plan_run(args, os.environ, torch.cuda.device_count())
    world, rank, local_rank, mode = pl["world"], pl["rank"], pl["local_rank"], pl["mode"]
    torch.cuda.set_device(local_rank)
    dist = None
    if mode == "procs":
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if args.trainer == "torch":  # the test harness exchanges through torch's own RCCL
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
        else:
            # libfm_hip runs every exchange over its own RCCL communicators; torch only hands the RCCL id
            # around, and carries the barriers and the max-over-ranks time (gloo on the host)
            dist.init_process_group("gloo", rank=rank, world_size=world)

    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.engine import FMContext
    from fm_spark_amd._native import CSRHost

    cfg = CONFIGS[args.config]
    F, k, B, zipf_s, desc = cfg
    if args.features or args.k or args.rows or args.zipf:
        F, k, B, zipf_s = args.features or F, args.k or k, args.rows or B, args.zipf or zipf_s
        desc = f"override F={F} k={k} B={B} zipf={zipf_s} ({desc})"
        cfg = (F, k, B, zipf_s, desc)
    t0 = time.perf_counter()
    lab = {}
    if args.config == "c5":  # y = <w*, x> + N(0, 0.1) (BASELINE.md synthetic data)
        lab = dict(labels="regression", w_star=np.random.default_rng(20261015).normal(0.0, 0.1, F))
    # global rank g of this process's local rank l steps its own B-row batch (weak scaling); a
    # one-process group gets the local ranks' batches concatenated and splits them back by rows
    L = pl["n_local"]
    granks = [rank * L + l for l in range(L)]
    rank_batches = [[synthetic_batch(B, F, batch_index=g * 1000 + i, zipf_s=zipf_s, **lab) for i in range(args.batches)]
                    for g in granks]
    host_batches = [concat_batches([rb[i] for rb in rank_batches]) for i in range(args.batches)]
    log(f"[rank {rank}] generated {args.batches} batches of {L} x {B} rows in {time.perf_counter() - t0:.1f}s")
    z = host_batches[0].nnz / host_batches[0].n_rows

    median_ms = None
    fit = None
    fused = False
    host_path = None
    host_trace = None
    xg = None
    if mode == "single":
        ctx = FMContext(F, k, device=local_rank, seed=20261015, init_sd=INIT_SD,
                        fuse={"auto": None, "on": True, "off": False}[args.fuse])
        # launch on a torch stream of our own so torch events can bracket every step on it
        main_stream = torch.cuda.Stream()
        torch.cuda.set_stream(main_stream)
        ctx.set_stream(main_stream.cuda_stream)
        ctx.init_random_range(0, F)
        dbatches = [ctx.batch(CSRHost(b.row_ptr, b.col, b.val, b.label)) for b in host_batches]
        ctx.reserve(B, max(b.nnz for b in host_batches))
        nb = len(dbatches)
        # U and the singleton share of every batch, counted on the host (the device's n_unique)
        ids_stats = [batch_ids(b) for b in host_batches]
        t = 0
        prefetch = not args.no_prefetch and not args.host_path
        depth = max(1, min(args.prefetch_depth or 1, nb - 1))
        # the pipeline from the first warmup step on: the batches of the first `depth` steps are sorted
        # before it (as the steps before them would have, in a training loop), and every step -- warmup
        # and timed alike, one sequence g = 0, 1, ... -- sorts the batch `depth` steps ahead on the side
        # stream while it runs.  So every launch of a kernel in a profile of this command is the same
        # variant in the same overlap, and the timed region holds K steps and K sorts in the steady
        # state (the last `depth` sorts for batches stepped after it).
        if prefetch:
            for j in range(depth):
                dbatches[j % nb].prepare()
        for g in range(args.warmup):
            t += 1
            if prefetch:
                dbatches[(g + depth) % nb].prepare()
            ctx.step_batch(dbatches[g % nb], t, STEP_SIZE, REG_PARAM, sync=False)
        ctx.sync()
        torch.cuda.synchronize()
        if args.profile_kernels:
            ctx.profile_reset()
        prof_on = ProfileSampler(ctx, args)
        g0 = args.warmup
        if args.host_path:
            hosts = [CSRHost(b.row_ptr, b.col, b.val, b.label) for b in host_batches]
            t_start = time.perf_counter()
            for i in range(args.steps):
                t += 1
                ctx.step(hosts[(g0 + i) % len(hosts)], t, STEP_SIZE, REG_PARAM, sync=False)
        else:
            t_start = time.perf_counter()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        for i in range(0 if args.host_path else args.steps):
            t += 1
            prof_on(i)
            evs[i].record(main_stream)
            g = g0 + i
            if prefetch:
                dbatches[(g + depth) % nb].prepare()  # sorted on the side stream during step g
            ctx.step_batch(dbatches[g % nb], t, STEP_SIZE, REG_PARAM, sync=False)
        evs[args.steps].record(main_stream)
        ctx.sync()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        if not args.host_path:
            median_ms = median_step_ms(evs)
        prof = ctx.profile_read() if args.profile_kernels else {}
        prof_on.off()
        losses = ctx.loss_history()
        assert np.all(np.isfinite(losses)), "non-finite loss"
        if args.host_path_steps > 0 and not args.host_path:
            hmed, hmean, t = host_path_leg(ctx, host_batches, t, args.host_path_steps, torch)
            host_path = {"median_ms_per_step": hmed, "mean_ms_per_step": hmean, "steps": args.host_path_steps,
                         "samples_per_s": B / (hmed * 1e-3) if hmed else None,
                         "what": "fm_step with the host CSR each call: 8 B/entry + row_ptr + fp64 labels over PCIe, "
                                 "device-side explode, then the step (two upload slots, copies overlap the previous step)"}
        fit = None
        if args.fit_iters > 0 and not args.host_path:
            fit = fit_leg(ctx, F, B, zipf_s, lab, args.fit_iters)
        timed_b = [(g0 + i) % nb for i in range(args.steps)]
        U_mean = float(np.mean([ids_stats[j][0] for j in timed_b]))
        # the step variant from the context itself (fm_fuse_active), not from which phases were profiled
        fused = ctx.fuse_active and prefetch
        # the singleton rows' share of the rows updated, weighted by each timed batch's U
        single_frac = float(np.sum([ids_stats[j][0] * ids_stats[j][1] for j in timed_b])) / max(U_mean * len(timed_b), 1.0)
        parallelism = "single table" + (", fused step (singleton rows updated by the forward)" if fused else "") + \
            ((", next batch sorted during the current step" if depth == 1 else
              f", batches sorted {depth} steps ahead on the side stream") if prefetch else "")
        if args.host_path:
            parallelism += ", host CSR uploaded by fm_step every step (PCIe-inclusive)"
    elif args.trainer == "lib":
        from fm_spark_amd.engine import comm_unique_id

        par = pl["parallel"]
        cid = None
        if mode == "procs":
            # rank 0's RCCL id reaches the others over the (gloo) torch group; then every exchange of
            # the step runs inside libfm_hip (fm_group.hip)
            idt = torch.zeros(128, dtype=torch.uint8)
            if rank == 0:
                idt.copy_(torch.tensor(list(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, src=0)
            cid = bytes(idt.tolist())
        ctx = FMContext(F, k, seed=20261015, init_sd=INIT_SD, parallel=par, n_gpus=L, devices=pl["devices"],
                        transport="copy" if args.copy_ranks > 1 else "rccl", n_procs=world if mode == "procs" else 1,
                        proc_rank=rank, comm_id=cid,
                        fuse={"auto": None, "on": True, "off": False}[args.fuse])
        main_stream = None
        if L == 1:  # launch on a torch stream so torch events time each step on it
            main_stream = torch.cuda.Stream()
            torch.cuda.set_stream(main_stream)
            ctx.set_stream(main_stream.cuda_stream)
        ctx.init_random_range(0, F)
        dbatches = [ctx.batch(CSRHost(b.row_ptr, b.col, b.val, b.label)) for b in host_batches]
        prefetch = not args.no_prefetch
        nb = len(dbatches)
        t = 0
        uniques = []
        for i in range(max(args.warmup, nb)):  # every batch once: its distinct ids (U) for the roofline
            t += 1
            uniques.append(ctx.step_batch(dbatches[i % nb], t, STEP_SIZE, REG_PARAM, sync=True).n_unique)
        ctx.sync()
        for d in pl["devices"]:
            torch.cuda.synchronize(d)
        if dist is not None:
            dist.barrier()
        if args.profile_kernels:
            ctx.profile_reset()
        prof_on = ProfileSampler(ctx, args)
        # sharded, fm_batch_prepare is two-phase: it enqueues the batch's route and count gather, and
        # reads the counts of the batch prepared before it (exchange + owner slot sort on the side
        # streams); depth 2 gives each route a whole step to finish before the host reads its counts.
        # The pipeline in its steady state: the first `depth` timed steps' batches were prepared
        # before the timed region, and every timed step prepares the batch `depth` steps ahead (K
        # steps and K prepares inside the timed region)
        depth = max(1, min(args.prefetch_depth or 2, nb - 1))
        if prefetch:
            for j in range(depth):
                dbatches[j % nb].prepare()
            ctx.sync()
            for d in pl["devices"]:
                torch.cuda.synchronize(d)
            if dist is not None:
                dist.barrier()
        t_start = time.perf_counter()
        # batch i + depth's batch-only work (sharded: route, entry exchange and slot sort; replicated:
        # its sort) is enqueued on the side streams behind step i: inside the timed region, off the
        # critical path
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if main_stream else None
        h_step, h_prep = [], []  # host time in each call: the GPU never waits on the host if their sum < the step
        for i in range(args.steps):
            t += 1
            prof_on(i)
            if evs:
                evs[i].record(main_stream)
            h0 = time.perf_counter()
            ctx.step_batch(dbatches[i % nb], t, STEP_SIZE, REG_PARAM, sync=False)
            h1 = time.perf_counter()
            if prefetch:
                dbatches[(i + depth) % nb].prepare()
                h_prep.append(time.perf_counter() - h1)
            h_step.append(h1 - h0)
        if evs:
            evs[args.steps].record(main_stream)
        ctx.sync()
        for d in pl["devices"]:
            torch.cuda.synchronize(d)
        elapsed = time.perf_counter() - t_start
        median_ms = median_step_ms(evs) if evs else None
        prof = ctx.profile_read() if args.profile_kernels else {}
        prof_on.off()
        losses = ctx.loss_history()
        assert np.all(np.isfinite(losses)), "non-finite loss"
        R = world
        fused = False  # multi-GPU contexts never fuse (fm_fuse_active; selects the matching PMC file)
        # rows one rank updates: sharded, the global distinct ids over the owners; replicated, every
        # replica applies every touched row
        U_mean = float(np.mean(uniques)) / (R if par == "sharded" else 1)
        if par == "sharded":
            xg = exchange_bytes(rank_batches[0][0], R, granks[0], (k + 3) // 4 * 4)
        else:
            gbytes = F * ((k + 3) // 4 * 4 + 4) * 4
            xg = {"allreduce_B": gbytes, "ring_bytes_per_rank": 2 * gbytes * (R - 1) / R}
        who = (f"one process driving {L} GPUs through one fm_ctx" if mode == "group" else
               f"{world} processes (torch.distributed.run), one fm_ctx each")
        parallelism = (f"row-sharded x{R}, owner-computes, {who}, exchanges inside libfm_hip over RCCL (grouped "
                       f"send/recv of entries, partial sums and S rows)" if par == "sharded" else
                       f"replicated x{R}, {who}, per-slot gradient sums all-reduced inside libfm_hip over RCCL")
        if prefetch:
            parallelism += f", batches prepared {depth} step{'s' if depth > 1 else ''} ahead (route beside the steps)"
        host_trace = {"step_enqueue_ms_median": 1e3 * float(np.median(h_step)),
                      "prepare_ms_median": 1e3 * float(np.median(h_prep)) if h_prep else None,
                      "what": "host time inside fm_step_batch (out = NULL: enqueue only) and fm_batch_prepare of the "
                              "next batch, per iteration; below the step time the GPU never waits on the host"}
    else:
        from fm_spark_amd.distributed import ShardedTrainer

        tr = ShardedTrainer(F, k, rank=rank, world=world, device=local_rank, seed=20261015, init_sd=INIT_SD)
        tr.init_random_range(0, F)
        dbatches = [tr.batch(CSRHost(b.row_ptr, b.col, b.val, b.label)) for b in host_batches]
        t = 0
        uniques = []
        prefetch = not args.no_prefetch
        nb = len(dbatches)
        for i in range(args.warmup):
            t += 1
            nxt = dbatches[(i + 1) % nb] if prefetch and i + 1 < args.warmup else None
            o = tr.step(dbatches[i % nb], t, STEP_SIZE, REG_PARAM, prefetch=nxt)
            uniques.append(o.n_unique)
        torch.cuda.synchronize()
        dist.barrier()
        if args.profile_kernels:
            tr.ctx.profile_reset()
            tr.ctx.profile_enable(True)
        t_start = time.perf_counter()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        for i in range(args.steps):
            t += 1
            nxt = dbatches[(i + 1) % nb] if prefetch and i + 1 < args.steps else None
            evs[i].record(tr.engine.main_stream)
            tr.step(dbatches[i % nb], t, STEP_SIZE, REG_PARAM, sync=False, prefetch=nxt)
        evs[args.steps].record(tr.engine.main_stream)
        tr.ctx.sync()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        median_ms = median_step_ms(evs)
        prof = tr.ctx.profile_read() if args.profile_kernels else {}
        losses = tr.ctx.loss_history()
        assert np.all(np.isfinite(losses)), "non-finite loss"
        U_mean = float(np.mean(uniques)) / world if uniques else 0.0  # rows one owner updates
        xg = exchange_bytes(host_batches[0], world, rank, (k + 3) // 4 * 4)
        parallelism = (f"row-sharded x{world}, owner-computes, torch.distributed harness (RCCL all-to-all of entries, "
                       f"partial sums, S)" + (", next batch routed, exchanged and slot-sorted during the current step"
                                              if prefetch else ""))

    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        if args.trainer == "torch":
            tt = tt.cuda()
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        dist.barrier()

    if rank == 0:
        ms_per_step = 1000.0 * elapsed / args.steps
        value = world * B * args.steps / elapsed
        fwd_b, upd_b = algorithmic_bytes(F, k, B, z, U_mean)
        line = {
            "metric": "FM SGD train samples/sec at k=16, 1/8 GPUs; % of HBM roofline" if k == 16 else
                      f"FM SGD train samples/sec at k={k}",
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "median_ms_per_step": median_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Criteo-shaped, Zipf(%.2f) hashed ids, seed 20261015), random-init tables" % zipf_s,
            "config": {"workload": f"{args.config}: {desc}", "num_features": F, "k": k, "batch_rows_per_gpu": B,
                       "global_batch": B * world, "nnz_per_row": z, "rows_updated_per_gpu": U_mean,
                       "step_size": STEP_SIZE, "reg_param": REG_PARAM, "parallelism": parallelism,
                       "launch": mode},
            "loss_sum_all_steps": float(np.sum(losses)),
        }
        if args.trainer == "lib" and not args.host_path and not args.no_prefetch:
            line["timed_work"] = (f"{args.steps} steps and {args.steps} batch preparations (sorts / routes) inside the "
                                  f"timed region: the pipeline in its steady state, each step preparing the batch "
                                  f"{depth} steps ahead (the first {depth} timed steps' batches were prepared before it)")
        if prof:
            # "host_*": the one-thread multi-GPU driver's host time per phase (fm_group.hip HostClock)
            hostp = {name: ms / max(n, 1) for name, (ms, n) in prof.items() if name.startswith("host_")}
            if hostp:
                line.setdefault("host_trace", {})["phases_ms"] = hostp
            kern = {name: {"avg_ms": ms / max(n, 1), "launches": n} for name, (ms, n) in prof.items()
                    if not name.startswith("host_")}
            line["kernels"] = kern
            if args.trainer == "lib" and not args.host_path:
                line["kernels_sampled"] = f"HIP events on every {max(1, args.profile_every)}. timed step (launch streams)"
            if world > 1 or mode != "single":
                line["kernels_of"] = "local rank 0 (HIP events on its streams)"
            # single table: "forward" gathers, "update" does the row read-modify-write; sharded:
            # "owner_forward" / "owner_update" do the same on the rank's own rows (per rank: the
            # entries an owner receives ~ its own batch's, the rows it updates ~ U / world)
            algo = {"forward": fwd_b, "update": upd_b, "owner_forward": fwd_b, "owner_update": upd_b}
            algo_what = {"forward": "CSR (8z + 12 B per sample) + the gather of w and V (4z(k+1) B per sample)",
                         "update": "read + write of every touched row (8(k+1) B per row)"}
            if fused and mode == "single":
                # the fused forward also writes the singleton rows back (4(k+1) B each: their read is
                # the forward's own gather, already counted); the segmented update keeps the rows with
                # two or more entries (read + write)
                algo["forward"] = fwd_b + upd_b * single_frac / 2.0
                algo["update"] = upd_b * (1.0 - single_frac)
                algo_what["forward"] += " + the write-back of each singleton row (4(k+1) B; read by the gather)"
                algo_what["update"] = "read + write of the rows with two or more entries (8(k+1) B per row)"
            dom = max((n for n in kern if n in algo), key=lambda n: kern[n]["avg_ms"])
            ach = algo[dom] / (kern[dom]["avg_ms"] * 1e-3) / 1e9
            traffic, tsrc = pmc_traffic(F, k, B, dom, fused, world)
            line["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                                "algorithmic_bytes": algo[dom], "algorithmic_bytes_what": algo_what.get(dom),
                                "kernel_avg_ms": kern[dom]["avg_ms"],
                                "kernel_avg_of": "HIP events on the kernel's launch stream, every "
                                                 f"{max(1, args.profile_every)}. timed step (the warmup steps run the "
                                                 "same pipeline, so a rocprofv3 --kernel-trace --stats of this command "
                                                 "averages the same launches)",
                                "traffic_source": tsrc}
            # the ceiling that binds a random-row gather: L2 line requests per second
            reqs = {}
            for ph in ("forward", "update", "owner_forward", "owner_update"):
                if ph in kern:
                    rq, _ = pmc_requests(F, k, B, ph, fused, world)
                    rr = requests_roof(rq, kern[ph]["avg_ms"] * 1e-3)
                    if rr:
                        reqs[ph] = rr
            if reqs:
                line["roofline"]["requests"] = reqs.get(dom)
                line["roofline"]["requests_by_kernel"] = reqs
            if C3_SKELETON and dom == "forward" and fused and mode == "single" and (F, k, B, zipf_s) == CONFIGS["c3"][:4]:
                # the forward against its own access stream: tools/gather_ceiling.hip replays this batch
                # stream's memory skeleton (CSR read, every row's record gathered, the singleton rows'
                # records written back, the S records written; no arithmetic) alone on the GPU
                fw_ms = kern[dom]["avg_ms"]
                rq = (reqs.get("forward") or {}).get("l2_requests")
                sk_rate = C3_SKELETON["l2_requests_per_s"] / 1e9
                line["roofline"]["c3_stream"] = {
                    "skeleton_ms": C3_SKELETON["ms"], "skeleton_l2_requests": C3_SKELETON["l2_requests"],
                    "skeleton_G_per_s": sk_rate, "forward_ms_in_step": fw_ms,
                    "time_frac": C3_SKELETON["ms"] / fw_ms,
                    "requests_frac": (rq / (fw_ms * 1e-3) / 1e9) / sk_rate if rq else None,
                    "source": "profiles/gather_ceiling.json c3_stream (tools/c3_stream.py + tools/gather_ceiling.hip)"}
            if args.k == 0 and k == 16:
                # k = 16: a row's 68 algorithmic bytes sit in a 128-B record (one line per random access),
                # so at the ~6.3 TB/s random-line rate the forward's HBM fraction is capped near
                # 68/128 x 6.3/8 = 0.42 ("Ceilings of this design")
                line["roofline"]["layout_cap_frac"] = 68.0 / 128.0 * 6.3 / 8.0
            step_bytes = fwd_b + upd_b
            line["step_roofline"] = {"bytes_per_step": step_bytes,
                                     "achieved_GBs": step_bytes / (ms_per_step * 1e-3) / 1e9,
                                     "frac": step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS}
            if mode == "single":
                st_t, st_r, st_src = step_traffic(F, k, B, fused)
                if st_t:  # every kernel of the step, counted (PMC), against the step's time
                    line["step_roofline"].update(traffic=st_t, traffic_GBs=st_t / (ms_per_step * 1e-3) / 1e9,
                                                 traffic_frac=st_t / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                 traffic_source=st_src)
                if st_r:
                    line["step_roofline"]["requests"] = requests_roof(st_r, ms_per_step * 1e-3)
        if xg is not None:
            step_s = (median_ms or ms_per_step) * 1e-3
            if "entries_B" in xg:
                egress = xg["entries_B"] + xg["s_rows_B"] + xg["partials_B"]
                line["exchange"] = dict(xg, per="rank 0, per iteration, egress (ingress alike by symmetry)",
                                        egress_B=egress, egress_GBs_at_step_time=egress / step_s / 1e9,
                                        xgmi_peak_GBs=XGMI_LINK_GBS * max(world - 1, 0),
                                        xgmi_frac_at_step_time=(egress / step_s / 1e9 / (XGMI_LINK_GBS * (world - 1))
                                                                if world > 1 else None))
            else:
                # the replicated leg: the dense fp32 gradient buffer [F][kp + 4] all-reduced every iteration
                # (ring: 2 (R - 1) / R of it leaves each rank), against the step's own algorithmic bytes
                line["exchange"] = dict(xg, per="per iteration, the gradient all-reduce (fp32 sums across ranks)",
                                        ring_GBs_at_step_time=xg["ring_bytes_per_rank"] / step_s / 1e9,
                                        xgmi_peak_GBs=XGMI_LINK_GBS * max(world - 1, 0),
                                        xgmi_frac_at_step_time=(xg["ring_bytes_per_rank"] / step_s / 1e9 /
                                                                (XGMI_LINK_GBS * (world - 1)) if world > 1 else None),
                                        vs_step_algorithmic_bytes=xg["allreduce_B"] / max(fwd_b + upd_b, 1.0))
        if host_trace:
            line["host_trace"] = {**host_trace, **line.get("host_trace", {})}
        if host_path:
            line["host_path_ms_per_step"] = host_path["median_ms_per_step"]
            line["host_path"] = host_path
        if fit:
            line["fit_ms_per_iter"] = fit["fit_ms_per_iter"]
            fit["vs_step"] = fit["fit_ms_per_iter"] / ms_per_step
            if fit.get("fit_ms_per_iter_steady"):
                fit["steady_vs_step"] = fit["fit_ms_per_iter_steady"] / ms_per_step
            line["fit"] = fit
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline belongs to the N = 1 line
            try:
                line["cpu_baseline"] = cpu_baseline(cfg, host_batches[0], args.cpu_steps)
            except Exception as e:  # reported, never silently replaced
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
