"""Host-side mirror of the reference's spark.ml API over the C-ABI.

    FactorizationMachinesSGD   <- FactorizationMachinesSGD.scala:28-86, 254-256 (Estimator)
    FactorizationMachinesModel <- FactorizationMachinesModel.scala:43-133, 135-241 (Model)
    Strength, FactorizedInteraction <- FactorizationMachinesModel.scala:281, :289
    VectorSum                  <- FactorizationMachines.scala:45-81 (UDAF)

Same names, Params, defaults and error behaviour as the Scala classes.  The per-iteration
work of ``fit`` (the foldLeft body, SGD.scala:116-211) runs as one fm_step per mini-batch on
the GPU; the mini-batches come from the randomSplit replay (fm_random_split).  ``DataFrame``
is a minimal local stand-in for a Spark DataFrame: named columns plus a partitioning (the
partitioning matters: randomSplit sorts and samples per partition).

Scala-side integration (JNI) is described in INTEGRATION.md; this module is what the parity
tests drive.
"""

from __future__ import annotations

import logging
import math
import uuid
from dataclasses import dataclass
from typing import NamedTuple

import numpy as np

from . import _native as N
from .engine import FMContext
from .linalg import DenseVector, Vector, Vectors, active_map

log = logging.getLogger("org.apache.spark.ml.fm")


@dataclass(frozen=True)
class Param:
    """A named parameter of an estimator (org.apache.spark.ml.param.Param): ``fm.regParam``;
    param maps (ParamGridBuilder, ``copy(extra)``) are keyed by its name."""

    parent: str
    name: str


# ------------------------------------------------------------------------ DataFrame
class DataFrame:
    """Columns by name + partition sizes (rows laid out partition after partition)."""

    def __init__(self, columns: dict, partition_sizes=None):
        self.columns = {k: list(v) for k, v in columns.items()}
        n = len(next(iter(self.columns.values()))) if self.columns else 0
        for k, v in self.columns.items():
            if len(v) != n:
                raise ValueError(f"column {k} has {len(v)} rows, expected {n}")
        self.partition_sizes = list(partition_sizes) if partition_sizes is not None else [n]
        if sum(self.partition_sizes) != n:
            raise ValueError("partition sizes do not add up to the row count")

    @staticmethod
    def from_rows(rows, names, num_partitions: int = 1) -> "DataFrame":
        """Seq(rows).toDF(names) on local[num_partitions]: ParallelCollectionRDD slicing,
        slice i = [i*n/p, (i+1)*n/p)."""
        rows = list(rows)
        cols = {nm: [r[i] for r in rows] for i, nm in enumerate(names)}
        n = len(rows)
        sizes = [((i + 1) * n) // num_partitions - (i * n) // num_partitions for i in range(num_partitions)]
        return DataFrame(cols, sizes)

    @property
    def schema(self):
        return list(self.columns)

    def count(self) -> int:
        return sum(self.partition_sizes)

    def __len__(self):
        return self.count()

    def collect(self):
        names = self.schema
        return [dict(zip(names, vals)) for vals in zip(*[self.columns[n] for n in names])]

    def with_column(self, name, values) -> "DataFrame":
        cols = dict(self.columns)
        cols[name] = list(values)
        return DataFrame(cols, self.partition_sizes)

    def __getitem__(self, name):
        return self.columns[name]


# ------------------------------------------------------------------------ table rows
class Strength(NamedTuple):
    """Strength(id: Int, strength: Double), FactorizationMachinesModel.scala:281."""

    id: int
    strength: float


class FactorizedInteraction(NamedTuple):
    """FactorizedInteraction(id: Int, vec: DenseVector), FactorizationMachinesModel.scala:289."""

    id: int
    vec: DenseVector


def _explode(vectors):
    """explode(udfVecToMap(features)) (Model.scala:148-153, :244-250) -> CSR arrays."""
    row_ptr = np.zeros(len(vectors) + 1, dtype=np.int64)
    cols, vals = [], []
    for i, v in enumerate(vectors):
        m = active_map(v)
        for j in sorted(m):
            cols.append(j)
            vals.append(m[j])
        row_ptr[i + 1] = len(cols)
    return row_ptr, np.asarray(cols, dtype=np.int32), np.asarray(vals, dtype=np.float64)


def _check_schema(df: DataFrame, features_col: str, label_col: str | None):
    """validateAndTransformSchema (FactorizationMachines.scala:33-37): features must be
    vectors (VectorUDT), the label a double."""
    if features_col not in df.columns:
        raise ValueError(f"Column {features_col} does not exist.")
    for v in df.columns[features_col]:
        if not isinstance(v, Vector):
            raise ValueError(f"Column {features_col} must be of type VectorUDT")
    if label_col is not None:
        if label_col not in df.columns:
            raise ValueError(f"Column {label_col} does not exist.")
        for y in df.columns[label_col]:
            if not isinstance(y, (float, np.floating)):
                raise ValueError(f"Column {label_col} must be of type DoubleType")


# ------------------------------------------------------------------------- VectorSum
class VectorSum:
    """UDAF summing k-vectors per group (FactorizationMachines.scala:45-81), on the device:
    the stable radix sort groups the keys, each group is summed in fp64 in input order."""

    def __init__(self, vec_size: int, ctx: FMContext | None = None):
        self.vec_size = int(vec_size)
        self._ctx = ctx

    def __call__(self, keys, vectors):
        ctx = self._ctx or FMContext(1, 1)
        vecs = np.zeros((len(vectors), self.vec_size))
        for i, v in enumerate(vectors):
            if v is None:
                continue  # update: if (input.isNullAt(0)) return  (FactorizationMachines.scala:57)
            a = v.to_array()
            vecs[i, :] = a[: self.vec_size]
        k, s = ctx.vector_sum_by_key(np.asarray(keys, dtype=np.int32), vecs)
        return {int(kk): DenseVector(ss) for kk, ss in zip(k, s)}


# ----------------------------------------------------------------------------- Model
class FactorizationMachinesModel:
    """FactorizationMachinesModel.scala:43-241.  The Strength / FactorizedInteraction tables
    live on the device (fm_ctx); ``dimensionStrength`` / ``factorizedInteraction`` export them."""

    def __init__(self, uid: str, dimFactorization: int, globalBias: float, dimensionStrength=None,
                 factorizedInteraction=None, *, num_features: int | None = None, ctx: FMContext | None = None,
                 device: int = 0):
        self.uid = uid
        self.dimFactorization = int(dimFactorization)
        self.globalBias = float(globalBias)
        self._params = {"sampleIdCol": "sampleId", "featuresCol": "features", "predictionCol": "prediction",
                        "labelCol": "label", "minLabel": 0.0, "maxLabel": 1.0}  # Model.scala:54-61
        self.parent = None
        if ctx is not None:
            self._ctx = ctx
        else:
            ds = list(dimensionStrength or [])
            fi = list(factorizedInteraction or [])
            ids = sorted({s.id for s in ds} | {f.id for f in fi})
            F = num_features if num_features is not None else (max(ids) + 1 if ids else 1)
            self._ctx = FMContext(F, self.dimFactorization, device=device, w0=self.globalBias)
            if ids:
                w = {s.id: s.strength for s in ds}
                vec = {f.id: f.vec.to_array() for f in fi}
                ids_a = np.asarray(ids, dtype=np.int32)
                w_a = np.asarray([w.get(i, 0.0) for i in ids])
                V_a = np.asarray([vec.get(i, np.zeros(self.dimFactorization)) for i in ids])
                self._ctx.load_tables(ids_a, w_a, V_a)

    # params ----------------------------------------------------------------------------
    def setMinLabel(self, value: float):
        self._params["minLabel"] = float(value)
        return self

    def setMaxLabel(self, value: float):
        self._params["maxLabel"] = float(value)
        return self

    def getMinLabel(self) -> float:
        return self._params["minLabel"]

    def getMaxLabel(self) -> float:
        return self._params["maxLabel"]

    def copy(self, extra: dict | None = None) -> "FactorizationMachinesModel":
        """Model.scala:63-66: same tables, params copied then overridden by extra."""
        m = FactorizationMachinesModel(self.uid, self.dimFactorization, self.globalBias, ctx=self._ctx)
        m._params = dict(self._params)
        m._params.update(extra or {})
        m.parent = self.parent
        return m

    # tables ------------------------------------------------------------------------------
    @property
    def dimensionStrength(self):
        ids, w, _ = self._ctx.export_tables()
        return [Strength(int(i), float(x)) for i, x in zip(ids, w)]

    @property
    def factorizedInteraction(self):
        ids, _, V = self._ctx.export_tables()
        return [FactorizedInteraction(int(i), DenseVector(v)) for i, v in zip(ids, V)]

    # transform / predict ---------------------------------------------------------------
    def transformSchema(self, schema):
        return list(schema) + [self._params["predictionCol"]]

    def transform(self, dataset: DataFrame) -> DataFrame:
        """Model.scala:69-87 + predict :90-133: inner-join semantics for unknown ids, clamp to
        [minLabel, maxLabel], rows without a learned feature get globalBias (na.fill)."""
        fcol = self._params["featuresCol"]
        _check_schema(dataset, fcol, None)
        rp, col, val = _explode(dataset[fcol])
        csr = N.CSRHost(rp, col, val, np.zeros(dataset.count()))
        pred = self._ctx.predict(csr, self.getMinLabel(), self.getMaxLabel())
        return dataset.with_column(self._params["predictionCol"], [float(p) for p in pred])

    def calcLossGrad(self, dfSampleIndexed: DataFrame, initialSd: float, seed: int = 0) -> DataFrame:
        """Model.scala:135-234: one row per active entry with columns label, sampleId,
        featureId, prediction, loss, deltaWi, deltaVi (deltaVi before the (pred - label) factor).
        Ids the model lacks get per-entry N(0, initialSd^2) draws (:144-146, 170-171); the
        reference's draws are unseeded, here they are keyed by `seed` and the entry.  A model whose
        table is row-sharded over several GPUs (setParallel("sharded")) refuses it with FMError:
        the per-entry rows would need every owner's rows on one device (fm_loss_grad, include/fm_hip.h);
        a replicated or single-GPU model answers it."""
        if not initialSd > 0.0:
            raise ValueError("requirement failed: initSd (initial Standard Deviation) must be > 0.0")
        fcol, lcol = self._params["featuresCol"], self._params["labelCol"]
        _check_schema(dfSampleIndexed, fcol, lcol)
        rp, col, val = _explode(dfSampleIndexed[fcol])
        labels = np.asarray(dfSampleIndexed[lcol], dtype=np.float64)
        csr = N.CSRHost(rp, col, val, labels)
        pred, loss, dw, dv = self._ctx.loss_grad(csr, initial_sd=initialSd, seed=seed)
        rows = np.repeat(np.arange(len(labels)), np.diff(rp))
        sids = dfSampleIndexed["sampleId"] if "sampleId" in dfSampleIndexed.columns else list(range(len(labels)))
        return DataFrame({
            lcol: [float(labels[r]) for r in rows],
            "sampleId": [sids[r] for r in rows],
            "featureId": [int(c) for c in col],
            self._params["predictionCol"]: pred.tolist(),
            "loss": loss.tolist(),
            "deltaWi": dw.tolist(),
            "deltaVi": [DenseVector(v) for v in dv],
        })

    @staticmethod
    def addSampleId(dataset: DataFrame, columnName: str = "sampleId") -> DataFrame:
        """monotonically_increasing_id (Model.scala:268-272): (partition << 33) + row index."""
        ids = []
        for p, n in enumerate(dataset.partition_sizes):
            ids.extend((p << 33) + r for r in range(n))
        return dataset.with_column(columnName, ids)


# ------------------------------------------------------------------------- Estimator
class FactorizationMachinesSGD:
    """FactorizationMachinesSGD.scala:28-256 (Estimator[FactorizationMachinesModel])."""

    _DEFAULTS = {  # SGD.scala:61-74
        "dimFactorization": 10, "featuresCol": "features", "labelCol": "label", "predictionCol": "prediction",
        "sampleIdCol": "sampleId", "maxIter": 10, "miniBatchFraction": 0.1, "regParam": 0.1, "stepSize": 1.0,
        "minLabel": 0.0, "maxLabel": 1.0, "initialSd": 0.01,
        # HasFitIntercept, mixed into the estimator's params (FactorizationMachines.scala:18), Spark's
        # default true; the reference never reads it (w0 stays 0.0, SGD.scala:246), nor does fit here
        "fitIntercept": True,
        # not in the reference: the init draw is unseeded there; device / seed here
        "seed": 0, "device": 0, "numFeatures": None,
        # not in the reference: the table over several GPUs of this process (include/fm_hip.h
        # fm_config.parallel), in place of Spark's hash-partitioned model Datasets
        "parallel": None, "nGpus": 1, "devices": None, "transport": "auto",
    }

    def __init__(self, uid: str | None = None):
        self.uid = uid or "fm_" + uuid.uuid4().hex[:12]  # Identifiable.randomUID("fm")
        self._params = dict(self._DEFAULTS)

    # setters / getters (SGD.scala:35-59) ------------------------------------------------
    def _set(self, name, value):
        self._params[name] = value
        return self

    def setDimFactorization(self, v: int):
        if int(v) < 1:  # IntParam, ParamValidators.gtEq(1) (FactorizationMachines.scala:26)
            raise ValueError("dimFactorization must be >= 1")
        return self._set("dimFactorization", int(v))

    def setFeaturesCol(self, v): return self._set("featuresCol", v)
    def setLabelCol(self, v): return self._set("labelCol", v)
    def setPredictionCol(self, v): return self._set("predictionCol", v)
    def setMaxIter(self, v): return self._set("maxIter", int(v))
    def setMiniBatchFraction(self, v): return self._set("miniBatchFraction", float(v))
    def setRegParam(self, v): return self._set("regParam", float(v))
    def setStepSize(self, v): return self._set("stepSize", float(v))
    def setMinLabel(self, v): return self._set("minLabel", float(v))
    def setMaxLabel(self, v): return self._set("maxLabel", float(v))
    def setInitialSd(self, v): return self._set("initialSd", float(v))
    def setSeed(self, v): return self._set("seed", int(v))
    def setNumFeatures(self, v): return self._set("numFeatures", int(v))

    def setParallel(self, mode, n_gpus: int = 1, devices=None, transport: str = "auto"):
        """Train (and transform) on n_gpus GPUs of this process: mode "sharded" splits the table's
        rows by id % R (owner-computes), "replicated" keeps a copy per GPU (gradient all-reduce);
        the mini-batches split by rows across the GPUs.  transport "copy" shares one device."""
        self._set("parallel", mode)
        self._set("nGpus", int(n_gpus))
        self._set("devices", None if devices is None else [int(d) for d in devices])
        return self._set("transport", transport)

    def getDimFactorization(self): return self._params["dimFactorization"]
    def getMaxIter(self): return self._params["maxIter"]
    def getMiniBatchFraction(self): return self._params["miniBatchFraction"]
    def getRegParam(self): return self._params["regParam"]
    def getStepSize(self): return self._params["stepSize"]
    def getMinLabel(self): return self._params["minLabel"]
    def getMaxLabel(self): return self._params["maxLabel"]
    def getInitialSd(self): return self._params["initialSd"]
    def getFitIntercept(self): return self._params["fitIntercept"]

    def copy(self, extra: dict | None = None) -> "FactorizationMachinesSGD":
        """defaultCopy (SGD.scala:254): same uid, params overridden by extra (keyed by name or Param)."""
        c = FactorizationMachinesSGD(self.uid)
        c._params = dict(self._params)
        for key, value in (extra or {}).items():
            name = key.name if isinstance(key, Param) else key
            if name == "fitIntercept" and not isinstance(value, (bool, np.bool_)):
                raise TypeError("fitIntercept is a BooleanParam")  # Spark's BooleanParam rejects non-booleans
            c._params[name] = value
        return c

    def transformSchema(self, schema):
        return schema

    # fit (SGD.scala:76-216) --------------------------------------------------------------
    def fit(self, dataset: DataFrame, initial_tables=None, pipelined: bool | None = None) -> FactorizationMachinesModel:
        """createInitialModel (:218-252) + addSampleId + runMiniBatchSGD (:88-216).
        ``initial_tables`` = (ids, w, V) injects M0 (the reference's draw is unseeded, P9).
        ``pipelined`` (default: on): the dataset is kept on the device (every GPU of a multi-GPU estimator
        gathers its share of a split from its own copy)
        -- dfData.cache(), :93 --, each randomSplit split is gathered there from its row list
        (fm_batch_from_rows) and sorted on the side stream while the previous iteration steps, and
        the steps only enqueue; the loss log lines (:139) are written, in iteration order, when the
        loop has run.  False: every split crosses PCIe as a host CSR and its step returns its loss
        (the same model: the splits hold the same rows in the same order)."""
        p = self._params
        _check_schema(dataset, p["featuresCol"], p["labelCol"])
        k = p["dimFactorization"]
        vectors = dataset[p["featuresCol"]]
        labels = np.asarray(dataset[p["labelCol"]], dtype=np.float64)
        rp, col, val = _explode(vectors)
        F = p["numFeatures"] or (int(col.max()) + 1 if len(col) else 1)
        ctx = FMContext(F, k, device=p["device"], seed=p["seed"], init_sd=p["initialSd"], w0=0.0,
                        parallel=p["parallel"], n_gpus=p["nGpus"], devices=p["devices"], transport=p["transport"])
        if pipelined is None:
            pipelined = True
        # randomSplit(Array.fill(maxIter)(miniBatchFraction), 1234L) (:111-112)
        order_cols = []
        extra = None
        for name in dataset.schema:
            if name == p["labelCol"]:
                order_cols.append("L")
            elif name == p["featuresCol"]:
                order_cols.append("F")
            else:
                vals = dataset[name]
                if extra is not None or not all(isinstance(v, (int, np.integer)) for v in vals):
                    raise ValueError(f"randomSplit replay supports one extra integer column, not {name!r}")
                extra = np.asarray(vals, dtype=np.int64)
                order_cols.append("I")
        from .sampler import random_split

        split_of, _, order = random_split(dataset.partition_sizes, labels, vectors,
                                          [p["miniBatchFraction"]] * p["maxIter"], 1234, "".join(order_cols),
                                          extra=extra)
        # split i's rows in per-partition sorted order (the order Spark's sampled partitions keep)
        splits = [order[split_of[order] == i] for i in range(p["maxIter"])]
        data = None
        if pipelined and len(labels):
            # dfData.cache() (:93): the exploded dataset uploaded once, laid out split after split (the
            # rows no split samples last, for createInitialModel), so every iteration's mini-batch is a
            # contiguous range of it, stepped in place (fm_batch_split_view)
            rest = order[split_of[order] < 0]
            lay = np.concatenate(splits + [rest]).astype(np.int64)
            split_rows = np.concatenate([[0], np.cumsum([len(r) for r in splits] + [len(rest)])])
            data = ctx.batch_splits(_select_csr(rp, col, val, labels, lay), split_rows)
        elif initial_tables is None and len(labels):
            data = ctx.batch(N.CSRHost(rp, col, val, labels))
        if initial_tables is not None:
            ctx.load_tables(*initial_tables)
        elif len(col):
            # createInitialModel (:224-241): the draw for every distinct active feature id, on the
            # device over the whole dataset's entries
            ctx.init_from_batch(data)
        if pipelined:
            if data is not None:
                run_minibatch_sgd_splits(ctx, data, p["stepSize"], p["regParam"], n_iter=p["maxIter"])
            else:
                for i in range(p["maxIter"]):
                    log.warning("Iteration (%d/%d). The size of sampled batch is zero", i + 1, p["maxIter"])
        else:
            for i, rows in enumerate(splits):
                it = i + 1  # iter = index + 1 (:119)
                if len(rows) == 0:
                    log.warning("Iteration (%d/%d). The size of sampled batch is zero", it, p["maxIter"])
                    continue
                csr = _select_csr(rp, col, val, labels, rows)
                out = ctx.step(csr, it, p["stepSize"], p["regParam"])
                log.info("Loss of Iteration (%d/%d): %s", it, p["maxIter"], out.loss_sum)
        model = FactorizationMachinesModel(self.uid, k, 0.0, ctx=ctx)
        model.setMinLabel(p["minLabel"]).setMaxLabel(p["maxLabel"])
        model.parent = self
        return model


def _select_csr(rp, col, val, labels, rows) -> N.CSRHost:
    """The host CSR of the given rows (the synchronous fit's per-split batch)."""
    rows = np.asarray(rows, dtype=np.int64)
    lens = rp[rows + 1] - rp[rows]
    sub_rp = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=sub_rp[1:])
    idx = np.repeat(rp[rows] - sub_rp[:-1], lens) + np.arange(sub_rp[-1], dtype=np.int64)
    return N.CSRHost(sub_rp, col[idx], val[idx], labels[rows])


def run_minibatch_sgd_resident(ctx: FMContext, data, splits, step_size: float, reg_param: float,
                               max_iter: int | None = None, bufs: list | None = None):
    """The foldLeft of runMiniBatchSGD (FactorizationMachinesSGD.scala:114-211) over a dataset kept
    on the device (`data`, dfData.cache() at :93): split i's rows (`splits[i]`, the randomSplit row
    lists) are gathered there (fm_batch_from_rows, on the copy stream) two iterations ahead into one
    of three batches used in turn, and sorted on the side stream (fm_batch_prepare) while iteration
    i - 1 steps, so a sort never waits for its split's copy and gather; every step only enqueues
    (fm_step_batch with out = NULL).  An empty split is skipped with the reference's warning
    (:126-128).  The loss log lines (:134-139) are written in iteration order after the loop, from
    the device's loss history.  Returns the loss sums of the executed iterations.  `bufs`: a list of
    three batches (or Nones) to refill and leave open for the caller (another loop reuses their
    device buffers); by default they are made here and closed at the end."""
    n_iter = len(splits) if max_iter is None else max_iter
    work = [(i, rows) for i, rows in enumerate(splits) if len(rows)]
    own = bufs is None
    if own:
        bufs = [None, None, None]
    nb = len(bufs)

    def gather(j):
        bufs[j % nb] = ctx.batch_from_rows(data, work[j][1], into=bufs[j % nb])

    e0 = ctx.epoch
    if work:
        gather(0)
        bufs[0].prepare()
    if len(work) > 1:
        gather(1)
    for j, (i, _) in enumerate(work):
        ctx.step_batch(bufs[j % nb], i + 1, step_size, reg_param, sync=False)  # iter = index + 1 (:119)
        if j + 1 < len(work):
            bufs[(j + 1) % nb].prepare()  # sorted on the side stream while this step runs
        if j + 2 < len(work):
            gather(j + 2)  # copied and gathered on the copy stream behind step j - 1
    ctx.sync()
    out = _log_losses(ctx, e0, [i for i, _ in work], len(splits), n_iter)
    if own:
        for b in bufs:
            if b is not None:
                b.close()
    return out


def _log_losses(ctx, e0, iters, n_splits, n_iter):
    """The loss log lines of SGD.scala:134-139 (and the zero-size warning of :126-128) for splits
    0 .. n_splits - 1, in iteration order, from the device's loss history of the executed iterations
    `iters` (their steps start at epoch e0); returns their losses."""
    hist = ctx.loss_history()[e0:]
    done = {i: float(hist[j]) for j, i in enumerate(iters)}
    for i in range(n_splits):
        if i in done:
            log.info("Loss of Iteration (%d/%d): %s", i + 1, n_iter, done[i])
        else:
            log.warning("Iteration (%d/%d). The size of sampled batch is zero", i + 1, n_iter)
    return [done[i] for i in iters]


def run_minibatch_sgd_splits(ctx: FMContext, data, step_size: float, reg_param: float, n_iter: int | None = None,
                             bufs: list | None = None):
    """The foldLeft of runMiniBatchSGD (FactorizationMachinesSGD.scala:114-211) over a dataset kept on
    the device laid out split after split (`data`, FMContext.batch_splits: dfData.cache() at :93 with
    the randomSplit splits of :111-112 in iteration order): iteration i steps split i in place
    (fm_batch_split_view re-points one of two batches used in turn -- no copy, no gather), sorted on
    the side stream (fm_batch_prepare) while iteration i - 1 steps; every step only enqueues.  An
    empty split is skipped with the reference's warning (:126-128); the loss log lines (:134-139) are
    written in iteration order after the loop.  n_iter: the iterations are splits 0 .. n_iter - 1
    (default: every split; fit's dataset ends with a split of the rows no iteration samples and
    passes maxIter).  `bufs`: a list of two views (or Nones) to re-point and leave open for the
    caller.  Returns the loss sums of the executed iterations."""
    sizes = np.diff(np.asarray(data.split_rows))
    n_iter = len(sizes) if n_iter is None else int(n_iter)
    if n_iter > len(sizes):
        raise ValueError("n_iter exceeds the dataset's splits")
    work = [i for i in range(n_iter) if sizes[i] > 0]
    own = bufs is None
    if own:
        bufs = [None, None]
    nb = len(bufs)

    def view(j):
        bufs[j % nb] = ctx.split_view(data, work[j], into=bufs[j % nb])

    e0 = ctx.epoch
    if work:
        view(0)
        bufs[0].prepare()
    for j, i in enumerate(work):
        ctx.step_batch(bufs[j % nb], i + 1, step_size, reg_param, sync=False)  # iter = index + 1 (:119)
        if j + 1 < len(work):
            view(j + 1)  # re-points the batch step j - 1 read (its sort waits for that step)
            bufs[(j + 1) % nb].prepare()  # sorted on the side stream while this step runs
    ctx.sync()
    out = _log_losses(ctx, e0, work, n_iter, n_iter)
    if own:
        for b in bufs:
            if b is not None:
                b.close()
    return out


# fm.regParam, fm.dimFactorization, ...: the Param handles spark.ml tuning keys grids by
for _name in ("dimFactorization", "featuresCol", "labelCol", "predictionCol", "maxIter", "miniBatchFraction",
              "regParam", "stepSize", "minLabel", "maxLabel", "initialSd", "seed", "fitIntercept"):
    setattr(FactorizationMachinesSGD, _name, property(lambda self, _n=_name: Param(self.uid, _n)))
del _name
