"""CPU oracle — TEST INFRASTRUCTURE ONLY.

fp64 NumPy restatement of Rainbowboys/fm_spark's training hot path.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as
the checker.  The product path (fm_spark_amd) never imports it.

Parity status (see DESIGN.md "Oracle"):
  * forward / predict  — PINNED by the reference's own KAT
    (FactorizationMachinesSuite.scala:30-68: 23.77 / 5.275 / 5.2 / 5.0, unclamped, 1e-8);
  * VectorSum          — PINNED by the reference's own KAT
    (FactorizationMachinesSuite.scala:77-100: exactly (111.11, 222.22, 333.33));
  * gradient, update, L1, step loop — parity unpinned by the reference's tests: restated
    here from the Scala source line by line (no JVM / Spark in this image to run it).

Every function cites the reference file:line it follows.  All paths below are relative to
/root/reference/src/main/scala/org/apache/spark/ml/fm/.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


# ----------------------------------------------------------------------------- vectors
@dataclass
class SparkVector:
    """org.apache.spark.ml.linalg.{DenseVector, SparseVector} as plain data."""

    size: int
    values: np.ndarray
    indices: np.ndarray | None = None  # None => dense

    @property
    def is_dense(self) -> bool:
        return self.indices is None


def dense(*vals) -> SparkVector:
    v = np.asarray(vals[0] if len(vals) == 1 and not np.isscalar(vals[0]) else vals, dtype=np.float64)
    return SparkVector(size=len(v), values=v)


def sparse(size: int, pairs) -> SparkVector:
    pairs = sorted(pairs, key=lambda p: p[0])
    idx = np.asarray([p[0] for p in pairs], dtype=np.int32)
    val = np.asarray([p[1] for p in pairs], dtype=np.float64)
    return SparkVector(size=size, values=val, indices=idx)


def active_entries(vec: SparkVector) -> dict[int, float]:
    """udfVecToMap, FactorizationMachinesModel.scala:244-250.

    ``vec.foreachActive`` visits every index of a DenseVector (zeros included) and every
    stored entry of a SparseVector (explicit zeros included); ``m += (i -> value)`` keeps
    the last value per index.  The Map is then exploded (Model.scala:152)."""
    m: dict[int, float] = {}
    if vec.is_dense:
        for i, x in enumerate(vec.values):
            m[int(i)] = float(x)
    else:
        for i, x in zip(vec.indices, vec.values):
            m[int(i)] = float(x)
    return m


@dataclass
class CSR:
    """The exploded mini-batch (label, sampleId, featureId, featureValue), Model.scala:148-153."""

    row_ptr: np.ndarray  # int64 [B+1]
    col: np.ndarray  # int32 [N]
    val: np.ndarray  # float64 [N]
    label: np.ndarray  # float64 [B]

    @property
    def n_rows(self) -> int:
        return len(self.label)

    @property
    def nnz(self) -> int:
        return len(self.col)


def explode(labels, vectors) -> CSR:
    """Model.scala:148-153 with udfVecToMap (:244-250): one entry per active index."""
    row_ptr = [0]
    cols: list[int] = []
    vals: list[float] = []
    for v in vectors:
        m = active_entries(v)
        for i in sorted(m):
            cols.append(i)
            vals.append(m[i])
        row_ptr.append(len(cols))
    return CSR(
        row_ptr=np.asarray(row_ptr, dtype=np.int64),
        col=np.asarray(cols, dtype=np.int32),
        val=np.asarray(vals, dtype=np.float64),
        label=np.asarray(labels, dtype=np.float64),
    )


# ------------------------------------------------------------------------------ model
@dataclass
class Model:
    """Strength(id, strength) and FactorizedInteraction(id, vec) tables
    (Model.scala:281, :289) held densely over [0, F) with a present mask; globalBias w0
    (Model.scala:45)."""

    k: int
    w: np.ndarray  # float64 [F]
    V: np.ndarray  # float64 [F, k]
    present: np.ndarray  # bool [F]
    w0: float = 0.0

    @staticmethod
    def empty(num_features: int, k: int, w0: float = 0.0) -> "Model":
        return Model(k=k, w=np.zeros(num_features), V=np.zeros((num_features, k)),
                     present=np.zeros(num_features, dtype=bool), w0=w0)

    def load(self, ids, w, V) -> None:
        ids = np.asarray(ids, dtype=np.int64)
        self.w[ids] = np.asarray(w, dtype=np.float64)
        self.V[ids] = np.asarray(V, dtype=np.float64).reshape(len(ids), self.k)
        self.present[ids] = True

    def copy(self) -> "Model":
        return Model(k=self.k, w=self.w.copy(), V=self.V.copy(), present=self.present.copy(), w0=self.w0)


# ---------------------------------------------------------------------------- forward
@dataclass
class Forward:
    pred: np.ndarray  # [B] unclamped prediction (NaN for rows without entries)
    vfxi_sum: np.ndarray  # [B, k]
    has_entries: np.ndarray  # [B] bool
    loss_sum: float
    n_loss_rows: int


def forward(model: Model, csr: CSR) -> Forward:
    """calcLossGrad forward, Model.scala:173-221, per sample, in entry order:
        wixi   = strength * x                                  (:178)
        vfxi   = v * x (Breeze elementwise)                    (:179, :252-254)
        vi2xi2 = (sum_f v_f * v_f) * x * x                     (:180, :256-258)
        vfxiSum = VectorSum(vfxi) over the sample              (:191, FactorizationMachines.scala:56-67)
        wixiSum, vi2xi2Sum = sum over the sample               (:211-212)
        pred = 0.5 * (sum_f vfxiSum_f^2 - vi2xi2Sum) + wixiSum + w0   (:221, sumVx :260-262)
    Loss (yhat - y)^2 (:230), summed over samples that have entries (SGD.scala:134-138)."""
    B, k = csr.n_rows, model.k
    vfxi_sum = np.zeros((B, k))
    pred = np.full(B, np.nan)
    has = np.diff(csr.row_ptr) > 0
    loss_sum = 0.0
    for s in range(B):
        e0, e1 = csr.row_ptr[s], csr.row_ptr[s + 1]
        if e0 == e1:
            continue
        wsum = 0.0
        vv = 0.0
        acc = np.zeros(k)
        for e in range(e0, e1):
            i, x = int(csr.col[e]), float(csr.val[e])
            v = model.V[i]
            wsum += model.w[i] * x
            acc = acc + v * x
            vv += float(np.sum(v * v)) * x * x
        vfxi_sum[s] = acc
        yhat = 0.5 * (float(np.sum(acc * acc)) - vv) + wsum + model.w0
        pred[s] = yhat
        d = yhat - csr.label[s]
        loss_sum += d * d
    return Forward(pred=pred, vfxi_sum=vfxi_sum, has_entries=has, loss_sum=loss_sum,
                   n_loss_rows=int(has.sum()))


def loss_grad(model: Model, csr: CSR):
    """calcLossGrad output columns per exploded entry (Model.scala:225-233):
    prediction, loss, deltaWi = x (:200), deltaVi = vfxiSum * x - vfxi * x (:201-204)."""
    fw = forward(model, csr)
    N = csr.nnz
    pred = np.zeros(N)
    loss = np.zeros(N)
    dw = np.zeros(N)
    dv = np.zeros((N, model.k))
    for s in range(csr.n_rows):
        for e in range(csr.row_ptr[s], csr.row_ptr[s + 1]):
            i, x = int(csr.col[e]), float(csr.val[e])
            pred[e] = fw.pred[s]
            d = fw.pred[s] - csr.label[s]
            loss[e] = d * d
            dw[e] = x
            vfxi = model.V[i] * x
            dv[e] = fw.vfxi_sum[s] * x - vfxi * x
    return pred, loss, dw, dv


def predict(model: Model, csr: CSR, min_label: float, max_label: float, num_features=None) -> np.ndarray:
    """FactorizationMachinesModel.predict + transform, Model.scala:69-133.
    Entries whose id is not in the model are dropped by the inner joins (:103-112); a row
    left with no entry gets globalBias unclamped via na.fill (:78-86); otherwise the score
    (:127) is clamped to [minLabel, maxLabel] (:129-132)."""
    F = len(model.w) if num_features is None else num_features
    out = np.zeros(csr.n_rows)
    for s in range(csr.n_rows):
        acc = np.zeros(model.k)
        wsum = 0.0
        vv = 0.0
        n = 0
        for e in range(csr.row_ptr[s], csr.row_ptr[s + 1]):
            i, x = int(csr.col[e]), float(csr.val[e])
            if i < 0 or i >= F or not model.present[i]:
                continue
            v = model.V[i]
            wsum += model.w[i] * x
            acc = acc + v * x
            vv += float(np.sum(v * v)) * x * x
            n += 1
        if n == 0:
            out[s] = model.w0
        else:
            yhat = 0.5 * (float(np.sum(acc * acc)) - vv) + wsum + model.w0
            out[s] = min(max(yhat, min_label), max_label)
    return out


# ------------------------------------------------------------------------------- step
def soft_threshold(z, lam: float):
    """signum(z) * max(0, |z| - shrinkageVal), FactorizationMachinesSGD.scala:101-107, :179."""
    return np.sign(z) * np.maximum(0.0, np.abs(z) - lam)


@dataclass
class StepResult:
    executed: bool
    loss_sum: float = 0.0
    n_rows: int = 0
    n_loss_rows: int = 0
    n_unique: int = 0


def sgd_step(model: Model, csr: CSR, t: int, step_size: float, reg_param: float) -> StepResult:
    """One foldLeft iteration, FactorizationMachinesSGD.scala:116-211, in place on `model`.

        currentStepSize = stepSize / sqrt(iter)                 (:121)
        shrinkageVal    = currentStepSize * regParam            (:122)
        miniBatchSize   = count (empty rows included)           (:124)  [P4]
        miniBatchSize == 0 -> model unchanged                   (:126-128)
        per entry: g_w = deltaWi * pred - label = x*yhat - y    (:145)   [P1 precedence]
                   g_V = deltaVi * (pred - label)               (:146)
        per feature: deltaWiSum = (sum g_w / m) * eta           (:150)
                     deltaViSum = VectorSum(g_V) * (eta / m)    (:151-154)
        every present row: strength' = strength - deltaWiSum (0 if untouched)   (:171)
                           vec' = vec - deltaViSum                              (:172-175)
        L1 on every row: S_lambda(strength'), S_lambda(vec')     (:177-181)
    Rows touched by the batch but absent from the model would be created by the outer
    joins (:157-166); fit never produces them (createInitialModel covers every id)."""
    m = csr.n_rows
    if m == 0:
        return StepResult(executed=False)
    eta = step_size / math.sqrt(t)
    lam = eta * reg_param
    fw = forward(model, csr)
    gw: dict[int, float] = {}
    gv: dict[int, np.ndarray] = {}
    for s in range(m):
        e0, e1 = csr.row_ptr[s], csr.row_ptr[s + 1]
        if e0 == e1:
            continue
        yhat = fw.pred[s]
        y = csr.label[s]
        r = yhat - y
        for e in range(e0, e1):
            i, x = int(csr.col[e]), float(csr.val[e])
            vfxi = model.V[i] * x
            delta_vi = fw.vfxi_sum[s] * x - vfxi * x
            gw[i] = gw.get(i, 0.0) + (x * yhat - y)
            gv[i] = gv.get(i, np.zeros(model.k)) + delta_vi * r
    touched = np.asarray(sorted(gw), dtype=np.int64)
    scale_v = eta / m
    w_new = model.w.copy()
    V_new = model.V.copy()
    for i in touched:
        w_new[i] = model.w[i] - (gw[i] / m) * eta
        V_new[i] = model.V[i] - gv[i] * scale_v
    rows = model.present.copy()
    rows[touched] = True
    model.w[rows] = soft_threshold(w_new[rows], lam)
    model.V[rows] = soft_threshold(V_new[rows], lam)
    model.present = rows
    return StepResult(executed=True, loss_sum=fw.loss_sum, n_rows=m, n_loss_rows=fw.n_loss_rows,
                      n_unique=len(touched))


def sgd_step_fast(model: Model, csr: CSR, t: int, step_size: float, reg_param: float) -> StepResult:
    """Vectorised form of sgd_step (same arithmetic per entry, numpy reductions) for the
    medium-size fixtures; agrees with sgd_step to fp64 rounding."""
    m = csr.n_rows
    if m == 0:
        return StepResult(executed=False)
    eta = step_size / math.sqrt(t)
    lam = eta * reg_param
    k = model.k
    rows = np.repeat(np.arange(m), np.diff(csr.row_ptr))
    ids = csr.col.astype(np.int64)
    x = csr.val
    V = model.V[ids]
    vfxi = V * x[:, None]
    vfxi_sum = np.zeros((m, k))
    np.add.at(vfxi_sum, rows, vfxi)
    wsum = np.zeros(m)
    np.add.at(wsum, rows, model.w[ids] * x)
    vv = np.zeros(m)
    np.add.at(vv, rows, np.sum(V * V, axis=1) * x * x)
    yhat = 0.5 * (np.sum(vfxi_sum * vfxi_sum, axis=1) - vv) + wsum + model.w0
    has = np.diff(csr.row_ptr) > 0
    d = (yhat - csr.label)[has]
    loss_sum = float(np.sum(d * d))
    r = (yhat - csr.label)[rows]
    g_w = x * yhat[rows] - csr.label[rows]
    g_v = (vfxi_sum[rows] * x[:, None] - vfxi * x[:, None]) * r[:, None]
    F = len(model.w)
    GW = np.zeros(F)
    np.add.at(GW, ids, g_w)
    GV = np.zeros((F, k))
    np.add.at(GV, ids, g_v)
    touched = np.unique(ids)
    w_new = model.w.copy()
    V_new = model.V.copy()
    w_new[touched] = model.w[touched] - (GW[touched] / m) * eta
    V_new[touched] = model.V[touched] - GV[touched] * (eta / m)
    pres = model.present.copy()
    pres[touched] = True
    model.w[pres] = soft_threshold(w_new[pres], lam)
    model.V[pres] = soft_threshold(V_new[pres], lam)
    model.present = pres
    return StepResult(executed=True, loss_sum=loss_sum, n_rows=m, n_loss_rows=int(has.sum()),
                      n_unique=len(touched))


# -------------------------------------------------------------------------- VectorSum
def vector_sum(vectors) -> np.ndarray:
    """VectorSum UDAF, FactorizationMachines.scala:45-81: buffer starts at zeros (:54),
    update adds input(i) element-wise in arrival order (:56-67).  A single-partition
    groupBy sees the rows in input order, so this is a sequential fp64 sum."""
    vecs = list(vectors)
    k = vecs[0].size
    buf = [0.0] * k
    for v in vecs:
        arr = v.values if v.is_dense else _to_dense(v)
        for i in range(k):
            buf[i] += float(arr[i])
    return np.asarray(buf)


def _to_dense(v: SparkVector) -> np.ndarray:
    out = np.zeros(v.size)
    out[v.indices] = v.values
    return out


def vector_sum_by_key(keys, vecs: np.ndarray):
    """groupBy(key).agg(VectorSum(vec)) with rows in input order per key."""
    keys = np.asarray(keys)
    out_k = np.unique(keys)
    sums = np.zeros((len(out_k), vecs.shape[1]))
    pos = {int(kk): j for j, kk in enumerate(out_k)}
    for kk, v in zip(keys, vecs):
        j = pos[int(kk)]
        for f in range(vecs.shape[1]):
            sums[j, f] += v[f]
    return out_k, sums


# ------------------------------------------------------------------------------- fit
def fit(model: Model, batches, step_size: float, reg_param: float):
    """runMiniBatchSGD fold (SGD.scala:114-212) over pre-sampled batches (one per split,
    zipWithIndex -> iter = index + 1, :119)."""
    results = []
    for index, csr in enumerate(batches):
        results.append(sgd_step_fast(model, csr, index + 1, step_size, reg_param))
    return results


# ------------------------------------------------------------------- seeded init draw
def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def init_draw(ids, k: int, seed: int, sd: float):
    """createInitialModel's N(0, initialSd^2) draw (FactorizationMachinesSGD.scala:234-241)
    made deterministic: a counter-based Box-Muller keyed by (seed, id, factor), f = -1 for
    w.  Mirrors gauss_draw in fm_spark_amd/csrc/fm_kernels.hip; returns fp32-rounded values."""
    ids = np.asarray(ids, dtype=np.int64)
    with np.errstate(over="ignore"):
        f = np.arange(-1, k, dtype=np.int64)
        c = (ids[:, None].astype(np.uint64) << np.uint64(10)) ^ (f[None, :] + 1).astype(np.uint64)
        h1 = _splitmix64(np.uint64(seed) ^ _splitmix64(c))
        h2 = _splitmix64(h1 ^ np.uint64(0x632BE59BD9B4E019))
    u1 = ((h1 >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    u2 = (h2 >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    g = np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)
    vals = (g * sd).astype(np.float32).astype(np.float64)
    return vals[:, 0], vals[:, 1:]
