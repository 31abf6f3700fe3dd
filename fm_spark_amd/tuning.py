"""The spark.ml tuning pieces the reference's demo drives the estimator with
(FactorizationMachinesSample.scala:41-70): ``ParamGridBuilder``, ``CrossValidator`` /
``CrossValidatorModel`` and ``RegressionEvaluator``, restated from Spark 2.1.0 (spark-mllib_2.11,
pinned in build.sbt:7-12) so that ``CrossValidator`` runs over ``FactorizationMachinesSGD`` exactly
as it does in Spark: it only calls ``copy`` / ``fit`` / ``transform``, so each fold and grid point
trains on the device through the same C-ABI, with several models alive at once (independent
fm_ctx handles).

Fold assignment replays ``MLUtils.kFold(dataset.toDF.rdd, numFolds, seed)``:
``PartitionwiseSampledRDD`` seeds partition p with the p-th ``java.util.Random(seed).nextLong()``,
and ``BernoulliCellSampler(lb, ub)`` keeps a row when its ``XORShiftRandom.nextDouble()`` lies in
``[lb, ub)`` with ``lb = (fold - 1) / numFolds`` and ``ub = fold / numFolds`` computed in Float; the
training set is the complement.  The default seed is ``"org.apache.spark.ml.tuning.CrossValidator"
.hashCode`` (HasSeed).
"""

from __future__ import annotations

import itertools

import numpy as np

from .ml import DataFrame, Param
from .sampler import next_doubles

__all__ = ["Param", "ParamGridBuilder", "CrossValidator", "CrossValidatorModel", "RegressionEvaluator", "k_fold"]


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode (signed 32-bit, over UTF-16 code units)."""
    h = 0
    units = s.encode("utf-16-be")
    for i in range(0, len(units), 2):
        h = (31 * h + ((units[i] << 8) | units[i + 1])) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


class JavaRandom:
    """java.util.Random (48-bit LCG): the per-partition seeds of PartitionwiseSampledRDD."""

    _MULT, _ADD, _MASK = 0x5DEECE66D, 0xB, (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self._MULT) & self._MASK

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * self._MULT + self._ADD) & self._MASK
        r = self.seed >> (48 - bits)
        return r - (1 << bits) if r >= (1 << (bits - 1)) else r  # (int) cast of the top bits

    def next_long(self) -> int:
        v = (self._next(32) << 32) + self._next(32)
        v &= (1 << 64) - 1
        return v - (1 << 64) if v >= (1 << 63) else v


class ParamGridBuilder:
    """org.apache.spark.ml.tuning.ParamGridBuilder: the cartesian product of the added grids."""

    def __init__(self):
        self._grid = {}

    def addGrid(self, param, values):
        self._grid[param.name if isinstance(param, Param) else str(param)] = list(values)
        return self

    def baseOn(self, *pairs):
        for param, value in pairs:
            self.addGrid(param, [value])
        return self

    def build(self):
        names = list(self._grid)
        return [dict(zip(names, combo)) for combo in itertools.product(*(self._grid[n] for n in names))]


class RegressionEvaluator:
    """org.apache.spark.ml.evaluation.RegressionEvaluator (RegressionMetrics over
    (prediction, label)): rmse (default), mse, r2, mae."""

    def __init__(self):
        self._params = {"metricName": "rmse", "predictionCol": "prediction", "labelCol": "label"}

    def setMetricName(self, v):
        if v not in ("rmse", "mse", "r2", "mae"):
            raise ValueError(f"unsupported metric {v!r}")
        self._params["metricName"] = v
        return self

    def setPredictionCol(self, v):
        self._params["predictionCol"] = v
        return self

    def setLabelCol(self, v):
        self._params["labelCol"] = v
        return self

    def getMetricName(self):
        return self._params["metricName"]

    def isLargerBetter(self) -> bool:
        return self._params["metricName"] == "r2"

    def evaluate(self, dataset: DataFrame) -> float:
        p = np.asarray(dataset[self._params["predictionCol"]], dtype=np.float64)
        y = np.asarray(dataset[self._params["labelCol"]], dtype=np.float64)
        err = y - p
        m = self._params["metricName"]
        if m == "mae":
            return float(np.mean(np.abs(err)))
        mse = float(np.mean(err * err))
        if m == "mse":
            return mse
        if m == "rmse":
            return float(np.sqrt(mse))
        ss_tot = float(np.sum((y - y.mean()) ** 2))
        return 1.0 - float(np.sum(err * err)) / ss_tot  # r2


def k_fold(dataset: DataFrame, num_folds: int, seed: int):
    """MLUtils.kFold replay: [(training, validation)] per fold, partitions preserved."""
    if num_folds < 2:
        raise ValueError("numFolds must be >= 2")
    rnd = JavaRandom(seed)
    xs = [next_doubles(rnd.next_long(), n) for n in dataset.partition_sizes]  # sampler.setSeed(split.seed)
    folds = []
    nf = np.float32(num_folds)
    for fold in range(1, num_folds + 1):
        lb = float(np.float32(fold - 1) / nf)
        ub = float(np.float32(fold) / nf)
        val_idx, tr_idx, val_sizes, tr_sizes = [], [], [], []
        off = 0
        for x in xs:
            keep = (x >= lb) & (x < ub)
            rows = np.arange(off, off + len(x))
            val_idx.append(rows[keep])
            tr_idx.append(rows[~keep])
            val_sizes.append(int(keep.sum()))
            tr_sizes.append(int((~keep).sum()))
            off += len(x)
        folds.append((_take(dataset, np.concatenate(tr_idx), tr_sizes),
                      _take(dataset, np.concatenate(val_idx), val_sizes)))
    return folds


def _take(df: DataFrame, rows, sizes) -> DataFrame:
    return DataFrame({k: [v[int(r)] for r in rows] for k, v in df.columns.items()}, sizes)


class CrossValidatorModel:
    def __init__(self, uid, best_model, avg_metrics):
        self.uid = uid
        self.bestModel = best_model
        self.avgMetrics = list(avg_metrics)

    def transform(self, dataset: DataFrame) -> DataFrame:
        return self.bestModel.transform(dataset)


class CrossValidator:
    """org.apache.spark.ml.tuning.CrossValidator (Spark 2.1.0 fit): per fold, fit every param map
    on the training part, sum the evaluator's metric on the validation part, average over folds,
    refit the best param map (first best: maxBy / minBy) on the whole dataset."""

    def __init__(self, uid: str | None = None):
        self.uid = uid or "cv"
        self._params = {"numFolds": 3, "seed": java_string_hash("org.apache.spark.ml.tuning.CrossValidator")}
        self._est = self._epm = self._eval = None

    def setEstimator(self, est):
        self._est = est
        return self

    def setEstimatorParamMaps(self, epm):
        self._epm = list(epm)
        return self

    def setEvaluator(self, ev):
        self._eval = ev
        return self

    def setNumFolds(self, n: int):
        self._params["numFolds"] = int(n)
        return self

    def setSeed(self, s: int):
        self._params["seed"] = int(s)
        return self

    def getSeed(self) -> int:
        return self._params["seed"]

    def fit(self, dataset: DataFrame) -> CrossValidatorModel:
        est, epm, ev = self._est, self._epm, self._eval
        if est is None or epm is None or ev is None:
            raise ValueError("estimator, estimatorParamMaps and evaluator must be set")
        metrics = np.zeros(len(epm))
        for training, validation in k_fold(dataset, self._params["numFolds"], self._params["seed"]):
            for i, pm in enumerate(epm):
                model = est.copy(pm).fit(training)
                mparams = {k: v for k, v in pm.items() if k in model._params}  # copyValues: the model's own params
                metrics[i] += ev.evaluate(model.copy(mparams).transform(validation))
        metrics /= self._params["numFolds"]
        best = int(np.argmax(metrics)) if ev.isLargerBetter() else int(np.argmin(metrics))
        best_model = est.copy(epm[best]).fit(dataset)
        return CrossValidatorModel(self.uid, best_model, metrics)
