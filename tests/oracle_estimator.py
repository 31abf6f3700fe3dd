"""TEST INFRASTRUCTURE: an Estimator/Model pair with the interface of fm_spark_amd.ml
(copy / fit / transform, _params) whose fit and transform run on the CPU oracle
(oracle/fm_ref.py step + predict, oracle/spark_sampler.py randomSplit replay, the seeded
createInitialModel draw of oracle/fm_ref.init_draw), so the product CrossValidator can drive
both and their metrics can be compared."""

import numpy as np

from fm_spark_amd.ml import Param
from oracle import fm_ref as R
from oracle import spark_sampler as S

DEFAULTS = {"dimFactorization": 10, "featuresCol": "features", "labelCol": "label", "predictionCol": "prediction",
            "maxIter": 10, "miniBatchFraction": 0.1, "regParam": 0.1, "stepSize": 1.0, "minLabel": 0.0,
            "maxLabel": 1.0, "initialSd": 0.01, "seed": 0}


def _oracle_vec(v):
    return R.sparse(v.size, list(zip(v.indices.tolist(), v.values.tolist())))


class OracleFMSGD:
    def __init__(self, **params):
        self.uid = "oracle_fm"
        self._params = dict(DEFAULTS)
        self._params.update(params)

    def copy(self, extra=None):
        c = OracleFMSGD(**self._params)
        for k, v in (extra or {}).items():
            c._params[k.name if isinstance(k, Param) else k] = v
        return c

    def fit(self, df):
        p = self._params
        k = p["dimFactorization"]
        labels = np.asarray(df[p["labelCol"]], dtype=np.float64)
        vecs = [_oracle_vec(v) for v in df[p["featuresCol"]]]
        csr_all = R.explode(labels, vecs)
        F = int(csr_all.col.max()) + 1
        ids = np.unique(csr_all.col)
        w0, V0 = R.init_draw(ids, k, p["seed"], p["initialSd"])
        model = R.Model.empty(F, k)
        model.load(ids, w0, V0)
        rows = [{"label": float(y), "features": v} for y, v in zip(labels, vecs)]
        parts, off = [], 0
        for n in df.partition_sizes:
            parts.append(rows[off:off + n])
            off += n
        starts = np.concatenate([[0], np.cumsum(df.partition_sizes)])
        splits, _ = S.random_split(parts, [p["miniBatchFraction"]] * p["maxIter"], 1234, "LF")
        for i, sp in enumerate(splits):
            idx = [int(starts[q] + r) for (q, r) in sp]
            if not idx:
                continue
            R.sgd_step_fast(model, R.explode([labels[j] for j in idx], [vecs[j] for j in idx]), i + 1,
                            p["stepSize"], p["regParam"])
        return OracleFMModel(model, p)


class OracleFMModel:
    def __init__(self, model, est_params):
        self.model = model
        self._params = {"featuresCol": est_params["featuresCol"], "predictionCol": est_params["predictionCol"],
                        "labelCol": est_params["labelCol"], "minLabel": est_params["minLabel"],
                        "maxLabel": est_params["maxLabel"]}

    def copy(self, extra=None):
        m = OracleFMModel(self.model, dict(self._params, featuresCol=self._params["featuresCol"],
                                           predictionCol=self._params["predictionCol"],
                                           labelCol=self._params["labelCol"], initialSd=0, seed=0,
                                           dimFactorization=0, maxIter=0, miniBatchFraction=0, regParam=0,
                                           stepSize=0))
        m._params.update(extra or {})
        return m

    def transform(self, df):
        p = self._params
        vecs = [_oracle_vec(v) for v in df[p["featuresCol"]]]
        csr = R.explode(np.zeros(len(vecs)), vecs)
        pred = R.predict(self.model, csr, p["minLabel"], p["maxLabel"], num_features=len(self.model.w))
        return df.with_column(p["predictionCol"], [float(x) for x in pred])
