"""GPU, config c5 shape (Zipf(1.2)-skewed hashed features, regression labels, CrossValidator
grid over k and regParam; FactorizationMachinesSample.scala:41-70): the product CrossValidator
driving the device estimator equals the same CrossValidator driving the CPU-oracle estimator
(tests/oracle_estimator.py): per-grid-point average metrics within the north_star's 1e-5, the
same best model, and its predictions."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _c5_frame(n_rows, F, parts):
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.linalg import SparseVector
    from fm_spark_amd.ml import DataFrame

    w_star = np.random.default_rng(17).normal(0.0, 0.5, F)
    b = synthetic_batch(n_rows, F, batch_index=n_rows, zipf_s=1.2, labels="regression", w_star=w_star)
    vecs = [SparseVector(F, b.col[b.row_ptr[i]:b.row_ptr[i + 1]], b.val[b.row_ptr[i]:b.row_ptr[i + 1]])
            for i in range(n_rows)]
    return DataFrame({"label": [float(y) for y in b.label], "features": vecs}, parts)


def test_cross_validator_c5_matches_oracle(gpu):
    from fm_spark_amd.ml import FactorizationMachinesSGD
    from fm_spark_amd.tuning import CrossValidator, ParamGridBuilder, RegressionEvaluator
    from oracle_estimator import OracleFMSGD

    df = _c5_frame(700, 3000, [400, 300])
    lo, hi = min(df["label"]), max(df["label"])
    common = dict(maxIter=4, miniBatchFraction=0.3, minLabel=lo, maxLabel=hi, initialSd=0.01, stepSize=0.2, seed=3)
    fm = FactorizationMachinesSGD()
    for name, v in common.items():
        fm._params[name] = v
    grid = ParamGridBuilder().addGrid(fm.dimFactorization, [4, 8]).addGrid(fm.regParam, [0.05, 0.0]).build()
    ev = RegressionEvaluator().setMetricName("mae")
    cv_gpu = CrossValidator().setEstimator(fm).setEstimatorParamMaps(grid).setEvaluator(ev).setNumFolds(2).fit(df)
    cv_ref = (CrossValidator().setEstimator(OracleFMSGD(**common)).setEstimatorParamMaps(grid).setEvaluator(ev)
              .setNumFolds(2).fit(df))
    np.testing.assert_allclose(cv_gpu.avgMetrics, cv_ref.avgMetrics, rtol=1e-5)
    assert int(np.argmin(cv_gpu.avgMetrics)) == int(np.argmin(cv_ref.avgMetrics))
    test = _c5_frame(120, 3000, [120])
    pg = np.asarray(cv_gpu.transform(test)["prediction"])
    pr = np.asarray(cv_ref.transform(test)["prediction"])
    np.testing.assert_allclose(pg, pr, rtol=1e-5, atol=1e-7)


@pytest.mark.timeout(600)
def test_cross_validator_c5_million_features(gpu):
    """The same comparison at BASELINE c5's feature space and grid: F = 1M hashed features with
    Zipf(1.2) hot rows (the rank-1 id of a field sits in ~16 % of the rows), regression labels,
    k in {8, 16} x regParam in {1e-6, 1e-4}, 24K rows in 2 folds -- the device path
    through the product CrossValidator against the CPU oracle estimator."""
    from fm_spark_amd.ml import FactorizationMachinesSGD
    from fm_spark_amd.tuning import CrossValidator, ParamGridBuilder, RegressionEvaluator
    from oracle_estimator import OracleFMSGD

    F = 1_000_000
    df = _c5_frame(24000, F, [12000, 12000])
    lo, hi = min(df["label"]), max(df["label"])
    common = dict(maxIter=3, miniBatchFraction=0.3, minLabel=lo, maxLabel=hi, initialSd=0.01, stepSize=0.1, seed=5)
    fm = FactorizationMachinesSGD()
    for name, v in common.items():
        fm._params[name] = v
    grid = ParamGridBuilder().addGrid(fm.dimFactorization, [8, 16]).addGrid(fm.regParam, [1e-6, 1e-4]).build()
    ev = RegressionEvaluator().setMetricName("mae")
    cv_gpu = CrossValidator().setEstimator(fm).setEstimatorParamMaps(grid).setEvaluator(ev).setNumFolds(2).fit(df)
    cv_ref = (CrossValidator().setEstimator(OracleFMSGD(**common)).setEstimatorParamMaps(grid).setEvaluator(ev)
              .setNumFolds(2).fit(df))
    np.testing.assert_allclose(cv_gpu.avgMetrics, cv_ref.avgMetrics, rtol=1e-5)
    assert int(np.argmin(cv_gpu.avgMetrics)) == int(np.argmin(cv_ref.avgMetrics))
    test = _c5_frame(2000, F, [2000])
    pg = np.asarray(cv_gpu.transform(test)["prediction"])
    pr = np.asarray(cv_ref.transform(test)["prediction"])
    np.testing.assert_allclose(pg, pr, rtol=1e-5, atol=1e-7)
