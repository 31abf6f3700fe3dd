"""CPU: the spark.ml tuning restatement (fm_spark_amd/tuning.py) -- java.util.Random and
String.hashCode known answers, the kFold replay's fold structure, ParamGridBuilder, and the
RegressionEvaluator metrics."""

import numpy as np
import pytest

from fm_spark_amd.linalg import Vectors
from fm_spark_amd.ml import DataFrame, FactorizationMachinesSGD, Param
from fm_spark_amd.tuning import (JavaRandom, ParamGridBuilder, RegressionEvaluator, java_string_hash, k_fold)


def test_java_known_answers():
    # java.lang.String.hashCode: "hello" -> 99162322, "" -> 0; Integer overflow wraps
    assert java_string_hash("hello") == 99162322
    assert java_string_hash("") == 0
    assert java_string_hash("polygenelubricants") == -2147483648
    # java.util.Random(42).nextInt() == -1170105035 (the first 32-bit draw of nextLong)
    r = JavaRandom(42)
    assert r._next(32) == -1170105035
    v = JavaRandom(0).next_long()
    assert -(1 << 63) <= v < (1 << 63)


def test_param_handles_and_grid():
    fm = FactorizationMachinesSGD()
    assert fm.regParam == Param(fm.uid, "regParam")
    grid = ParamGridBuilder().addGrid(fm.dimFactorization, [4, 8]).addGrid(fm.regParam, [1e-6, 0.0]).build()
    assert grid == [{"dimFactorization": 4, "regParam": 1e-6}, {"dimFactorization": 4, "regParam": 0.0},
                    {"dimFactorization": 8, "regParam": 1e-6}, {"dimFactorization": 8, "regParam": 0.0}]
    c = fm.copy({fm.regParam: 0.5, "maxIter": 3})
    assert c.getRegParam() == 0.5 and c.getMaxIter() == 3 and c.uid == fm.uid
    assert fm.getRegParam() == 0.1  # the original is unchanged (default, SGD.scala:61-74)


@pytest.mark.parametrize("folds,parts", [(2, [50]), (3, [40, 37, 23]), (5, [7, 0, 93])])
def test_k_fold_partitions_rows(folds, parts):
    n = sum(parts)
    df = DataFrame({"label": [float(i) for i in range(n)],
                    "features": [Vectors.sparse(3, [(0, 1.0)]) for _ in range(n)]}, parts)
    splits = k_fold(df, folds, seed=-1159716171)
    seen = []
    for tr, va in splits:
        assert tr.count() + va.count() == n
        assert sorted(tr["label"] + va["label"]) == [float(i) for i in range(n)]
        assert len(tr.partition_sizes) == len(parts) == len(va.partition_sizes)
        seen.extend(va["label"])
    assert sorted(seen) == [float(i) for i in range(n)]  # every row validates exactly once
    again = k_fold(df, folds, seed=-1159716171)
    assert [v["label"] for _, v in again] == [v["label"] for _, v in splits]


def test_regression_evaluator():
    df = DataFrame({"label": [1.0, 2.0, 4.0], "prediction": [1.5, 2.0, 3.0]})
    ev = RegressionEvaluator()
    assert ev.evaluate(df) == pytest.approx(np.sqrt((0.25 + 0 + 1) / 3))
    assert ev.setMetricName("mae").evaluate(df) == pytest.approx(0.5)
    assert not ev.isLargerBetter()
    assert ev.setMetricName("r2").isLargerBetter()
    assert ev.evaluate(df) == pytest.approx(1 - 1.25 / np.sum((np.array([1, 2, 4]) - 7 / 3) ** 2))
