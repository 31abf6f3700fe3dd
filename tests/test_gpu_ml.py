"""GPU: the reference's own test suite (FactorizationMachinesSuite.scala) re-expressed on the
mirror API, and fit() end-to-end (randomSplit replay + device steps) against the golden
fixtures."""

import math
import os

import numpy as np
import pytest

from fm_spark_amd.linalg import DenseVector, SparseVector, Vectors

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_factorization_machines_model_suite(gpu):
    """FactorizationMachinesSuite.scala:24-75."""
    from fm_spark_amd.ml import DataFrame, FactorizedInteraction, FactorizationMachinesModel, Strength

    num_feature_dimensions, dim_factorization, global_bias = 4, 3, 5.0
    inp = DataFrame.from_rows([
        (100, Vectors.dense(1.0, 2.0, 1.5, -1.0)),                                   # dense
        (101, Vectors.sparse(num_feature_dimensions, [(0, 0.5), (2, -1.5)])),        # sparse
        (102, Vectors.sparse(num_feature_dimensions + 1, [(0, 2.0), (4, 1.5)])),     # unlearned dim
        (103, Vectors.sparse(num_feature_dimensions, [])),                           # empty
    ], ["rowId", "features"], num_partitions=4)
    ds = [Strength(0, 0.1), Strength(1, 0.2), Strength(2, 0.3), Strength(3, 0.4)]
    fi = [FactorizedInteraction(0, Vectors.dense(1.0, 2.0, 3.0)), FactorizedInteraction(1, Vectors.dense(3.0, 2.0, 1.0)),
          FactorizedInteraction(2, Vectors.dense(-0.1, -0.1, -0.2)), FactorizedInteraction(3, Vectors.dense(-0.5, 0.3, 0.0))]
    sus = FactorizationMachinesModel("uid", dim_factorization, global_bias, ds, fi)
    # the suite's expectations are the pre-clamp scores: open the clamp
    actual = sorted(sus.copy({"minLabel": -math.inf, "maxLabel": math.inf}).transform(inp).collect(),
                    key=lambda r: r["rowId"])
    assert len(actual) == 4
    for row, want in zip(actual, [23.77, 5.275, 5.2, 5.0]):
        assert row["prediction"] == pytest.approx(want, rel=1e-6)  # fp32 tables (reference: 1e-8 in fp64)
    # with the model's default [0, 1] clamp (Model.scala:54-61)
    clamped = sorted(sus.transform(inp).collect(), key=lambda r: r["rowId"])
    assert [r["prediction"] for r in clamped] == pytest.approx([1.0, 1.0, 1.0, 5.0])
    # the tables round-trip through the device
    assert [s.strength for s in sus.dimensionStrength] == pytest.approx([0.1, 0.2, 0.3, 0.4])


def test_vector_sum_suite(gpu):
    """FactorizationMachinesSuite.scala:77-102: exact equality."""
    from fm_spark_amd.ml import VectorSum

    vecs = [Vectors.dense(0.01, 0.02, 0.03), Vectors.dense(0.1, 0.2, 0.3).toSparse(), Vectors.dense(1.0, 2.0, 3.0),
            Vectors.dense(10.0, 20.0, 30.0).toSparse(), Vectors.dense(100.0, 200.0, 300.0)]
    actual = VectorSum(3)([1] * 5, vecs)
    assert list(actual) == [1]
    assert actual[1] == Vectors.dense(111.11, 222.22, 333.33)


@pytest.mark.parametrize("name", ["c1_sample.npz", "synth_small.npz"])
def test_fit_matches_golden(gpu, name):
    from fm_spark_amd.data import read_libsvm, synthetic_batch
    from fm_spark_amd.ml import DataFrame, FactorizationMachinesSGD

    g = np.load(os.path.join(GOLD, name))
    if name.startswith("c1"):
        labels, pairs, nf = read_libsvm(os.path.join(GOLD, "sample.txt"))
        vecs = [Vectors.sparse(nf, p) for p in pairs]
    else:
        b = synthetic_batch(2000, 5000, batch_index=7)
        labels = b.label
        vecs = [SparseVector(5000, b.col[b.row_ptr[i]:b.row_ptr[i + 1]], b.val[b.row_ptr[i]:b.row_ptr[i + 1]])
                for i in range(b.n_rows)]
    df = DataFrame({"label": [float(y) for y in labels], "features": vecs}, g["part_sizes"].tolist())
    fm = (FactorizationMachinesSGD().setDimFactorization(int(g["k"])).setMaxIter(int(g["max_iter"]))
          .setStepSize(float(g["step"])).setRegParam(float(g["reg"])).setNumFeatures(int(g["F"])))
    model = fm.fit(df, initial_tables=(g["ids"], g["w0"], g["V0"]))
    ids, w, V = model._ctx.export_tables()
    np.testing.assert_array_equal(ids, g["ids"])
    np.testing.assert_allclose(w, g["w"], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(V, g["V"], rtol=1e-5, atol=1e-8)
    losses = model._ctx.loss_history()
    np.testing.assert_allclose(losses, g["losses"][~np.isnan(g["losses"])], rtol=1e-5)


def test_fit_default_init_is_seeded_and_deterministic(gpu):
    from fm_spark_amd.ml import DataFrame, FactorizationMachinesSGD

    rng = np.random.default_rng(0)
    rows = [(float(rng.integers(0, 2)), Vectors.sparse(50, [(int(i), 1.0) for i in rng.choice(50, 5, replace=False)]))
            for _ in range(300)]
    df = DataFrame.from_rows(rows, ["label", "features"], num_partitions=3)
    outs = []
    for _ in range(2):
        m = FactorizationMachinesSGD().setDimFactorization(4).setMaxIter(3).setRegParam(1e-6).setSeed(9).fit(df)
        outs.append(m._ctx.export_tables())
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_fit_and_transform_on_several_gpus(gpu, mode):
    """fit + transform with the table spread over 3 ranks of one context (one GPU, COPY
    transport): the same model and predictions as the single-table fit, through the same
    estimator API (randomSplit replay, createInitialModel on the device, clamp on transform)."""
    from fm_spark_amd.data import synthetic_batch
    from fm_spark_amd.ml import DataFrame, FactorizationMachinesSGD

    b = synthetic_batch(3000, 4000, batch_index=11)
    vecs = [SparseVector(4000, b.col[b.row_ptr[i]:b.row_ptr[i + 1]], b.val[b.row_ptr[i]:b.row_ptr[i + 1]])
            for i in range(b.n_rows)]
    df = DataFrame({"label": [float(y) for y in b.label], "features": vecs}, [1000, 1000, 1000])

    def est():
        return (FactorizationMachinesSGD().setDimFactorization(8).setMaxIter(4).setStepSize(0.5).setRegParam(1e-5)
                .setNumFeatures(4000).setSeed(9))

    single = est().fit(df)
    multi = est().setParallel(mode, n_gpus=3, devices=[0, 0, 0], transport="copy").fit(df)
    i1, w1, V1 = single._ctx.export_tables()
    i2, w2, V2 = multi._ctx.export_tables()
    np.testing.assert_array_equal(i2, i1)
    np.testing.assert_allclose(w2, w1, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(V2, V1, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(multi._ctx.loss_history(), single._ctx.loss_history(), rtol=1e-6)
    p1 = [r["prediction"] for r in single.transform(df).collect()]
    p2 = [r["prediction"] for r in multi.transform(df).collect()]
    np.testing.assert_allclose(p2, p1, rtol=1e-5, atol=1e-7)
