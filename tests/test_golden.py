"""CPU: the committed golden fixtures (tests/golden/make_golden.py) -- the oracle and the C++
sampler replay reproduce them (guards the restatement against drift)."""

import os

import numpy as np
import pytest

from fm_spark_amd.data import read_libsvm
from oracle import fm_ref as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_inputs(name):
    g = np.load(os.path.join(GOLD, name))
    if name.startswith("c1"):
        labels, pairs, nf = read_libsvm(os.path.join(GOLD, "sample.txt"))
        vecs = [R.sparse(nf, p) for p in pairs]
    else:
        from fm_spark_amd.data import synthetic_batch

        b = synthetic_batch(2000, 5000, batch_index=7)
        labels = b.label
        vecs = [R.sparse(5000, list(zip(b.col[b.row_ptr[i]:b.row_ptr[i + 1]].tolist(),
                                        b.val[b.row_ptr[i]:b.row_ptr[i + 1]].tolist()))) for i in range(b.n_rows)]
    return g, labels, vecs


def test_sample_txt_reader_keeps_explicit_zeros():
    labels, rows, nf = read_libsvm(os.path.join(GOLD, "sample.txt"))
    assert labels.tolist() == [0, 1, 2, 3, 4, 5] and nf == 3
    assert rows[0] == [(0, 0.0), (1, 0.0), (2, 0.0)]  # stored zeros are active entries (P5)


@pytest.mark.parametrize("name", ["c1_sample.npz", "c1_default_step.npz", "synth_small.npz"])
def test_oracle_reproduces_golden(name):
    g, labels, vecs = load_inputs(name)
    k, F = int(g["k"]), int(g["F"])
    model = R.Model.empty(F, k)
    model.load(g["ids"], g["w0"], g["V0"])
    for i in range(int(g["max_iter"])):
        sel = np.nonzero(g["split_of"] == i)[0]
        csr = R.explode([labels[j] for j in sel], [vecs[j] for j in sel])
        res = R.sgd_step_fast(model, csr, i + 1, float(g["step"]), float(g["reg"]))
        if res.executed:
            assert res.loss_sum == pytest.approx(g["losses"][i], rel=1e-12)
    np.testing.assert_allclose(model.w[g["ids"]], g["w"], rtol=1e-12)
    np.testing.assert_allclose(model.V[g["ids"]], g["V"], rtol=1e-12)


@pytest.mark.parametrize("name", ["c1_sample.npz", "synth_small.npz"])
def test_sampler_reproduces_golden_splits(name):
    from fm_spark_amd import sampler as S
    from fm_spark_amd.linalg import SparseVector

    g, labels, vecs = load_inputs(name)
    lv = [SparseVector(v.size, v.indices, v.values) for v in vecs]
    split_of, _, _ = S.random_split(g["part_sizes"].tolist(), labels, lv, [0.1] * int(g["max_iter"]), 1234, "LF")
    assert split_of.tolist() == g["split_of"].tolist()
