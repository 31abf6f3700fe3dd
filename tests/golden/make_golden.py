"""Generates the committed golden fixtures from the CPU oracle (oracle/fm_ref.py,
oracle/spark_sampler.py).  Run from the repo root:  python tests/golden/make_golden.py

  c1_sample.npz     data/sample.txt (copied here as sample.txt, the reference's own fixture
                    file) as config c1: k = 4, maxIter = 3, stepSize = 0.01, regParam = 1e-6,
                    one partition; M0 injected (fp32-rounded N(0, 0.1^2), seed 11) because the
                    reference's initial draw is unseeded.
  c1_default_step.npz  the same with the reference's default stepSize = 1.0: the x*yhat - y
                    w-gradient on sample.txt's values (x up to 9.2) diverges
                    (loss ~1e25 at iteration 3) -- pins the oracle's faithfulness, CPU only.
  synth_small.npz   2000 synthetic Criteo-shaped rows (fm_spark_amd.data, F = 5000), k = 8,
                    maxIter = 5, two partitions, stepSize = 0.1, regParam = 1e-4, M0 as above.
Each stores the inputs, the randomSplit assignment, and the per-iteration loss and tables.
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from fm_spark_amd.data import read_libsvm, synthetic_batch  # noqa: E402
from oracle import fm_ref as R  # noqa: E402
from oracle import spark_sampler as S  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def f32(a):
    return np.asarray(a, dtype=np.float32).astype(np.float64)


def run(name, labels, vecs, part_sizes, k, max_iter, step, reg, F, m0_seed=11, sd=0.1):
    rows = [{"label": float(y), "features": v, "extra": 0} for y, v in zip(labels, vecs)]
    parts, off = [], 0
    for p in part_sizes:
        parts.append(rows[off:off + p])
        off += p
    splits, _ = S.random_split(parts, [0.1] * max_iter, 1234, "LF")
    starts = np.concatenate([[0], np.cumsum(part_sizes)])
    split_of = np.full(len(rows), -1, dtype=np.int32)
    split_rows = []
    for i, sp in enumerate(splits):
        idx = [int(starts[p] + r) for (p, r) in sp]
        for j in idx:
            split_of[j] = i
        split_rows.append(idx)
    csr_all = R.explode(labels, vecs)
    ids = np.unique(csr_all.col)
    rng = np.random.default_rng(m0_seed)
    w0 = f32(rng.normal(0, sd, len(ids)))
    V0 = f32(rng.normal(0, sd, (len(ids), k)))
    model = R.Model.empty(F, k)
    model.load(ids, w0, V0)
    losses = []
    for i in range(max_iter):
        sel = split_rows[i]
        csr = R.explode([labels[j] for j in sel], [vecs[j] for j in sel])
        res = R.sgd_step_fast(model, csr, i + 1, step, reg)
        losses.append(res.loss_sum if res.executed else np.nan)
        if i == 0:
            w1, V1 = model.w[ids].copy(), model.V[ids].copy()
    np.savez_compressed(os.path.join(HERE, name), ids=ids, w0=w0, V0=V0, split_of=split_of,
                        part_sizes=np.asarray(part_sizes), losses=np.asarray(losses), w1=w1, V1=V1,
                        w=model.w[ids], V=model.V[ids], k=k, max_iter=max_iter, step=step, reg=reg, F=F)
    print(name, "splits", [len(s) for s in split_rows], "losses", losses)


def main():
    labels, pairs, nf = read_libsvm(os.path.join(HERE, "sample.txt"))
    vecs = [R.sparse(nf, p) for p in pairs]
    run("c1_sample.npz", labels, vecs, [len(vecs)], k=4, max_iter=3, step=0.01, reg=1e-6, F=nf)
    run("c1_default_step.npz", labels, vecs, [len(vecs)], k=4, max_iter=3, step=1.0, reg=1e-6, F=nf)
    b = synthetic_batch(2000, 5000, batch_index=7)
    vecs = [R.sparse(5000, list(zip(b.col[b.row_ptr[i]:b.row_ptr[i + 1]].tolist(),
                                    b.val[b.row_ptr[i]:b.row_ptr[i + 1]].tolist()))) for i in range(b.n_rows)]
    run("synth_small.npz", b.label, vecs, [1000, 1000], k=8, max_iter=5, step=0.1, reg=1e-4, F=5000)


if __name__ == "__main__":
    main()
