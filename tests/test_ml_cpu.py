"""CPU: Params, defaults, copy and schema checks of the mirror API (no device needed)."""

import pytest

from fm_spark_amd.linalg import Vectors
from fm_spark_amd.ml import DataFrame, FactorizationMachinesModel, FactorizationMachinesSGD, _check_schema


def test_defaults_match_reference():
    # FactorizationMachinesSGD.scala:61-74
    fm = FactorizationMachinesSGD()
    assert fm.getDimFactorization() == 10 and fm.getMaxIter() == 10
    assert fm.getMiniBatchFraction() == 0.1 and fm.getRegParam() == 0.1 and fm.getStepSize() == 1.0
    assert fm.getMinLabel() == 0.0 and fm.getMaxLabel() == 1.0 and fm.getInitialSd() == 0.01
    assert fm.uid.startswith("fm_")


def test_setters_chain_and_copy_keeps_uid():
    fm = FactorizationMachinesSGD("fm_x").setMaxIter(5).setMiniBatchFraction(0.2).setRegParam(1e-6)
    c = fm.copy({"regParam": 0.0})
    assert c.uid == "fm_x" and c.getRegParam() == 0.0 and fm.getRegParam() == 1e-6
    assert c.getMaxIter() == 5 and c.getMiniBatchFraction() == 0.2
    with pytest.raises(ValueError):
        fm.setDimFactorization(0)


def test_schema_validation():
    df = DataFrame({"label": [1.0], "features": [Vectors.dense(1.0)]})
    _check_schema(df, "features", "label")
    with pytest.raises(ValueError):
        _check_schema(DataFrame({"label": [1], "features": [Vectors.dense(1.0)]}), "features", "label")
    with pytest.raises(ValueError):
        _check_schema(DataFrame({"label": [1.0], "features": [[1.0]]}), "features", "label")


def test_from_rows_partitions_and_sample_ids():
    df = DataFrame.from_rows([(i, Vectors.dense(float(i))) for i in range(10)], ["rowId", "features"], 4)
    assert df.partition_sizes == [2, 3, 2, 3]  # ParallelCollectionRDD slicing
    sid = FactorizationMachinesModel.addSampleId(df)["sampleId"]
    assert sid[:3] == [0, 1, 1 << 33] and sid[-1] == (3 << 33) + 2


def test_fit_intercept_param_survives_copy_and_param_maps():
    """HasFitIntercept (FactorizationMachines.scala:18): Spark's default true, settable through a
    ParamMap / copy(extra) by name or by the Param handle, as CrossValidator does; a BooleanParam."""
    fm = FactorizationMachinesSGD("fm_y")
    assert fm.getFitIntercept() is True
    assert fm.fitIntercept.name == "fitIntercept" and fm.fitIntercept.parent == "fm_y"
    c = fm.copy({fm.fitIntercept: False})
    assert c.getFitIntercept() is False and fm.getFitIntercept() is True
    assert fm.copy({"fitIntercept": False}).getFitIntercept() is False
    with pytest.raises(TypeError):
        fm.copy({"fitIntercept": 1.5})


def test_select_csr_gathers_rows_in_order():
    """The synchronous fit's per-split host CSR (_select_csr): rows in the given order, repeats and
    empty rows kept, entries and labels carried along."""
    import numpy as np

    from fm_spark_amd.ml import _select_csr

    rp = np.array([0, 2, 2, 5, 6], dtype=np.int64)
    col = np.array([1, 4, 0, 2, 3, 7], dtype=np.int32)
    val = np.arange(6, dtype=np.float64) + 0.5
    lab = np.array([0.0, 1.0, 0.0, 1.0])
    c = _select_csr(rp, col, val, lab, [3, 1, 2, 0, 2])
    assert c.row_ptr.tolist() == [0, 1, 1, 4, 6, 9]
    assert c.col.tolist() == [7, 0, 2, 3, 1, 4, 0, 2, 3]
    assert c.val.tolist() == [5.5, 2.5, 3.5, 4.5, 0.5, 1.5, 2.5, 3.5, 4.5]
    assert c.label.tolist() == [1.0, 1.0, 0.0, 0.0, 0.0]
    e = _select_csr(rp, col, val, lab, [])
    assert e.row_ptr.tolist() == [0] and e.n_rows == 0 and e.nnz == 0


def test_resident_loop_orders_gather_prepare_step_per_buffer(caplog):
    """run_minibatch_sgd_resident's host schedule on a recording context: every split is gathered,
    then prepared, then stepped, in iteration order; a batch is regathered only after the step
    that read it was enqueued; empty splits are skipped with the reference's warning
    (FactorizationMachinesSGD.scala:126-128) and the losses come back in iteration order."""
    import logging

    from fm_spark_amd.ml import run_minibatch_sgd_resident

    events = []

    class Batch:
        def __init__(self, n):
            self.id, self.open = n, True

        def prepare(self):
            events.append(("prepare", self.id, self.rows))

        def close(self):
            self.open = False

    class Ctx:
        epoch = 7
        made = []

        def batch_from_rows(self, data, rows, into=None):
            b = into if into is not None else Batch(len(self.made))
            if into is None:
                self.made.append(b)
            b.rows = tuple(rows)
            events.append(("gather", b.id, b.rows))
            return b

        def step_batch(self, b, it, step, reg, sync=True):
            assert sync is False
            events.append(("step", b.id, b.rows, it))

        def sync(self):
            events.append(("sync",))

        def loss_history(self):
            return [None] * 7 + [10.0 * (j + 1) for j in range(64)]

    splits = [[0, 1], [], [2], [3, 4, 5], [6], [], [7, 8], [9]]
    ctx = Ctx()
    with caplog.at_level(logging.WARNING):
        out = run_minibatch_sgd_resident(ctx, None, splits, 1.0, 0.0)
    work = [(i, tuple(r)) for i, r in enumerate(splits) if r]
    assert out == [10.0 * (j + 1) for j in range(len(work))]
    assert len(ctx.made) == 3 and not any(b.open for b in ctx.made)
    assert sum("size of sampled batch is zero" in r.getMessage() for r in caplog.records) == 2
    steps = [e for e in events if e[0] == "step"]
    assert [(e[2], e[3]) for e in steps] == [(r, i + 1) for i, r in work]
    assert events[-1] == ("sync",)
    for rows in (r for _, r in work):
        g = events.index(next(e for e in events if e[0] == "gather" and e[2] == rows))
        p = events.index(next(e for e in events if e[0] == "prepare" and e[2] == rows))
        s = events.index(next(e for e in events if e[0] == "step" and e[2] == rows))
        assert g < p < s
    # a batch's contents stay put from its gather until its step was enqueued
    live = {}
    for e in events:
        if e[0] == "gather":
            assert e[1] not in live, "batch regathered before its step"
            live[e[1]] = e[2]
        elif e[0] == "step":
            assert live.pop(e[1]) == e[2]


def test_split_loop_orders_view_prepare_step_per_buffer(caplog):
    """run_minibatch_sgd_splits' host schedule on a recording context: iteration i steps split i of
    the split-ordered dataset through a view, prepared before its step; a view is re-pointed only
    after the step that read it was enqueued; empty splits (and the trailing split of unsampled rows)
    are not stepped, the empty ones logged with the reference's warning; losses in iteration order."""
    import logging

    import numpy as np

    from fm_spark_amd.ml import run_minibatch_sgd_splits

    events = []

    class View:
        def __init__(self, n):
            self.id, self.open = n, True

        def prepare(self):
            events.append(("prepare", self.id, self.split))

        def close(self):
            self.open = False

    class Data:
        split_rows = np.array([0, 2, 2, 3, 6, 7, 7, 9, 10, 40])  # 8 iterations + 30 unsampled rows

    class Ctx:
        epoch = 3
        made = []

        def split_view(self, data, split, into=None):
            b = into if into is not None else View(len(self.made))
            if into is None:
                self.made.append(b)
            b.split = split
            events.append(("view", b.id, split))
            return b

        def step_batch(self, b, it, step, reg, sync=True):
            assert sync is False
            events.append(("step", b.id, b.split, it))

        def sync(self):
            events.append(("sync",))

        def loss_history(self):
            return [None] * 3 + [10.0 * (j + 1) for j in range(64)]

    ctx = Ctx()
    with caplog.at_level(logging.WARNING):
        out = run_minibatch_sgd_splits(ctx, Data(), 1.0, 0.0, n_iter=8)
    work = [0, 2, 3, 4, 6, 7]
    assert out == [10.0 * (j + 1) for j in range(len(work))]
    assert len(ctx.made) == 2 and not any(b.open for b in ctx.made)
    assert sum("size of sampled batch is zero" in r.getMessage() for r in caplog.records) == 2
    steps = [e for e in events if e[0] == "step"]
    assert [(e[2], e[3]) for e in steps] == [(i, i + 1) for i in work]
    assert events[-1] == ("sync",)
    for i in work:
        v = events.index(next(e for e in events if e[0] == "view" and e[2] == i))
        p = events.index(next(e for e in events if e[0] == "prepare" and e[2] == i))
        s = events.index(next(e for e in events if e[0] == "step" and e[2] == i))
        assert v < p < s
    live = {}
    for e in events:
        if e[0] == "view":
            assert e[1] not in live, "view re-pointed before its step"
            live[e[1]] = e[2]
        elif e[0] == "step":
            assert live.pop(e[1]) == e[2]
