"""CPU: bench.py's run planning -- how --gpus N, the launcher's environment and the visible GPUs map
onto the single-table path, one process driving N GPUs through one multi-GPU fm_ctx, or one process
per GPU -- and that an impossible request exits non-zero instead of measuring fewer GPUs."""

import argparse

import numpy as np
import pytest

import bench


def _args(**kw):
    base = dict(gpus=1, config="c3", parallel="auto", force_sharded=False, trainer="lib", copy_ranks=0)
    base.update(kw)
    return argparse.Namespace(**base)


def test_default_is_the_single_table():
    pl = bench.plan_run(_args(), {}, 1)
    assert pl["mode"] == "single" and pl["world"] == 1 and pl["devices"] == [0]


def test_more_gpus_than_visible_fails_loudly():
    with pytest.raises(SystemExit) as ei:
        bench.plan_run(_args(gpus=2), {}, 1)
    assert "needs 2 visible GPUs" in str(ei.value) and ei.value.code != 0
    with pytest.raises(SystemExit):
        bench.plan_run(_args(gpus=8), {}, 4)


def test_one_process_drives_n_gpus():
    pl = bench.plan_run(_args(gpus=8), {}, 8)
    assert pl["mode"] == "group" and pl["world"] == 8 and pl["n_local"] == 8
    assert pl["devices"] == list(range(8)) and pl["parallel"] == "sharded"
    pl = bench.plan_run(_args(gpus=8, config="c2"), {}, 8)
    assert pl["parallel"] == "sharded"  # c2 at R = 8: the pairs move less than the dense all-reduce
    pl = bench.plan_run(_args(gpus=2, parallel="replicated", config="c2"), {}, 2)
    assert pl["parallel"] == "replicated"


def test_auto_layout_follows_the_exchange_projection():
    """per rank, the dense all-reduce (2 (R-1)/R F (kp+4) 4 B) against the pairs'
    partial sums and S rows (2 B R(1-(1-1/R)^z) (kp+2) 4 (R-1)/R B)."""
    assert bench.auto_parallel(1_000_000, 8, 65536, 39, 8) == "sharded"     # c2: 84 MB against 36 MB
    assert bench.auto_parallel(100_000, 8, 65536, 39, 8) == "replicated"    # 8.4 MB against 36 MB
    assert bench.auto_parallel(100_000_000, 16, 262144, 39, 8) == "sharded"  # c3
    assert bench.auto_parallel(1_000_000, 8, 65536, 39, 1) == "sharded"


def test_copy_ranks_run_on_one_gpu():
    pl = bench.plan_run(_args(copy_ranks=8), {}, 1)
    assert pl["mode"] == "group" and pl["world"] == 8 and pl["devices"] == [0] * 8


def test_launcher_one_process_per_gpu():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    pl = bench.plan_run(_args(gpus=4), env, 4)
    assert pl["mode"] == "procs" and pl["world"] == 4 and pl["rank"] == 2 and pl["devices"] == [2]
    assert pl["n_local"] == 1
    with pytest.raises(SystemExit):  # --gpus disagrees with the launcher
        bench.plan_run(_args(gpus=2), env, 4)
    with pytest.raises(SystemExit):  # the local rank's GPU is not visible
        bench.plan_run(_args(gpus=4), env, 2)


def test_group_path_on_one_gpu():
    pl = bench.plan_run(_args(force_sharded=True), {}, 1)
    assert pl["mode"] == "group" and pl["n_local"] == 1 and pl["parallel"] == "sharded"
    pl = bench.plan_run(_args(parallel="replicated"), {}, 1)
    assert pl["mode"] == "group" and pl["parallel"] == "replicated"


def test_torch_harness_needs_the_launcher():
    with pytest.raises(SystemExit):
        bench.plan_run(_args(gpus=2, trainer="torch"), {}, 2)


def test_no_gpu_fails_loudly():
    with pytest.raises(SystemExit):
        bench.plan_run(_args(), {}, 0)


def test_concat_batches_splits_back_by_rows():
    from fm_spark_amd.data import synthetic_batch

    parts = [synthetic_batch(100 + 7 * i, 5000, batch_index=i) for i in range(3)]
    cat = bench.concat_batches(parts)
    assert cat.n_rows == sum(p.n_rows for p in parts) and cat.nnz == sum(p.nnz for p in parts)
    r0 = 0
    for p in parts:  # the library's contiguous row split of the concatenation gives each part back
        e0, e1 = cat.row_ptr[r0], cat.row_ptr[r0 + p.n_rows]
        np.testing.assert_array_equal(cat.row_ptr[r0:r0 + p.n_rows + 1] - e0, p.row_ptr)
        np.testing.assert_array_equal(cat.col[e0:e1], p.col)
        np.testing.assert_array_equal(cat.val[e0:e1], p.val)
        np.testing.assert_array_equal(cat.label[r0:r0 + p.n_rows], p.label)
        r0 += p.n_rows


def test_batch_ids():
    from fm_spark_amd.data import Batch

    b = Batch(row_ptr=np.array([0, 3, 5]), col=np.array([1, 2, 3, 3, 4], np.int32), val=np.ones(5), label=np.zeros(2))
    U, single = bench.batch_ids(b)  # ids 1, 2, 3, 4; 3 of them with one entry
    assert U == 4 and single == pytest.approx(3 / 4)


def test_pmc_traffic_matches_workload_variant_and_mode():
    # the committed passes: c3 unfused and fused single-table steps, c2 and c5 (profiles/pmc_*.json)
    t_unf, src_unf = bench.pmc_traffic(100_000_000, 16, 262144, "update", fused=False)
    t_fus, src_fus = bench.pmc_traffic(100_000_000, 16, 262144, "forward", fused=True)
    assert t_unf and t_fus and src_unf != src_fus
    assert bench.pmc_traffic(1_000_000, 16, 65536, "update")[0]  # c5
    assert bench.pmc_traffic(1_000_000, 8, 65536, "update")[0]  # c2
    # a sharded owner phase or another world size never borrows the single-table counters
    assert bench.pmc_traffic(100_000_000, 16, 262144, "owner_update", fused=False, world=8)[0] is None
    assert bench.pmc_traffic(100_000_000, 16, 262144, "update", fused=False, world=2)[0] is None
    assert bench.pmc_traffic(123, 16, 262144, "update")[0] is None


def test_profile_sampler_toggles_every_nth_step():
    calls = []

    class Ctx:
        def profile_enable(self, on):
            calls.append(on)

    s = bench.ProfileSampler(Ctx(), argparse.Namespace(profile_kernels=1, profile_every=4))
    for i in range(9):
        s(i)
    s.off()
    assert calls == [True, False, True, False, True, False]
    calls.clear()
    s = bench.ProfileSampler(Ctx(), argparse.Namespace(profile_kernels=0, profile_every=4))
    for i in range(5):
        s(i)
    s.off()
    assert calls == []


def test_sort_passes_follow_the_digit_plan():
    # fm_sort.hip digit_bits: 27-bit slots 3 x 9, 20-bit 2 x 10, 24-bit 3 x 9 (8 is below the minimum
    # digit), 30-bit 3 x 10, 31-bit 4 x 9 (rounded up to the 9-bit minimum: 4 passes)
    assert bench.sort_passes(100_000_000) == 3
    assert bench.sort_passes(1_000_000) == 2
    assert bench.sort_passes(1 << 24) == 3
    assert bench.sort_passes(1 << 30) == 3
    assert bench.sort_passes(1 << 31) == 4


def test_step_traffic_covers_every_kernel_of_the_default_steps():
    """The committed PMC files (profiles/pmc_*.json) count every kernel bench.step_kernels says a c3
    (fused, LSD), c2 and c5 step launches, so the line's step_roofline carries traffic and
    requests; and the launch map follows the library's arrangement (the fused step's split at the
    step with its scatter, no separate tag pass)."""
    import bench

    ps = bench.step_kernels(100_000_000, True)
    assert ps["k_radix_scatter"] == 3 and ps["k_split_scatter"] == 1 and "k_tag_runs" not in ps
    assert bench.step_kernels(1_000_000, False)["k_radix_count"] == 2
    for cfg, fused in (("c3", True), ("c2", False), ("c5", False)):
        F, k, B, _, _ = bench.CONFIGS[cfg]
        t, r, src = bench.step_traffic(F, k, B, fused)
        assert t and r and src, cfg
        assert 1e8 < t < 1e10 and 1e6 < r < 1e8
