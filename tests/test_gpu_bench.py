"""GPU: bench.py's launch paths measure the same training.

The single-table step (fused and unfused), the one-process multi-GPU group context on one GPU
(--force-sharded: the row-sharded protocol with RCCL and one rank, what INTEGRATION.md's
createMulti gives a Spark driver) and its replicated layout must train the same model: the sum of
every executed step's loss agrees to 1e-6 (different but fixed summation orders).  Asking for more
GPUs than the box has must exit non-zero without a JSON line (no silent downgrade to one rank).
"""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--features", "200000", "--rows", "16384", "--steps", "6", "--warmup", "2", "--batches", "2",
         "--no-cpu-baseline", "--host-path-steps", "0"]


def _bench(*extra, check=True):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, *extra], capture_output=True,
                       text=True, timeout=100, env=env, cwd=ROOT)
    if not check:
        return p
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def single(gpu):
    return _bench("--fuse", "off")


def test_fused_single_table_trains_the_same_model(single):
    fused = _bench("--fuse", "on")
    assert "split" in fused["kernels"] and "split" not in single["kernels"]
    assert fused["loss_sum_all_steps"] == pytest.approx(single["loss_sum_all_steps"], rel=1e-6)


def test_group_path_on_one_gpu_matches_single_table(single):
    g = _bench("--force-sharded")
    assert g["config"]["launch"] == "group" and g["n_gpus"] == 1
    assert "owner_update" in g["kernels"]
    assert g["loss_sum_all_steps"] == pytest.approx(single["loss_sum_all_steps"], rel=1e-6)
    assert g["host_trace"]["step_enqueue_ms_median"] < g["ms_per_step"]


def test_replicated_group_on_one_gpu_matches_single_table(single):
    r = _bench("--parallel", "replicated")
    assert r["config"]["launch"] == "group" and "replicated" in r["config"]["parallelism"]
    assert r["loss_sum_all_steps"] == pytest.approx(single["loss_sum_all_steps"], rel=1e-6)


def test_more_gpus_than_visible_exits_nonzero(gpu):
    import torch

    n = torch.cuda.device_count()
    p = _bench("--gpus", str(n + 1), check=False)
    assert p.returncode != 0
    assert f"needs {n + 1} visible GPUs" in p.stderr and '"metric"' not in p.stdout
