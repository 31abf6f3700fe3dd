"""CPU: the multi-GPU exchange bookkeeping that fm_group.hip runs on every rank
(fm_spark_amd/csrc/fm_plan.h: route-count transposition, packed all-to-all-v plans, the chunked
partial exchange), checked for R = 1..9 simulated ranks by tests/native/plan_check.cpp (built with
g++ under ASan/UBSan from the product header): every tagged element reaches the block the receiving
rank's own plan expects.  This is the part of the N > 1 protocol that needs no GPU; the data path
runs through COPY (R up to 8) and RCCL in tests/test_gpu_group.py."""

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_exchange_plans_agree_across_ranks(tmp_path):
    exe = tmp_path / "plan_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "fm_spark_amd", "csrc"), os.path.join(HERE, "native", "plan_check.cpp"),
                    "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "0 failure(s)" in r.stdout
