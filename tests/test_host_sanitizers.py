"""CPU: the library's host-only C++ (libsvm reader, randomSplit replay, MurmurHash3 / XORShift)
built from the product sources with g++ -fsanitize=address,undefined and exercised by
tests/native/host_sanitize.cpp (malformed inputs, too-small buffers, the SMHasher value)."""

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_sanitize"
    srcs = [os.path.join(HERE, "native", "host_sanitize.cpp"),
            os.path.join(ROOT, "fm_spark_amd", "csrc", "fm_sampler.cpp"),
            os.path.join(ROOT, "fm_spark_amd", "csrc", "fm_libsvm.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-pthread", *srcs, "-o", str(exe)], check=True)
    # the process environment is passed through unchanged; ASan is told not to insist on being the
    # first library loaded
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_random_split_partitions_under_tsan(tmp_path):
    """fm_random_split runs its partitions on the host thread pool: the same program under
    -fsanitize=thread reports no data race (the partitions write disjoint rows)."""
    exe = tmp_path / "host_tsan"
    srcs = [os.path.join(HERE, "native", "host_sanitize.cpp"),
            os.path.join(ROOT, "fm_spark_amd", "csrc", "fm_sampler.cpp"),
            os.path.join(ROOT, "fm_spark_amd", "csrc", "fm_libsvm.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", *srcs, "-o", str(exe)],
                   check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout and "ThreadSanitizer" not in r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_host_pool_jobs_and_exceptions(tmp_path, san):
    """The library's host thread pool (fm_hostpool.h): every index of a job runs once; a job's
    exception reaches the caller after the job drained (no worker still holds it) and the pool serves
    the next job; no data race under -fsanitize=thread, no memory error under ASan/UBSan."""
    exe = tmp_path / "host_pool"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-pthread",
                    os.path.join(HERE, "native", "host_pool.cpp"), "-o", str(exe)], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout and "Sanitizer" not in r.stderr
