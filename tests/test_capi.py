"""CPU: the drop-in boundary.  libfm_hip.so loads, exports every function include/fm_hip.h
declares, the ctypes binding covers exactly that list, and without a GPU the context
constructor fails loudly through the error channel (no crash, no CPU fallback)."""

import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from fm_spark_amd import _native as N

HEADER = Path(__file__).resolve().parents[1] / "include" / "fm_hip.h"


def header_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(fm_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = header_functions()
    for required in ["fm_create", "fm_destroy", "fm_last_error", "fm_step", "fm_step_batch", "fm_predict",
                     "fm_export_tables", "fm_load_tables", "fm_random_split", "fm_shard_route", "fm_shard_owner_update"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = N.load()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.lib_path())], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (fm_\w+)$", out, flags=re.M))
    assert set(header_functions()) <= exported


def test_binding_matches_header():
    assert sorted(N.SIGNATURES) == header_functions()


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from fm_spark_amd.engine import FMContext

    with pytest.raises(N.FMError) as ei:
        FMContext(10, 4)
    assert "fm_create failed" in str(ei.value)


def test_null_arguments_are_errors_not_crashes():
    lib = N.load()
    assert lib.fm_create(None, None) == -1
    assert b"null" in lib.fm_last_error()
    assert lib.fm_step(None, None, 1, 1.0, 0.0, None) == -1
    assert lib.fm_batch_create_splits(None, None, 1, None, None) == -1
    assert lib.fm_batch_split_view(None, None, 0, None) == -1
    assert lib.fm_epoch(None) == -1
    lib.fm_destroy(None)
    lib.fm_batch_destroy(None)


def test_config_layout_matches_header(tmp_path):
    """fm_config as the C compiler lays it out == the ctypes mirror (the multi-GPU fields included)."""
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "fm_hip.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu\\n", sizeof(fm_config), offsetof(fm_config, parallel),'
                   ' offsetof(fm_config, devices), offsetof(fm_config, proc_rank), offsetof(fm_config, comm_id));'
                   'printf("%zu %zu\\n", offsetof(fm_config, fuse_single), offsetof(fm_config, xchg_chunks));'
                   'return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", f"-I{HEADER.parent}", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    F = N.fm_config
    assert got == [C.sizeof(F), F.parallel.offset, F.devices.offset, F.proc_rank.offset, F.comm_id.offset,
                   F.fuse_single.offset, F.xchg_chunks.offset]


def test_multi_gpu_context_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from fm_spark_amd.engine import FMContext

    with pytest.raises(N.FMError):
        FMContext(100, 4, parallel="sharded", n_gpus=2, devices=[0, 0])
    with pytest.raises(N.FMError):  # the copy transport is for one process
        FMContext(100, 4, parallel="sharded", n_gpus=1, n_procs=2, transport="copy")
