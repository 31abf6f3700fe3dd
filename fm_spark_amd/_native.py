"""ctypes binding of libfm_hip.so (include/fm_hip.h).

There is deliberately no fallback: if the HIP library is missing or cannot load, every
entry point raises.  The product path never routes through a CPU implementation.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_LIB_PATH = Path(__file__).resolve().parent / "lib" / "libfm_hip.so"

FM_OK = 0
FM_NOTHING_TO_DO = 1
FM_PARALLEL_NONE, FM_PARALLEL_SHARDED, FM_PARALLEL_REPLICATED = 0, 1, 2
FM_TRANSPORT_AUTO, FM_TRANSPORT_RCCL, FM_TRANSPORT_COPY = 0, 1, 2
FM_MAX_LOCAL = 16
FM_FUSE_DEFAULT, FM_FUSE_ON, FM_FUSE_OFF = 0, 1, -1


class FMError(RuntimeError):
    """A negative return code of the C-ABI, with fm_last_error()'s message."""


class fm_config(C.Structure):
    _fields_ = [
        ("num_features", C.c_int64),
        ("k", C.c_int32),
        ("device", C.c_int32),
        ("seed", C.c_uint64),
        ("init_sd", C.c_double),
        ("w0", C.c_double),
        ("shard_index", C.c_int32),
        ("shard_count", C.c_int32),
        ("parallel", C.c_int32),
        ("n_gpus", C.c_int32),
        ("devices", C.c_int32 * FM_MAX_LOCAL),
        ("transport", C.c_int32),
        ("n_procs", C.c_int32),
        ("proc_rank", C.c_int32),
        ("comm_id", C.c_uint8 * 128),
        ("fuse_single", C.c_int32),
        ("xchg_chunks", C.c_int32),
    ]


class fm_csr(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("nnz", C.c_int64),
        ("row_ptr", C.POINTER(C.c_int64)),
        ("col", C.POINTER(C.c_int32)),
        ("val", C.POINTER(C.c_double)),
        ("label", C.POINTER(C.c_double)),
    ]


class fm_step_out(C.Structure):
    _fields_ = [
        ("loss_sum", C.c_double),
        ("n_rows", C.c_int64),
        ("n_loss_rows", C.c_int64),
        ("n_unique", C.c_int64),
    ]


_P = C.c_void_p
_I64P = C.POINTER(C.c_int64)
_I32P = C.POINTER(C.c_int32)
_DP = C.POINTER(C.c_double)

# name -> (restype, argtypes); the full export list of include/fm_hip.h
SIGNATURES = {
    "fm_create": (C.c_int, [C.POINTER(fm_config), C.POINTER(_P)]),
    "fm_destroy": (None, [_P]),
    "fm_last_error": (C.c_char_p, []),
    "fm_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "fm_set_stream": (C.c_int, [_P, _P]),
    "fm_sync": (C.c_int, [_P]),
    "fm_reserve": (C.c_int, [_P, C.c_int64, C.c_int64]),
    "fm_load_tables": (C.c_int, [_P, _I32P, C.c_int64, _DP, _DP]),
    "fm_init_random": (C.c_int, [_P, _I32P, C.c_int64]),
    "fm_init_random_range": (C.c_int, [_P, C.c_int64, C.c_int64]),
    "fm_export_tables": (C.c_int, [_P, _I32P, _DP, _DP, C.c_int64, _I64P]),
    "fm_export_rows": (C.c_int, [_P, _I32P, C.c_int64, _DP, _DP, C.POINTER(C.c_int8)]),
    "fm_num_present": (C.c_int64, [_P]),
    "fm_epoch": (C.c_int64, [_P]),
    "fm_batch_create": (C.c_int, [_P, C.POINTER(fm_csr), C.POINTER(_P)]),
    "fm_batch_destroy": (None, [_P]),
    "fm_batch_prepare": (C.c_int, [_P, _P]),
    "fm_batch_from_rows": (C.c_int, [_P, _P, _I64P, C.c_int64, C.POINTER(_P)]),
    "fm_batch_create_splits": (C.c_int, [_P, C.POINTER(fm_csr), C.c_int32, _I64P, C.POINTER(_P)]),
    "fm_batch_split_view": (C.c_int, [_P, _P, C.c_int32, C.POINTER(_P)]),
    "fm_fuse_active": (C.c_int32, [_P]),
    "fm_batch_rows": (C.c_int64, [_P]),
    "fm_batch_nnz": (C.c_int64, [_P]),
    "fm_step": (C.c_int, [_P, C.POINTER(fm_csr), C.c_int32, C.c_double, C.c_double, C.POINTER(fm_step_out)]),
    "fm_step_batch": (C.c_int, [_P, _P, C.c_int32, C.c_double, C.c_double, C.POINTER(fm_step_out)]),
    "fm_loss_history": (C.c_int, [_P, _DP, C.c_int64, _I64P]),
    "fm_predict": (C.c_int, [_P, C.POINTER(fm_csr), C.c_double, C.c_double, _DP]),
    "fm_predict_batch": (C.c_int, [_P, _P, C.c_double, C.c_double, _DP]),
    "fm_init_from_batch": (C.c_int, [_P, _P, _I64P]),
    "fm_loss_grad": (C.c_int, [_P, C.POINTER(fm_csr), _DP, _DP, _DP, _DP]),
    "fm_calc_loss_grad": (C.c_int, [_P, C.POINTER(fm_csr), C.c_double, C.c_uint64, _DP, _DP, _DP, _DP]),
    "fm_vector_sum_by_key": (C.c_int, [_P, _I32P, C.c_int64, _DP, C.c_int32, _I32P, _DP, _I64P]),
    "fm_profile_enable": (C.c_int, [_P, C.c_int32]),
    "fm_profile_read": (C.c_int, [_P, C.c_char_p, C.c_int64, _DP, _I64P, C.c_int64, _I64P]),
    "fm_profile_reset": (C.c_int, [_P]),
    "fm_read_libsvm": (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, _DP, _I64P, _I32P, _DP, _I64P, _I64P, _I64P]),
    "fm_random_split": (
        C.c_int,
        [C.c_int32, _I64P, C.c_char_p, _DP, C.POINTER(C.c_int8), _I32P, _I64P, _I32P, _DP, _I64P,
         C.c_int32, _DP, C.c_int64, _I32P, _I64P, _I64P],
    ),
    "fm_xorshift_hash_seed": (C.c_int64, [C.c_int64]),
    "fm_murmur3_bytes_hash": (C.c_int32, [C.POINTER(C.c_uint8), C.c_int64, C.c_int32]),
    "fm_xorshift_next_doubles": (C.c_int, [C.c_int64, C.c_int64, _DP]),
    "fm_set_side_stream": (C.c_int, [_P, _P]),
    "fm_shard_route": (C.c_int, [_P, _P, _P, _P, _I64P]),
    "fm_shard_owner_prepare": (C.c_int, [_P, _P, _P, _P, C.c_int64, _I64P, _I64P]),
    "fm_shard_owner_forward": (C.c_int, [_P, _P, _P]),
    "fm_shard_combine": (C.c_int, [_P, _P, _P, _P]),
    "fm_shard_owner_update": (C.c_int, [_P, _P, _P, C.c_int32, C.c_double, C.c_double, C.c_int64]),
    "fm_repl_grad": (C.c_int, [_P, _P, _P]),
    "fm_repl_apply": (C.c_int, [_P, _P, C.c_int32, C.c_double, C.c_double, C.c_int64]),
    "fm_last_stats": (C.c_int, [_P, _DP, _I64P, _I64P]),
}

_lib = None


def lib_path() -> Path:
    return _LIB_PATH


def load() -> C.CDLL:
    """Load libfm_hip.so (raises if it was not built).  When torch is importable it is
    imported first so its bundled HIP runtime (soname libamdhip64.so.7) is the one the
    library binds to: one HIP runtime per process."""
    global _lib
    if _lib is not None:
        return _lib
    # FM_HIP_LIB: another build of the same library (an A/B of two builds in one GPU call)
    path = Path(os.environ.get("FM_HIP_LIB") or _LIB_PATH)
    if not path.exists():
        raise FMError(f"{path} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    if os.environ.get("FM_NO_TORCH_PRELOAD") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().fm_last_error()
        raise FMError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class CSRHost:
    """Keeps the numpy arrays of an fm_csr alive."""

    def __init__(self, row_ptr, col, val, label):
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.val = np.ascontiguousarray(val, dtype=np.float64)
        self.label = np.ascontiguousarray(label, dtype=np.float64)
        if len(self.row_ptr) == 0:
            self.row_ptr = np.zeros(1, dtype=np.int64)
        self.c = fm_csr(
            n_rows=len(self.label),
            nnz=len(self.col),
            row_ptr=ptr(self.row_ptr, C.c_int64),
            col=ptr(self.col, C.c_int32),
            val=ptr(self.val, C.c_double),
            label=ptr(self.label, C.c_double),
        )

    @property
    def n_rows(self) -> int:
        return len(self.label)

    @property
    def nnz(self) -> int:
        return len(self.col)
