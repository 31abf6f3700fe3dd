"""CPU oracle — TEST INFRASTRUCTURE ONLY.  ctypes wrapper + build recipe for fm_oracle.c
(the fp64 OpenMP C restatement used as second oracle and as bench.py's cpu_baseline)."""

from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = HERE / "fm_oracle.c"
LIB = HERE / "_build" / "liboracle.so"


def build(force: bool = False) -> Path:
    LIB.parent.mkdir(exist_ok=True)
    if force or not LIB.exists() or SRC.stat().st_mtime > LIB.stat().st_mtime:
        # portable flags: the library is built here and runs on the GPU box's host CPU
        subprocess.run(["gcc", "-O3", "-fopenmp", "-fPIC", "-shared", "-std=c11", str(SRC), "-o", str(LIB), "-lm"],
                       check=True)
    return LIB


def load():
    if not LIB.exists():
        build()
    lib = C.CDLL(str(LIB))
    P = C.c_void_p
    lib.oracle_create.argtypes = [C.c_int64, C.c_int32, C.c_double, C.POINTER(P)]
    lib.oracle_create.restype = C.c_int
    lib.oracle_destroy.argtypes = [P]
    lib.oracle_load.argtypes = [P, C.POINTER(C.c_int32), C.c_int64, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.oracle_init_random.argtypes = [P, C.c_uint64, C.c_double, C.c_int64, C.c_int64]
    lib.oracle_init_device_draw.argtypes = [P, C.c_uint64, C.c_double, C.c_int64, C.c_int64]
    lib.oracle_step.argtypes = [P, C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                C.POINTER(C.c_double), C.c_int64, C.c_int32, C.c_double, C.c_double,
                                C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.oracle_step.restype = C.c_int
    lib.oracle_w.argtypes = [P]
    lib.oracle_w.restype = C.POINTER(C.c_double)
    lib.oracle_V.argtypes = [P]
    lib.oracle_V.restype = C.POINTER(C.c_double)
    lib.oracle_present.argtypes = [P]
    lib.oracle_present.restype = C.POINTER(C.c_uint8)
    lib.oracle_num_threads.restype = C.c_int
    lib.oracle_set_threads.argtypes = [C.c_int]
    return lib


def threads(lib) -> int:
    return int(lib.oracle_num_threads())


def create(lib, F: int, k: int, w0: float = 0.0):
    h = C.c_void_p()
    rc = lib.oracle_create(int(F), int(k), float(w0), C.byref(h))
    if rc != 0:
        raise MemoryError("oracle_create failed")
    return h


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def load_tables(lib, m, ids, w, V):
    ids = np.ascontiguousarray(ids, np.int32)
    w = np.ascontiguousarray(w, np.float64)
    V = np.ascontiguousarray(V, np.float64)
    lib.oracle_load(m, _p(ids, C.c_int32), len(ids), _p(w, C.c_double), _p(V, C.c_double))


def step(lib, m, batch, t, step_size, reg_param):
    rp = np.ascontiguousarray(batch.row_ptr, np.int64)
    col = np.ascontiguousarray(batch.col, np.int32)
    val = np.ascontiguousarray(batch.val, np.float64)
    lab = np.ascontiguousarray(batch.label, np.float64)
    loss = C.c_double()
    nl = C.c_int64()
    nu = C.c_int64()
    rc = lib.oracle_step(m, _p(rp, C.c_int64), _p(col, C.c_int32), _p(val, C.c_double), _p(lab, C.c_double),
                         len(lab), int(t), float(step_size), float(reg_param), C.byref(loss), C.byref(nl),
                         C.byref(nu))
    return rc, loss.value, nl.value, nu.value


def tables(lib, m, F, k):
    w = np.ctypeslib.as_array(lib.oracle_w(m), shape=(F,)).copy()
    V = np.ctypeslib.as_array(lib.oracle_V(m), shape=(F * k,)).copy().reshape(F, k)
    pres = np.ctypeslib.as_array(lib.oracle_present(m), shape=(F,)).astype(bool)
    return w, V, pres
