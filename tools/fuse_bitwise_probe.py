"""Measurement tool (not product): is the fused step (singleton rows updated by the forward) bitwise
the unfused step?  The cases of tests/test_gpu_fuse.py; prints per case whether losses and tables
are bitwise equal, and the largest relative table difference (round 4: bitwise with the update
walking the whole sorted view, profiles/r04_j; not with the compacted multi view, whose run pieces
meet at other wave boundaries)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from problems import make_problem  # noqa: E402
from test_gpu_fuse import _steps  # noqa: E402

res = {}
for k in (3, 8, 12, 16):
    F = 20000
    csrs = [make_problem(700 + i, 1500, F, k, 12, hot=5 + i)[0] for i in range(3)]
    _, ids, w, V = make_problem(77, 1, F, k, 1)
    a = _steps(True, csrs, F, k, ids, w, V, 4)
    b = _steps(False, csrs, F, k, ids, w, V, 4)
    same_l = a[0] == b[0]
    same_t = all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))
    d = max(float(np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-30))) if x.size else 0.0 for x, y in zip(a[1][1:], b[1][1:]))
    res[f"k{k}"] = {"losses_bitwise": same_l, "tables_bitwise": same_t, "max_rel_diff": d}
for k in (8, 16):
    F = 400_000
    csrs = [make_problem(900 + i + k, 40_000, F, k, 10, empty_frac=0.05)[0] for i in range(2)]
    _, ids, w, V = make_problem(76, 1, F, k, 1)
    a = _steps(True, csrs, F, k, ids, w, V, 3, reg=1e-2)
    b = _steps(False, csrs, F, k, ids, w, V, 3, reg=1e-2)
    res[f"many_k{k}"] = {"losses_bitwise": a[0] == b[0],
                         "tables_bitwise": all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))}
print(json.dumps(res, indent=1))
