"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv (measurement tool).

Steps are delimited by the starts of the step's forward kernel; for the last N steps every kernel
that starts inside the step is printed with its start offset, duration and end offset (us), and
per-kernel totals over those steps.

usage: python tools/timeline.py <kernel_trace.csv> [n_steps] [marker] [first_step]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+)", name)
    s = m.group(1) if m else name[:40]
    rb = re.search(r"Li(\d+)EE", name)
    return s + (f"<{rb.group(1)}>" if rb and "radix" in s else "")


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_forward"
    first = int(sys.argv[4]) if len(sys.argv) > 4 else None  # first step index (default: the last n)
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    starts = [s for s, _, k in ev if k.startswith(marker)]
    if len(starts) < n + 1:
        print("not enough steps")
        return
    tot = defaultdict(float)
    lo = len(starts) - n - 1 if first is None else first
    for i in range(lo, lo + n):
        t0, t1 = starts[i], starts[i + 1]
        print(f"--- step {i}: {(t1 - t0) / 1e3:.1f} us")
        for s, e, k in ev:
            if t0 <= s < t1:
                print(f"  {k:28s} start {(s - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}  end {(e - t0) / 1e3:8.1f}")
                tot[k] += (e - s) / 1e3
    print("--- per-step average duration")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {k:28s} {v / n:8.1f} us")


if __name__ == "__main__":
    main()
