"""Per-kernel stats and the last few dispatches from a rocprofv3 rocpd database (measurement tool).

usage: python tools/rocpd_stats.py <results.db> [filter-regex] [n_last]
"""
import glob
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    if not path.endswith(".db"):
        path = glob.glob(path + "/**/*.db", recursive=True)[0]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    n_last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(path)
    t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = next(x for x in t if x.startswith("rocpd_kernel_dispatch"))
    ks = next(x for x in t if x.startswith("rocpd_info_kernel_symbol"))
    rows = list(c.execute(f"select s.kernel_name, d.start, d.end, d.grid_size_x from {kd} d join {ks} s "
                          f"on d.kernel_id = s.id order by d.start"))
    def short(n):
        m = re.search(r"(k_[a-z0-9_]+)", n)
        return (m.group(1) if m else n[:48]) + ("<%s>" % ",".join(re.findall(r"Li(\d+)E", n)) if m else "")
    agg = defaultdict(list)
    for n, s, e, g in rows:
        if pat and not pat.search(n):
            continue
        agg[short(n)].append((e - s) / 1e3)
    print(f"{'kernel':48s} {'calls':>6s} {'avg_us':>9s} {'tot_us':>10s}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:48s} {len(v):6d} {sum(v) / len(v):9.1f} {sum(v):10.1f}")
    if n_last:
        sel = [r for r in rows if not pat or pat.search(r[0])][-n_last:]
        t0 = sel[0][1]
        for n, s, e, g in sel:
            print(f"  {short(n):48s} start {(s - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} grid {g}")


if __name__ == "__main__":
    main()
