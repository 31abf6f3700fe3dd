"""Turn the rocprofv3 --pmc passes of tools/pmc.sh into the per-launch traffic JSON that
bench.py reports as roofline.traffic (profiles/pmc_<config>.json).

Corrections (MI355X_MICROARCH.md, HBM section, and our own calibration, tools/traffic_cal.hip,
profiles/r01_v2/cal): FETCH_SIZE and WRITE_SIZE are in KiB.  WRITE_SIZE counts whole-granule
row writes exactly (wr128: 1.328 GB counted for 1.309 GB written).  FETCH_SIZE counts read
requests x 64 B: a 128-B line request (the row gathers: V + header of one 128-B record, and
coalesced streams) is tallied at half its bytes (rd80 and stream: exactly 1/2), a 64-B request
in full (rd64: 1.03x).  The step kernels' reads are line requests except the update's S-row
gathers (64 B), so  traffic = 2 * FETCH + WRITE  is exact for k_forward and an upper bound
for k_segment_update (its S gathers are double counted).  With a 4th argument (a directory of
the update's ablation passes: base-FETCH_SIZE.csv and nos-FETCH_SIZE.csv, a build with and
without the S-row loads, as round 2 made them) the S gathers' FETCH share is measured and counted
once: traffic = 2 * (FETCH - S) + S + WRITE for k_segment_update."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else None
meta = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
# meta "timed_steps": N keeps only the last N launches of the once-per-step kernels of the main
# stream (bench.py's warmup and U-count steps run unprepared batches, i.e. the unfused variant)
timed = int(meta.get("timed_steps", 0))
PER_STEP = ("k_forward", "k_segment_update", "k_segment_combine", "k_pack_srec")
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")) +
                glob.glob(os.path.join(src, "p*_counters.csv"))):
    per = defaultdict(list)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append((int(r.get("Dispatch_Id") or 0),
                                                                         float(r["Counter_Value"])))
    for (kn, cn), vals in per.items():
        vals.sort()
        if timed and kn in PER_STEP:
            vals = vals[-timed:]
        acc[kn][cn] += [v for _, v in vals]
res = {"source": src, "units": "bytes per launch", **meta, "kernels": {}}
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    e = {"counters": m}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        e["fetch_bytes_counted"] = m["FETCH_SIZE"] * 1024
        e["write_bytes"] = m["WRITE_SIZE"] * 1024
        e["traffic_bytes"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
    res["kernels"][k] = e
abl = sys.argv[4] if len(sys.argv) > 4 else None
if abl and "k_segment_update" in res["kernels"]:

    def mean_fetch(path):
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
             if r["Kernel_Name"].startswith("k_segment_update") and r["Counter_Name"] == "FETCH_SIZE"]
        return sum(v) / len(v)

    s_kib = mean_fetch(os.path.join(abl, "base-FETCH_SIZE.csv")) - mean_fetch(os.path.join(abl, "nos-FETCH_SIZE.csv"))
    e = res["kernels"]["k_segment_update"]
    e["s_gather_fetch_bytes"] = s_kib * 1024
    e["traffic_bytes"] = 2 * (e["fetch_bytes_counted"] - s_kib * 1024) + s_kib * 1024 + e["write_bytes"]
    res["update_s_correction"] = abl
txt = json.dumps(res, indent=1, sort_keys=True)
if out:
    open(out, "w").write(txt + "\n")
else:
    print(txt)
