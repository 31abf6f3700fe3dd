"""Join tools/gather_ceiling.hip's per-variant event times with the TCC_HIT + TCC_MISS counts of a
rocprofv3 --pmc pass over the same binary: L2 requests per second per random-gather variant, and
the ceiling (the largest rate) -> profiles/gather_ceiling.json, which bench.py's roofline.requests
quotes.

  python tools/gather_ceiling.py <bench stdout> <pmc dir> <out json>
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

log, pmc, out = sys.argv[1], sys.argv[2], sys.argv[3]
ms = {}
for line in open(log):
    m = re.match(r"VARIANT (gather<[^>]*>) ms=([0-9.]+) rows=(\d+)", line)
    if m:
        ms[m.group(1).replace(" ", "")] = (float(m.group(2)), int(m.group(3)))
# rocprofv3 -T truncates the kernel names to "gather": the dispatches are attributed to the
# variants by order (each variant: 2 warm-up + 10 timed launches, in the order the tool prints them)
disp = defaultdict(float)
for f in glob.glob(os.path.join(pmc, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("gather") or "gather<" in r["Kernel_Name"]:
            disp[int(r.get("Dispatch_Id") or 0)] += float(r["Counter_Value"])  # TCC_HIT_sum + TCC_MISS_sum
order = [d for d in sorted(disp)]
req = {}
for i, name in enumerate(ms):  # dict order = the tool's print order
    chunk = order[12 * i: 12 * (i + 1)]
    if len(chunk) == 12:
        req[name] = [disp[d] for d in chunk[2:]]  # the timed launches
variants = {}
for name, (t, n) in ms.items():
    per = req.get(name, [])
    if not per:
        continue
    r = sum(per) / len(per)
    variants[name] = {"ms": t, "gathers": n, "l2_requests": r, "requests_per_gather": r / n,
                      "l2_requests_per_s": r / (t * 1e-3)}
synth = [v for k, v in variants.items() if k.endswith(",0>") or k.endswith(",1>")]
ceil = max(synth, key=lambda v: v["l2_requests_per_s"]) if synth else None
uni = [v for k, v in variants.items() if k.endswith(",0>")]
ceil_uni = max(uni, key=lambda v: v["l2_requests_per_s"]) if uni else None
# c3's own forward address stream (tools/c3_stream.py): its ids gathered in CSR order (MODE 2), and
# the fused forward's memory skeleton (MODE 3: CSR stream, whole-record gathers, singleton write-back,
# S records), whose time is the floor of the forward's access stream
c3 = {k: v for k, v in variants.items() if k.endswith(",2>") or k.endswith(",3>") or k.endswith(",4>")}
res = {"what": "L2 requests (TCC_HIT_sum + TCC_MISS_sum) per second of random row gathers "
               "(tools/gather_ceiling.hip: 10.2M gathers over a 100M-record table; <LPR lanes, U in flight, "
               "record floats, 0 uniform / 1 40 % hot>)",
       "variants": variants,
       "l2_requests_per_s": ceil["l2_requests_per_s"] if ceil else None,
       "uniform_l2_requests_per_s": ceil_uni["l2_requests_per_s"] if ceil_uni else None,
       "c3_stream": {"what": "one c3 batch's forward stream (tools/c3_stream.py, bench.py's first c3 batch): "
                             "<4,8,32,2> / <8,4,32,2> its ids gathered in CSR order (64 B / the whole 128-B record); "
                             "<8,5,32,3> the fused forward's memory skeleton (row_ptr, ids and x read, every row's "
                             "128-B record gathered, the singleton rows' records written back, the 128-B S record "
                             "written; no arithmetic); <4,3,32,4> the same skeleton in the forward's lane shape "
                             "(4 lanes of V quads + a header load per row, the record written back in two stores)",
                     "variants": c3} if c3 else None,
       "source": {"log": log, "pmc": pmc}}
open(out, "w").write(json.dumps(res, indent=1, sort_keys=True) + "\n")
print(json.dumps({k: v["l2_requests_per_s"] / 1e9 for k, v in variants.items()}, indent=1))
