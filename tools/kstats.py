"""Print a rocprofv3 kernel_stats.csv as name / calls / avg us / %."""
import csv
import sys

for r in list(csv.DictReader(open(sys.argv[1])))[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):5.1f}%")
