"""Average SQ / GRBM counters per dispatch for the kernels of a rocprofv3 --pmc csv
whose names contain one of the given substrings (default: conv3x3).

    python tools/pmc_sq.py CSV_GLOB [substring ...]
"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1], recursive=True):
    if "counter_collection" not in f:
        continue
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(s in k for s in (sys.argv[2:] or ["conv3x3"])):
            continue
        short = k.split("(")[0].replace("void kv::", "")
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[short]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}")
