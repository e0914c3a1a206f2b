"""Per-kernel HBM summary of the Winograd tower from rocprofv3 passes: HBM
bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE
counts half of a wide coalesced read, MI355X_MICROARCH.md HBM section), the
algorithmic bytes of each kernel at this batch, and GB/s with the kernel's
average duration from a --kernel-trace --stats csv.

    python tools/pmc_kernels.py FETCH_GLOB WRITE_GLOB STATS_CSV BATCH > out.json
"""
import csv
import glob
import json
import re
import sys

F32 = 4


def norm(name):
    name = name.replace(" ", "")
    m = re.search(r"(wino\w*kernel<[^>]*>)", name)
    return m.group(1) if m else name.split("(")[0]


def algorithmic(k, B):
    """Bytes a launch must move at B boards (every operand once)."""
    m = re.match(r"wino_gemm_kernel<(\d+),\d+,\d+,\d+,\d+,\d+,(\d+)>", k)
    if m:
        K, xi = int(m.group(1)), int(m.group(2))
        rows = {100: 1, 60: 2, 36: 4}[xi] * B
        return xi * rows * (K + 512) * F32 + xi * 512 * K * F32  # V read + M written, U once
    m = re.match(r"wino88_out_kernel<(\w+),(\w+),(\w+)>", k)
    if m:
        r, y, v = (s == "true" for s in m.groups())
        plane = 64 * 512 * F32
        return B * (100 * 512 * F32 + (plane if r else 0) + (plane if y else 0) + (100 * 512 * F32 if v else 0))
    m = re.match(r"wino88_in_kernel<(\d+)>", k)
    if m:
        C = int(m.group(1))
        return B * (64 * C + 100 * C) * F32
    return None


def load(pattern, counter):
    out = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                out.setdefault(norm(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    avg_ns = {}
    for r in csv.DictReader(open(sys.argv[3])):
        avg_ns[norm(r["Name"])] = float(r["AverageNs"])
    B = int(sys.argv[4])
    res = {}
    for k in sorted(set(fetch) & set(write)):
        f, w = sum(fetch[k]) / len(fetch[k]), sum(write[k]) / len(write[k])
        hbm = (2 * f + w) * 1024
        alg = algorithmic(k, B)
        ns = avg_ns.get(k)
        res[k] = {"launches": len(fetch[k]), "hbm_bytes_per_launch": hbm, "algorithmic_bytes": alg,
                  "traffic_over_algorithmic": hbm / alg if alg else None, "avg_ns": ns,
                  "hbm_GBps": hbm / ns if ns else None}
    print(json.dumps({"batch": B, "kernels": res,
                      "note": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md; FETCH / WRITE from "
                              "separate --pmc passes; avg_ns from the --kernel-trace --stats csv of the same command"},
                     indent=1))


if __name__ == "__main__":
    main()
