"""Summarise rocprofv3 PMC csv passes for one kernel: HBM bytes per launch =
(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of a wide
coalesced read, MI355X_MICROARCH.md HBM section).

    python tools/pmc_summary.py FETCH_GLOB WRITE_GLOB BATCH [resconv|wino_gemm|wino48_gemm|wino88_gemm|i8f32_gemm|i8f32_lag_gemm|i8f32_lagt_gemm|i8r3_gemm|i8r3k64_gemm|i8_gemm|i8r_gemm]
"""
import csv
import glob
import json
import sys

KERNELS = {
    "resconv": ("conv3x3_kernel<512,32", "conv3x3_kernel<512,32,*>"),
    "wino_gemm": ("wino_gemm_kernel<512,2,2,1,2,16,36>", "wino_gemm_kernel<512,2,2,1,2,16,36>"),
    "wino48_gemm": ("wino_gemm_kernel<512,4,2,1,2,32,60>", "wino_gemm_kernel<512,4,2,1,2,32,60>"),
    "wino88_gemm": ("wino_gemm_kernel<512,4,2,1,2,32,100>", "wino_gemm_kernel<512,4,2,1,2,32,100>"),
    "i8f32_gemm": ("wino88i_gemm_kernel<512,4,true,float,true>", "wino88i_gemm_kernel<512,4,true,float,true>"),
    "i8f32_lag_gemm": ("wino88i32_gemm_lag_kernel<512,false>", "wino88i32_gemm_lag_kernel<512,false>"),
    "i8f32_lagt_gemm": ("wino88i32_gemm_lagt_kernel<512,5", "wino88i32_gemm_lagt_kernel<512,5>"),
    "i8r3_gemm": ("wino88i32_gemm_lagt_kernel<512,5,1,false,3>", "wino88i32_gemm_lagt_kernel<512,5,3>"),
    "i8r3k64_gemm": ("wino88i32_gemm_r3k64_kernel<512,5,false,0>", "wino88i32_gemm_r3k64_kernel<512,5>"),
    "i8_gemm": ("wino88i_gemm_kernel<512,5,true,double>", "wino88i_gemm_kernel<512,5,true,double>"),
    "i8r_gemm": ("wino88i_gemm_lag5_kernel<512,3,4,8,true>", "wino88i_gemm_lag5_kernel<512,3,4,8,true>"),
}


def load(pattern, counter, sub):
    vals = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and sub in r.get("Kernel_Name", "").replace(" ", ""):
                vals.append(float(r["Counter_Value"]))
    return vals


def algorithmic_bytes(kind, B):
    if kind == "resconv":  # activations in + out, weights once
        return B * 64 * 512 * 4 * 2 + 512 * 9 * 512 * 4
    if kind in ("i8f32_gemm", "i8f32_lag_gemm", "i8f32_lagt_gemm", "i8r3_gemm", "i8r3k64_gemm", "i8_gemm",
                "i8r_gemm"):
        # V digits read + M written, U digits once
        d, mb = {"i8_gemm": (5, 8), "i8r_gemm": (4, 8), "i8r3_gemm": (3, 4), "i8r3k64_gemm": (3, 4)}.get(kind, (4, 4))
        return 100 * B * 512 * (d + mb) + 100 * 512 * 512 * d
    xi, rows = {"wino48_gemm": (60, 2 * B), "wino88_gemm": (100, B)}.get(kind, (36, 4 * B))  # V read + M write over the GEMMs, U once
    return xi * rows * 512 * 4 * 2 + xi * 512 * 512 * 4


def main():
    B = int(sys.argv[3])
    kind = sys.argv[4] if len(sys.argv) > 4 else "resconv"
    sub, name = KERNELS[kind]
    fetch = load(sys.argv[1], "FETCH_SIZE", sub)
    write = load(sys.argv[2], "WRITE_SIZE", sub)
    f = sum(fetch) / max(len(fetch), 1)
    w = sum(write) / max(len(write), 1)
    out = {"kernel": name, "batch": B, "launches_fetch": len(fetch), "launches_write": len(write),
           "FETCH_SIZE_kB_avg": f, "WRITE_SIZE_kB_avg": w, "hbm_bytes_per_launch": (2 * f + w) * 1024,
           "algorithmic_min_bytes_per_launch": algorithmic_bytes(kind, B),
           "note": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md; FETCH/WRITE from separate "
                   "--pmc passes"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
