#!/bin/bash
# round 6: the int8 GEMMs' LDS-DMA copies in the scalar-base + 32-bit-offset address form (KV_COPY_SADDR=1, the
# product build) against 64-bit VGPR address pairs (libkv_nosaddr.so), for R3's 64-k kernel (KV_I8R3_K64=1) and
# 32-k kernel, the 4-digit tower and the fp64 domain on radix-256 digits (KV_PREC=i8r4); every int8 GEMM
# bit-exact test on the product build; forward A/B with outputs compared; back-to-back GEMM times
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-r06_saddr_ab}
mkdir -p $O
export PYTHONUNBUFFERED=1 AB_DIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino_i8_gpu.py \
    -k "gemm_bit_exact or derived_bound" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
NS=$R/knightvision_amd/libkv_nosaddr.so
: > $O/b2b.log
for rep in 1 2; do
    timeout -k 10 60 python -u tools/gemm_b2b.py lagt32 >> $O/b2b.log 2>&1
    KV_LIB_PATH=$NS timeout -k 10 60 python -u tools/gemm_b2b.py lagt32_nosaddr >> $O/b2b.log 2>&1
    KV_I8R3_K64=1 timeout -k 10 60 python -u tools/gemm_b2b.py k64 >> $O/b2b.log 2>&1
    KV_I8R3_K64=1 KV_LIB_PATH=$NS timeout -k 10 60 python -u tools/gemm_b2b.py k64_nosaddr >> $O/b2b.log 2>&1
    timeout -k 10 60 python -u tools/gemm_b2b.py i8 2048 4 >> $O/b2b.log 2>&1
    KV_LIB_PATH=$NS timeout -k 10 60 python -u tools/gemm_b2b.py i8_nosaddr 2048 4 >> $O/b2b.log 2>&1
done
grep -v amdgpu $O/b2b.log
: > $O/ab.log
run() {  # tag env...
    local tag=$1; shift
    env "$@" timeout -k 10 200 python -u tools/ab_forward.py $tag 2048 256 >> $O/ab.log 2>&1
}
for rep in 1 2; do
    run r3k64 KV_ALGO=winograd88i8r3 KV_I8R3_K64=1
    run r3k64ns KV_ALGO=winograd88i8r3 KV_I8R3_K64=1 KV_LIB_PATH=$NS
    run r3 KV_ALGO=winograd88i8r3
    run i8 KV_ALGO=winograd88i8
    run i8ns KV_ALGO=winograd88i8 KV_LIB_PATH=$NS
    run i8r KV_PREC=i8r4
    run i8rns KV_PREC=i8r4 KV_LIB_PATH=$NS
done
python -u - >> $O/ab.log 2>&1 <<'PY'
import numpy as np
for a_, b_ in (("r3", "r3k64"), ("r3k64", "r3k64ns"), ("i8", "i8ns"), ("i8r", "i8rns")):
    for B in (2048, 256):
        for k in ("p", "v"):
            a = np.load(f"/tmp/ab_{a_}_{B}_{k}.npy"); b = np.load(f"/tmp/ab_{b_}_{B}_{k}.npy")
            print(b_, B, k, "bit-identical" if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f"DIFFER max {np.abs(a-b).max():.3e}")
PY
grep -v amdgpu $O/ab.log
echo saddr-ab-done
