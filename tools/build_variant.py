"""Build an A/B variant of libkv.so with extra compiler flags (e.g. -DKV_...) to
knightvision_amd/<name>; run it with KV_LIB_PATH pointing there.

    python tools/build_variant.py libkv_b.so -DKV_GEMM_STAGED_EPI
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import _build as B  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
out = os.path.join(B.HERE, name)
objs, procs = [], []
for s in B.SRC:
    o = os.path.join("/tmp", "kvvar_" + name + "_" + os.path.basename(s) + ".o")
    cmd = [B.HIPCC, *B.FLAGS, *extra, "-c", s, "-o", o]
    procs.append((subprocess.Popen(cmd), cmd))
    objs.append(o)
for p, cmd in procs:
    if p.wait() != 0:
        raise SystemExit("hipcc failed: " + " ".join(cmd))
subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs])
print(out)
