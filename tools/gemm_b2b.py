"""Back-to-back time of the headline GEMM at ROWS boards (kv_dev_gemm_clock: the product's fp32-tower GEMM on
seeded random digits for SECONDS, then one stamped launch for the clock). The kernel form follows the
environment (KV_I8R3_K64, KV_R3K64_ABL ...): one line per call.

    KV_I8R3_K64=1 python tools/gemm_b2b.py TAG [ROWS] [DIGITS] [SECONDS]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import _lib  # noqa: E402

tag = sys.argv[1]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
digits = int(sys.argv[3]) if len(sys.argv) > 3 else 3
secs = float(sys.argv[4]) if len(sys.argv) > 4 else 1.5
out = (C.c_double * 4)()
_lib.check(_lib.lib().kv_dev_gemm_clock(0, rows, digits, secs, out), "kv_dev_gemm_clock")
env = {k: v for k, v in os.environ.items() if k.startswith("KV_")}
print(f"{tag} rows={rows} digits={digits} us_back_to_back={out[1]:.1f} sclk_mhz={out[0]:.0f} launches={int(out[2])} "
      f"tpw={int(out[3])} env={env}", flush=True)
