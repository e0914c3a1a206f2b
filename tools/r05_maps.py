"""Library layout of a python process under rocprofv3 (round-3 SIGSEGV attribution):
import torch, initialise HIP, load libkv.so, run one tiny kernel, then write /proc/self/maps to the path
given as argv[1]. tools/r05_crash_map.py maps the round-3 stack's frame addresses onto it (libc's base
in that stack is known from its __restore_rt frame)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import _lib  # noqa: E402

torch.cuda.init()
x = torch.ones(16, device="cuda") * 2
torch.cuda.synchronize()
_lib.lib()
with open(sys.argv[1], "w") as f:
    f.write(open("/proc/self/maps").read())
print("maps written", float(x.sum()))
