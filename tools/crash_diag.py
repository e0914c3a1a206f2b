"""Run bench.py with the crashmaps SIGSEGV handler installed (diagnostics
only): under `rocprofv3 --pmc ... -- python3 tools/crash_diag.py <bench args>`
the profiler's crash prints each frame's library, offset and nearest dynamic
symbol and the executable mappings (tools/crashdiag/crashmaps.c), so the
faulting library can be named. Build the handler first (gcc, host code):
    gcc -O1 -shared -fPIC -o tools/crashdiag/libcrashmaps.so tools/crashdiag/crashmaps.c -ldl
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ctypes.CDLL(os.path.join(HERE, "crashdiag", "libcrashmaps.so")).crashmaps_install()
sys.path.insert(0, os.path.dirname(HERE))
sys.argv = [os.path.join(os.path.dirname(HERE), "bench.py")] + sys.argv[1:]
import bench  # noqa: E402

sys.exit(bench.main())
