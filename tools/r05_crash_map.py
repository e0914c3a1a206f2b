"""Map the round-3 rocprofv3 --pmc SIGSEGV stack (profiles/r03_pmc_tree_crash_stack.log) onto a library
layout captured under rocprofv3 --pmc on the GPU box (tools/r05_maps.py): libc's base in the crashed
process is fixed by its __restore_rt frame (libc.so.6 + 0x42520, glibc 2.35), and the libraries mapped
around libc keep their distances from it from one process to the next (same image, same load order), so
each frame's library and offset follow; the offset is then resolved with the library's own symbols.

    python tools/r05_crash_map.py gpurun_out/r05_maps/maps.txt
"""
import re
import subprocess
import sys

STACK = "profiles/r03_pmc_tree_crash_stack.log"
RESTORE_RT = 0x42520


def maps(path):
    out = []
    for line in open(path):
        p = line.split()
        if len(p) >= 6 and p[5].startswith("/"):
            lo, hi = (int(x, 16) for x in p[0].split("-"))
            out.append((lo, hi, int(p[2], 16), p[5]))
    return out


def base_of(mp, name):
    return min(lo - off for lo, hi, off, f in mp if f.endswith(name))


def main():
    mp = maps(sys.argv[1])
    libc_now = base_of(mp, "/libc.so.6")
    frames = [int(m.group(1), 16) for m in re.finditer(r"@\s+(0x[0-9a-f]+)", open(STACK).read())]
    pc = re.search(r"PC: @\s+(0x[0-9a-f]+)", open(STACK).read())
    restore = next(f for f in frames if (f - RESTORE_RT) & 0xfff == 0)
    libc_then = restore - RESTORE_RT
    delta = libc_now - libc_then
    print(f"libc base then {libc_then:#x}, now {libc_now:#x}")
    for f in ([int(pc.group(1), 16)] if pc else []) + frames:
        a = f + delta
        hit = next(((lo, hi, off, name) for lo, hi, off, name in mp if lo <= a < hi), None)
        if not hit:
            print(f"{f:#x}: not in a mapped file of this layout")
            continue
        lo, hi, off, name = hit
        foff = a - lo + off
        sym = ""
        try:
            r = subprocess.run(["addr2line", "-f", "-C", "-e", name, hex(foff)], capture_output=True, text=True,
                               timeout=20)
            sym = r.stdout.split("\n")[0]
        except Exception as e:  # noqa: BLE001
            sym = f"(addr2line: {e})"
        print(f"{f:#x}: {name} + {foff:#x}  {sym}")


if __name__ == "__main__":
    main()
