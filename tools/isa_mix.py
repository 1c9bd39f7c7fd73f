"""Static instruction mix of kernels in a gfx950 assembly listing (hipcc -S --cuda-device-only).

usage: python tools/isa_mix.py listing.s [substring ...]
Prints, per kernel whose symbol contains one of the substrings, the instruction count and
the counts per class (SALU, VALU, SGPR spill lanes, branches, loads ...).
"""
import collections
import sys


def kernels(lines):
    for i, l in enumerate(lines):
        if l.startswith("_Z") and l.split(";")[0].rstrip().endswith(":"):
            name = l.split(":")[0]
            end = next(j for j in range(i, len(lines)) if lines[j].startswith(".Lfunc_end"))
            yield name, lines[i:end]


def mix(body):
    c = collections.Counter()
    n = 0
    for l in body:
        if not l.startswith("\t"):
            continue
        t = l.strip()
        if not t or t[0] in ";.":
            continue
        op = t.split()[0]
        n += 1
        if op.startswith(("v_readlane", "v_writelane")):
            c["sgpr_spill_lane"] += 1
        elif op.startswith("v_readfirstlane"):
            c["readfirstlane"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            c["s_load"] += 1
        elif op.startswith(("s_cbranch", "s_branch")):
            c["branch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("global_load", "buffer_load", "flat_load")):
            c["vmem_load"] += 1
        elif op.startswith(("global_store", "buffer_store", "flat_store")):
            c["vmem_store"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        else:
            c["other"] += 1
    return n, c


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().split("\n")
    subs = sys.argv[2:] or [""]
    for name, body in kernels(lines):
        if any(s in name for s in subs):
            n, c = mix(body)
            print(f"{name[:90]:90s} {n:6d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
