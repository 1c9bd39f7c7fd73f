#!/usr/bin/env python3
"""Compact table of the eval kernels' register use, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (tools/isa_stats.sh writes /tmp/isa/remarks.txt).

usage: python tools/regs.py [remarks.txt]
"""
import re
import sys

FIELDS = ("VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
          "LDS Size [bytes/block]")


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa/remarks.txt"
    rows, cur = [], None
    pat = re.compile(r":\d+:\d+: +(?:remark: +)?(Function Name|" + "|".join(re.escape(f) for f in FIELDS) + r"): (\S+)")
    for line in open(path, errors="replace"):
        m = pat.search(line)
        if not m:
            continue
        if m.group(1) == "Function Name":
            cur = {"name": m.group(2)}
            rows.append(cur)
        elif cur is not None:
            cur[m.group(1)] = m.group(2)
    for r in rows:
        n = r["name"]
        if "allowed" not in n and "template" not in n:
            continue
        n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)
        n = re.sub(r"EE?EvN.*", "", n).replace("IN3acs", "<").replace("ELb", ",")
        print(f"{n:44s} vgpr {r.get('VGPRs', '?'):>4} scratch {r.get(FIELDS[1], '?'):>4} "
              f"occ {r.get(FIELDS[2], '?')} sgpr-spill {r.get('SGPRs Spill', '?'):>4} "
              f"vgpr-spill {r.get('VGPRs Spill', '?'):>3} lds {r.get(FIELDS[5], '?')}")


if __name__ == "__main__":
    main()
