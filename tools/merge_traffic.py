#!/usr/bin/env python3
"""profiles/traffic.json from this round's PMC passes only: the union of the given
tools/pmc_traffic.py outputs (one per config), replacing the file so that no bench line can
cite another build's counters.  usage: merge_traffic.py <out.json> <traffic_*.json>..."""
import json
import sys


def main():
    out = {}
    for p in sys.argv[2:]:
        for key, kernels in json.load(open(p)).items():
            out.setdefault(key, {}).update(kernels)
    json.dump(out, open(sys.argv[1], "w"), indent=1, sort_keys=True)
    for key, kernels in sorted(out.items()):
        for k, v in kernels.items():
            print(f"{key} {k}: {v['bytes_per_launch'] / 1e9:.3f} GB/launch (fetch {v['fetch_kib'] / 1e6:.3f} GiB-ish x2, "
                  f"write {v['write_kib'] / 1e6:.3f}) from {v['source']}")


if __name__ == "__main__":
    main()
