#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel trace stored as a rocpd SQLite database
(`rocprofv3 --kernel-trace --stats` without --output-format csv writes <out>_results.db):
calls, average / min / max duration and grid size per kernel name, written as CSV next to it.

usage: python tools/prof_db.py <run_results.db> [out.csv]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else db.replace("_results.db", "_kernel_stats.csv")
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    grid = next((c for c in ("grid_x", "grid_size", "grid_size_x") if c in cols), None)
    extra = [c for c in ("scratch_size", "vgpr_count", "sgpr_count", "lds_size") if c in cols]
    q = f"select {name}, start, end, " + ", ".join([grid or "0"] + extra) + " from kernels"
    agg, info = defaultdict(list), {}
    for row in con.execute(q):
        key = (row[0], row[3])
        agg[key].append(row[2] - row[1])
        info[key] = dict(zip(extra, row[4:]))
    rows = []
    for (k, g), d in agg.items():
        rows.append({"Name": k, "Grid": g, "Calls": len(d), "AverageNs": sum(d) / len(d), "MinNs": min(d),
                     "MaxNs": max(d), "TotalNs": sum(d), **info[(k, g)]})
    rows.sort(key=lambda r: -r["TotalNs"])
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:15]:
        print(f"{r['Name'][:60]:60s} grid {r['Grid']:>9} calls {r['Calls']:4d} avg {r['AverageNs'] / 1e6:.4f} ms "
              f"scratch {r.get('scratch_size')} vgpr {r.get('vgpr_count')}")


if __name__ == "__main__":
    main()
