"""Summarise rocprofv3 rocpd databases: per-kernel average duration (kernel-trace
runs) and per-dispatch PMC counter averages (--pmc runs), for our kernels.

  python scripts/prof_summary.py gpurun_out/<tag> [--filter orion] [--json out.json]

FETCH_SIZE is reported raw and x2 (MI355X_MICROARCH.md §HBM: on gfx950 it reads
exactly half the bytes of a wide coalesced streaming read).
"""
import argparse
import glob
import json
import os
import sqlite3
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("orion::", "")
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--filter", default="orion")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    out = {"kernels": {}, "counters": defaultdict(dict)}
    for db in sorted(glob.glob(os.path.join(args.root, "**", "*.db"), recursive=True)):
        cur = sqlite3.connect(db).cursor()
        tabs = {r[0] for r in cur.execute("select name from sqlite_master")}
        if "kernels" in tabs:
            for name, avg, cnt in cur.execute(
                    "select name, avg(duration), count(*) from kernels group by name"):
                if args.filter in name:
                    out["kernels"].setdefault(short(name), {"avg_us": avg / 1e3, "calls": cnt, "db": db})
        if "counters_collection" in tabs:
            rows = cur.execute("select kernel_name, counter_name, dispatch_id, sum(value) from counters_collection "
                               "group by kernel_name, counter_name, dispatch_id").fetchall()
            acc = defaultdict(list)
            for kname, cname, _, v in rows:
                if args.filter in kname:
                    acc[(short(kname), cname)].append(v)
            for (k, c), vs in acc.items():
                out["counters"][k][c] = sum(vs) / len(vs)
    print("kernel durations (kernel-trace runs):")
    for k, v in out["kernels"].items():
        print(f"  {k:40s} avg {v['avg_us']:9.2f} us  calls {v['calls']}")
    print("counters (mean per dispatch):")
    for k, cs in out["counters"].items():
        print(f"  {k}")
        for c, v in sorted(cs.items()):
            extra = f"   (x2 = {2 * v:.4g})" if c == "FETCH_SIZE" else ""
            print(f"     {c:28s} {v:16.6g}{extra}")
    if args.json:
        json.dump(out, open(args.json, "w"), indent=1, default=float)


if __name__ == "__main__":
    main()
