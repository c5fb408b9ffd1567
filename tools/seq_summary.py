"""Per-dispatch durations of our kernels from a rocprofv3 run (kernel trace, optionally
with GRBM_GUI_ACTIVE per dispatch: cycles / duration = the effective GPU clock), in
dispatch order, in blocks of 10 launches: how a kernel's time moves over a sequence.
  python tools/seq_summary.py gpurun_out/<tag>/<cfg> [--filter orion]"""
import argparse
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--filter", default="orion")
    a = ap.parse_args()
    rows, grbm = [], {}
    for db in sorted(glob.glob(os.path.join(a.root, "**", "*.db"), recursive=True)):
        cur = sqlite3.connect(db).cursor()
        tabs = {r[0] for r in cur.execute("select name from sqlite_master")}
        if "counters_collection" in tabs:
            for did, v in cur.execute("select dispatch_id, sum(value) from counters_collection "
                                      "where counter_name = 'GRBM_GUI_ACTIVE' group by dispatch_id"):
                grbm[did] = v
        if "kernels" in tabs:
            cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
            did = "dispatch_id" if "dispatch_id" in cols else None
            q = f"select name, start, end{', ' + did if did else ''} from kernels order by start"
            for r in cur.execute(q):
                if a.filter in r[0]:
                    rows.append((r[0].split("(")[0].replace("void ", "").replace("orion::", ""), r[1], r[2],
                                 r[3] if did else None))
    if not rows:
        print("no dispatches")
        return
    name = max({r[0] for r in rows}, key=lambda k: sum(1 for r in rows if r[0] == k))
    seq = [r for r in rows if r[0] == name]
    t0 = seq[0][1]
    print(f"{name}: {len(seq)} dispatches in order (us): start offset, duration, clock MHz (GRBM_GUI_ACTIVE / duration)")
    for i, (_, s, e, d) in enumerate(seq):
        dur = (e - s) / 1e3
        clk = f"{grbm[d] / (e - s) * 1e3:7.0f}" if d in grbm and e > s else "      -"
        print(f"  {i:3d} {(s - t0) / 1e3:10.1f} {dur:9.2f} {clk}")
    print("blocks of 10 launches: median duration (us), median clock (MHz)")
    for b in range(0, len(seq), 10):
        blk = seq[b: b + 10]
        ds = sorted((e - s) / 1e3 for _, s, e, _ in blk)
        cs = sorted(grbm[d] / (e - s) * 1e3 for _, s, e, d in blk if d in grbm and e > s)
        print(f"  {b:3d}-{b + len(blk) - 1:3d}: {ds[len(ds) // 2]:9.2f} us  "
              f"{(f'{cs[len(cs) // 2]:6.0f} MHz' if cs else '')}")


if __name__ == "__main__":
    main()
