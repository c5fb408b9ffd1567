"""Per-dispatch durations and inter-dispatch gaps of one kernel from a
rocprofv3 --kernel-trace CSV (run_kernel_trace.csv).
  python scripts/gaps.py <csv> [name-substring]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if (sys.argv[2] if len(sys.argv) > 2 else "orion") in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
g = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
print("durations us:", " ".join(f"{x:.1f}" for x in d))
print("gaps us:     ", " ".join(f"{x:.1f}" for x in g))
