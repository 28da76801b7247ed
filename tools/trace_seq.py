"""Launch sequence of a rocprofv3 --kernel-trace CSV: python tools/trace_seq.py <dir> [last N]
prints the last N dispatches in start order: kernel, grid, workgroup, duration and the gap
since the previous dispatch ended (ns)."""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
prev = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void raocp::", "")
    grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    wg = r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?"))
    gap = "" if prev is None else f"{s - prev:8d}"
    print(f"{name[:44]:44s} grid {grid:>8s} wg {wg:>5s} {e - s:9d} ns {gap}")
    prev = e
