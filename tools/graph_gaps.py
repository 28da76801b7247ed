"""Gaps between consecutive dispatches of a rocprofv3 --kernel-trace CSV (the CP loop's graph
replays): python tools/graph_gaps.py <dir> [marker]
Keeps the dispatches after the first half of the trace (steady state), splits them into
iterations at each dispatch whose name starts with `marker` (default: the CP loop's last
kernel per iteration), and prints per iteration: the span, the summed kernel time and their
difference (the gaps), then the average end -> start gap of every (previous, next) kernel pair."""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:]


def short(r):
    n = r["Kernel_Name"].split("(")[0].replace("void raocp::", "").replace("raocp::", "")
    n = n.replace("(anonymous namespace)::", "")
    n = n.split("<")[0]
    if not n:  # names the trace left empty: grid / workgroup
        n = "grid%s/wg%s" % (r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?")))
    return n


marker = sys.argv[2] if len(sys.argv) > 2 else None
names = [short(r) for r in rows]
if marker is None:
    # the kernel that appears once per iteration and comes last most often
    cnt = collections.Counter(names)
    marker = names[-1]
    print(f"marker {marker} ({cnt[marker]} dispatches)")
iters, cur = [], []
for r, n in zip(rows, names):
    cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if n.startswith(marker):
        iters.append(cur)
        cur = []
iters = [it for it in iters[1:] if it]  # the first may be partial
pairs = collections.defaultdict(list)
spans, busy = [], []
for k, it in enumerate(iters):
    prev_end = iters[k - 1][-1][2] if k else None
    span = it[-1][2] - (prev_end if prev_end is not None else it[0][1])
    spans.append(span)
    busy.append(sum(e - s for _, s, e in it))
    for a, b in zip([iters[k - 1][-1]] + it[:-1] if k else it[:-1], it if k else it[1:]):
        pairs[(a[0], b[0])].append(b[1] - a[2])
if not iters:
    sys.exit("no complete iteration in the trace")
m = len(iters)
print(f"{m} iterations, {len(iters[0])} dispatches each: span {sum(spans) / m / 1e3:.2f} us, "
      f"kernels {sum(busy) / m / 1e3:.2f} us, gaps {(sum(spans) - sum(busy)) / m / 1e3:.2f} us per iteration")
for (a, b), g in sorted(pairs.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {a[:28]:28s} -> {b[:28]:28s} x{len(g) / m:4.1f}/it  mean gap {sum(g) / len(g) / 1e3:6.2f} us")
