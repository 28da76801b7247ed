"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc2_*): per kernel, counters averaged per launch."""
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc2_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void raocp::", "").replace("raocp::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.argv[1:] or None
for k, cs in acc.items():
    if want and not any(w in k for w in want):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:36s} {sum(v) / len(v):14.4g}")
