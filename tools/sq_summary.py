"""Summarise one rocprofv3 --pmc pass of SQ counters (tools/gpu_r05.sh sqpmc): per kernel the
counters averaged over its dispatches, and the wave-cycle split (MI355X_MICROARCH.md rocprofv3
PMC slots: SQ_WAIT_ANY = parked on s_waitcnt / barriers, SQ_WAIT_INST_ANY = issue-stalled,
SQ_ACTIVE_INST_ANY = issuing; the three add up to SQ_WAVE_CYCLES).
python tools/sq_summary.py <rocprofv3 output dir> [kernel substrings...]"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void raocp::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.argv[2:] or ["cp5", "cp3", "cp4", "dy3", "k_dr", "ell3"]
for k, cs in sorted(acc.items()):
    if not any(w in k for w in want):
        continue
    av = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k, f"({len(next(iter(cs.values())))} dispatches)")
    for c, v in sorted(av.items()):
        print(f"   {c:30s} {v:14.4g}")
    wc = av.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print("   split of wave cycles: waiting %.2f  issue-stalled %.2f  issuing %.2f (VALU %.2f)" % (
            av.get("SQ_WAIT_ANY", 0) / wc, av.get("SQ_WAIT_INST_ANY", 0) / wc, av.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            av.get("SQ_ACTIVE_INST_VALU", 0) / wc))
