"""HBM traffic per launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes:
python tools/traffic.py <tag> [<dir>] reads <dir>/pmc*_{FETCH,WRITE}_SIZE (default gpurun_out,
the runner's tools/gpu_r04.sh pmc step writes gpurun_out/<run tag>/pmc_*).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE tallies wide reads at half their bytes, so it is doubled. Writes
profiles/<tag>/traffic.json: {kernel: {"fetch_bytes", "write_bytes", "traffic_bytes", "launches"}}.
Infinity-Cache hits are counted as fetches (the guide): at cache-resident sizes the
figure is an upper bound on true HBM bytes.
"""
import collections
import csv
import glob
import json
import sys

tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
base = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
for f in glob.glob(f"{base}/pmc*_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        # keep the template arguments: k_ell<20, 8> (config 2) and k_ell<32, 12> (config 4)
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void raocp::", "").replace("raocp::", "").strip()
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    fb = 2.0 * 1024 * sum(cs["FETCH_SIZE"]) / max(1, len(cs["FETCH_SIZE"]))
    wb = 1024.0 * sum(cs["WRITE_SIZE"]) / max(1, len(cs["WRITE_SIZE"]))
    out[k] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
              "launches": max(len(cs["FETCH_SIZE"]), len(cs["WRITE_SIZE"]))}
# aliases under the names raocp_kernel_info gives (the leading template arguments: k_dr<20, 8>
# for k_dr<20, 8, 2, 512, 4>, k_cp4<double, 20, 8> for k_cp4<double, 20, 8, 2, 1, 1>), where the
# truncation names one kernel only
alias = collections.defaultdict(set)
for k in out:
    if "<" in k:
        head, args = k.split("<", 1)
        parts = [a.strip() for a in args.rstrip(">").split(",")]
        for n in range(2, len(parts)):
            alias[f"{head}<{', '.join(parts[:n])}>"].add(k)
for a, ks in alias.items():
    if len(ks) == 1 and a not in out:
        out[a] = dict(out[next(iter(ks))], alias_of=next(iter(ks)))
json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH x2 (gfx950), KB x1024",
           "kernels": out}, open(f"profiles/{tag}/traffic.json", "w"), indent=1)
for k, v in sorted(((k, v) for k, v in out.items() if "alias_of" not in v), key=lambda kv: -kv[1]["traffic_bytes"]):
    print(f"{k:28s} {v['traffic_bytes'] / 1e6:10.3f} MB/launch  ({v['launches']} launches)")
