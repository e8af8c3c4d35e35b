"""Copy a gpu_final.sh run (gpurun_out/art) into profiles/: the bench line,
the rocprofv3 kernel stats of the same command, and the per-launch HBM traffic
of each kernel from the FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE doubled, as
MI355X_MICROARCH.md's HBM section prescribes for gfx950; both are in KB)."""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
art = os.path.join(ROOT, "gpurun_out", "art")
tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
prof = os.path.join(ROOT, "profiles")
bench = json.loads(open(os.path.join(art, "bench.json")).read().strip().splitlines()[-1])
json.dump(bench, open(os.path.join(prof, "%s_bench.json" % tag), "w"), indent=1)
shutil.copy(os.path.join(art, "prof", "run_kernel_stats.csv"), os.path.join(prof, "%s_rocprof_kernel_stats.csv" % tag))
traffic = {"build": bench["kernel"]["build"], "config": bench["config"]["workload"], "kernels": {}}
for i, (counter, scale) in enumerate((("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)), 1):
    f = os.path.join(art, "pmc%d" % i, "run_counter_collection.csv")
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0]
        agg[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in agg:
        d = traffic["kernels"].setdefault(k, {})
        d[counter.lower().replace("_size", "_bytes")] = int(agg[k] / len(disp[k]) * 1024 * scale)
traffic["note"] = ("per-launch averages; fetch_bytes = FETCH_SIZE x 1024 x 2 (gfx950 half-count correction), "
                   "write_bytes = WRITE_SIZE x 1024")
json.dump(traffic, open(os.path.join(prof, "%s_traffic.json" % tag), "w"), indent=1)
# the C3 passes (bench --config c3), when present
if os.path.exists(os.path.join(art, "c3pmc1", "run_counter_collection.csv")):
    t3 = {"build": traffic["build"], "config": "c3", "kernels": {}}
    for i, (counter, scale) in enumerate((("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)), 1):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(os.path.join(art, "c3pmc%d" % i, "run_counter_collection.csv"))):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            agg[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k in agg:
            t3["kernels"].setdefault(k, {})[counter.lower().replace("_size", "_bytes")] = int(agg[k] / len(disp[k]) * 1024 * scale)
    t3["note"] = traffic["note"]
    json.dump(t3, open(os.path.join(prof, "%s_c3_traffic.json" % tag), "w"), indent=1)
    print("c3 k_scan traffic", t3["kernels"].get("k_scan"))
ks = traffic["kernels"].get("k_scan", {})
print("bench", bench["value"], bench["unit"], "k_scan", bench["kernel"].get("k_scan_ms"), "ms; traffic", ks)
