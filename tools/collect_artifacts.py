"""Copy a tools/gpu/gpu_r5prof.sh run (gpurun_out/fin) into profiles/ under a tag:
the bench lines (C2 with the host path and index load, C3, C4), the rocprofv3
kernel stats of the C2 / C3 / C4 scans (tools/scan_once.py: one launch per call
over the configuration's own input) and of the C4 bench (scan + merge + hint
rescan), the SQ instruction counters per kernel, and the per-launch HBM traffic
of each kernel from the FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE doubled, as
MI355X_MICROARCH.md's HBM section prescribes for gfx950; both are in KB). The
C4 bench's traffic file lists only the merge kernels: its k_scan launches scan
inputs of different sizes (the 32 GiB and the merged hint file), so the C4
scan's own figure comes from the scan_once passes.
    python tools/collect_artifacts.py r5"""
import collections
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fin = os.path.join(ROOT, "gpurun_out", "fin")
tag = sys.argv[1] if len(sys.argv) > 1 else "r5"
prof = os.path.join(ROOT, "profiles")


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def traffic(cfg, fetch_pass, write_pass, build, only=None, source=""):
    t = {"build": build, "config": cfg, "source": source, "kernels": {}}
    for d, counter, scale in ((fetch_pass, "FETCH_SIZE", 2.0), (write_pass, "WRITE_SIZE", 1.0)):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(os.path.join(fin, d, "run_counter_collection.csv"))):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            if only and not only(k):
                continue
            agg[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k in agg:
            t["kernels"].setdefault(k, {})[counter.lower().replace("_size", "_bytes")] = int(
                agg[k] / len(disp[k]) * 1024 * scale)
    t["note"] = ("per-launch averages; fetch_bytes = FETCH_SIZE x 1024 x 2 (gfx950 half-count correction), "
                 "write_bytes = WRITE_SIZE x 1024")
    return t


b2 = last_json(os.path.join(fin, "bench_c2.json"))
build = b2["kernel"]["build"]
for cfg in ("c2", "c3", "c4"):
    b = last_json(os.path.join(fin, "bench_%s.json" % cfg))
    json.dump(b, open(os.path.join(prof, "%s_bench%s.json" % (tag, "" if cfg == "c2" else "_" + cfg)), "w"), indent=1)
for cfg in ("c2", "c3", "c4", "c5"):
    if not os.path.isdir(os.path.join(fin, cfg + "_stats")):
        continue
    shutil.copy(os.path.join(fin, cfg + "_stats", "run_kernel_stats.csv"),
                os.path.join(prof, "%s_%s_rocprof_kernel_stats.csv" % (tag, cfg)))
    t = traffic(cfg, cfg + "_p3", cfg + "_p4", build, source="tools/scan_once.py %s (one scan per launch)" % cfg)
    json.dump(t, open(os.path.join(prof, "%s_%s_traffic.json" % (tag, cfg)), "w"), indent=1)
    print(cfg, "k_scan traffic", t["kernels"].get("k_scan"), "k_emit", t["kernels"].get("k_emit"))
shutil.copy(os.path.join(fin, "c4m_stats", "run_kernel_stats.csv"),
            os.path.join(prof, "%s_c4_merge_rocprof_kernel_stats.csv" % tag))
t4 = traffic("c4", "c4m_p1", "c4m_p2", build, only=lambda k: k.startswith("k_m") or k.startswith("k_hint"),
             source="bench.py --config c4 (merge kernels only)")
json.dump(t4, open(os.path.join(prof, "%s_c4_merge_traffic.json" % tag), "w"), indent=1)
sq = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_agg.py"), fin, "c2", "c3", "c4", "c5"] +
                    (["c4m"] if os.path.isdir(os.path.join(fin, "c4m_p3")) else []),
                    capture_output=True, text=True).stdout
open(os.path.join(prof, "%s_pmc_sq.txt" % tag), "w").write(
    "# SQ counters per kernel launch (averages), build %s; per-4-KiB-block figures use the config's input bytes\n%s"
    % (build, sq))
print("c2", b2["value"], "merge kernels", {k: v for k, v in t4["kernels"].items()})
