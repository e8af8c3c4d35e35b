"""Per-dispatch averages of the tools/gpu_pmc_r3.sh passes, per config and kernel,
with per-4-KiB-block instruction counts for k_scan (python tools/pmc_r3_agg.py > out)."""
import collections
import csv
import glob
import os

ROOT = "gpurun_out/pmcr3"
BLOCKS = {"c2": 4294966272 / 4096, "c3": 34359738368 / 4096, "c4": 34359738368 / 4096}
KERNELS = {"c2": ["k_scan"], "c3": ["k_scan"], "c4": ["k_scan", "k_emit", "k_mcopy", "k_mhint", "k_mplace", "k_mplan"]}
for cfg in ("c2", "c3", "c4"):
    vals = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(ROOT, cfg + "_p*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].strip().split()[-1]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
        for (k, c), v in agg.items():
            vals[k][c] = v / len(disp[(k, c)])
    for k in KERNELS[cfg]:
        if k not in vals:
            continue
        print("== %s %s" % (cfg, k))
        for c, v in sorted(vals[k].items()):
            extra = ""
            if k == "k_scan" and c.startswith("SQ_INSTS"):
                extra = "   (%.1f per block)" % (v / BLOCKS[cfg])
            print("  %-24s %18.0f%s" % (c, v, extra))
