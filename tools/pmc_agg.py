"""Per-dispatch averages of rocprofv3 --pmc passes (run_counter_collection.csv
under DIR/<cfg>_p*), per kernel, with per-4-KiB-block instruction counts:
    python tools/pmc_agg.py DIR c2 [c4 ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
BLOCKS = {"small": 1013434099 / 4096, "c2": 4294966272 / 4096, "c3": 34359738368 / 4096, "c4": 34359738368 / 4096, "c5": 34359738368 / 4096, "c4m": 34359738368 / 4096}
for cfg in sys.argv[2:]:
    vals = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, cfg + "_p*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].strip().split()[-1]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
        for (k, c), v in agg.items():
            vals[k][c] = v / len(disp[(k, c)])
    for k in sorted(vals):
        if not any(c.startswith("SQ_") for c in vals[k]):
            continue
        if vals[k].get("SQ_WAVES", 1e9) < 64 and vals[k].get("SQ_INSTS_VALU", 1e9) < 1e6:
            continue
        print("== %s %s" % (cfg, k))
        for c, v in sorted(vals[k].items()):
            extra = ""
            if c.startswith("SQ_INSTS"):
                extra = "   (%.1f per 4-KiB block)" % (v / BLOCKS[cfg])
            print("  %-24s %18.0f%s" % (c, v, extra))
