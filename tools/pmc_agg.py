"""Aggregate rocprofv3 PMC passes (gpurun_out/pmc/p*) per dispatch of a kernel."""
import collections, csv, glob, sys
kern = sys.argv[1] if len(sys.argv) > 1 else "k_scan"
for f in sorted(glob.glob("gpurun_out/pmc/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
    for k, v in agg.items():
        print("%-28s %16.0f" % (k, v / len(cnt[k])))
