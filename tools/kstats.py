"""Average kernel durations (us) of rocprofv3 --stats CSVs: python tools/kstats.py DIR..."""
import csv
import sys

for d in sys.argv[1:]:
    rows = {r["Name"].split("(")[0].replace("void ", ""): (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
            for r in csv.DictReader(open(d + "/run_kernel_stats.csv"))}
    print(d)
    for k, (us, n) in sorted(rows.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        if not k.startswith("k_gen") and n:
            print("   %-28s %9.1f us x %d" % (k[:28], us, n))
