"""k_scan launches of bench.py's timed loop from a rocprofv3 kernel trace of
the bench itself (`rocprofv3 --kernel-trace --stats -- python3 bench.py`):
the longest run of consecutive scan calls (k_scan .. k_fin, nothing else
between them) is the warm-up + timed steps; prints their count and average
k_scan duration, to set beside the bench line's HIP-event k_scan time.
    python tools/bench_trace.py DIR/run_kernel_trace.csv"""
import csv
import sys

SCAN = ("k_scan", "k_link", "k_refix", "k_emit", "k_fin", "__amd_rocclr_copyBuffer")
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
runs, cur = [], []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    if name not in SCAN:
        if cur:
            runs.append(cur)
        cur = []
        continue
    if name == "k_scan":
        cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
if cur:
    runs.append(cur)
best = max(runs, key=len)
print("k_scan launches in the longest run of scan calls: %d, average %.4f ms, min %.4f, max %.4f" % (
    len(best), sum(best) / len(best), min(best), max(best)))
