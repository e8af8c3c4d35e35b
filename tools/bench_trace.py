"""k_scan launches of bench.py's timed loop from a rocprofv3 kernel trace of
the bench itself (`rocprofv3 --kernel-trace --stats -- python3 bench.py`):
the k_scan launches in issue order are split into runs of similar duration
(within 25 % of the run's first); the longest run holds the index-rebuild
scans, the warm-up and the timed steps, of which the last STEPS (default 20)
are the timed ones. Prints their count and average duration, to set beside the
bench line's HIP-event k_scan time.
    python tools/bench_trace.py DIR/run_kernel_trace.csv [STEPS]"""
import csv
import sys

steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
      if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] == "k_scan"]
runs, cur = [], []
for d in ks:
    if cur and abs(d - cur[0]) > 0.25 * cur[0]:
        runs.append(cur)
        cur = []
    cur.append(d)
runs.append(cur)
best = max(runs, key=len)[-steps:]
print("k_scan: %d launches in the trace; the timed loop's last %d: average %.4f ms, min %.4f, max %.4f" % (
    len(ks), len(best), sum(best) / len(best), min(best), max(best)))
