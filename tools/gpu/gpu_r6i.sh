#!/bin/bash
# round 6: the small-record leg's instruction counts (SQ) and section clocks of this build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6i
mkdir -p $D
export TMPDIR=/tmp
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES"
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
timeout -s KILL 200 rocprofv3 --pmc $S2 --kernel-trace --output-format csv -d $D/small_p2 -o run -- python3 tools/small_once.py libclyscan.so > $D/small_p2.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $S1 --kernel-trace --output-format csv -d $D/small_p1 -o run -- python3 tools/small_once.py libclyscan.so > $D/small_p1.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/small_once.py libexp_prof.so > $D/small_prof.log 2>&1 || exit $?
grep "^xp:" $D/small_prof.log | tail -1
python3 - <<'PY'
import csv, collections
for p in ("small_p2", "small_p1"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open("gpurun_out/r6i/%s/run_counter_collection.csv" % p)):
        k = r["Kernel_Name"].split("(")[0]
        if "k_scan" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k, d in agg.items():
        print(p, k, {c: round(v / len(n[k])) for c, v in sorted(d.items())})
PY
