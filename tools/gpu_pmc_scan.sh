#!/bin/bash
# PMC passes (tools/pmc_scan.txt, one rocprofv3 run per line) over tools/scan_once.py,
# then the per-dispatch averages of kernel $KERN into gpurun_out/pmc/summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  echo "pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/scan_once.py ${CFG:-c2} 2 ${LIB:-libclyscan.so} > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done < "${1:-tools/pmc_scan.txt}"
python3 tools/pmc_agg.py ${KERN:-k_scan} > gpurun_out/pmc/summary.txt
cat gpurun_out/pmc/summary.txt
