#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 pass per counter set).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done < "${1:-tools/pmc_sets_r2d.txt}"
exit 0
