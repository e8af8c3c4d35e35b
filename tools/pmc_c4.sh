#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc4
export TMPDIR=/tmp
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc4/p$i -o run -- python bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > gpurun_out/pmc4/p$i.log 2>&1 || exit $?
done < tools/pmc_sets_core.txt
exit 0
