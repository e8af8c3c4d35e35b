#!/bin/bash
# Round artifacts: bench with CPU baseline, rocprofv3 kernel stats of the same
# command, HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one --pmc pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/art
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/art/bench.json 2> gpurun_out/art/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/art/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/art/bench_prof.json 2> gpurun_out/art/prof.err || exit $?
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/art/pmc$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/art/pmc$i.log 2>&1 || exit $?
done < tools/pmc_traffic.txt
exit 0
