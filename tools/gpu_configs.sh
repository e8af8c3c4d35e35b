#!/bin/bash
# bench lines of BASELINE configs 3, 4 and 5 (per-GPU share) with the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
for c in ${CONFIGS:-c3 c4 c5}; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-host-path ${BENCH_ARGS} > gpurun_out/cfg/bench_$c.json 2> gpurun_out/cfg/bench_$c.err || exit $?
done
exit 0
