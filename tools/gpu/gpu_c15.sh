#!/bin/bash
# bench lines of the other configurations: C5's per-GPU share (one rank's 32 GiB) and C1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/c15
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config c5 --no-host-path --no-cpu-baseline > $D/bench_c5.json 2> $D/bench_c5.err || exit $?
tail -1 $D/bench_c5.json | cut -c1-400
timeout -k 10 300 python -u bench.py --config c1 --no-host-path > $D/bench_c1.json 2> $D/bench_c1.err || exit $?
tail -1 $D/bench_c1.json | cut -c1-400
