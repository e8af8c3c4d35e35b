#!/bin/bash
# the default bench line under rocprofv3 (kernel trace + stats of the same command)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/benchprof
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py > $D/bench.json 2> $D/bench.err || exit $?
tail -1 $D/bench.json | cut -c1-300
python3 tools/bench_trace.py $D/prof/run_kernel_trace.csv
