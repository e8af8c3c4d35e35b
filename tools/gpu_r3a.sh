#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/prof_sections.py c2 > gpurun_out/r3a/prof_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/prof_sections.py c3 > gpurun_out/r3a/prof_c3.log 2>&1 || exit $?
for c in c3 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r3a/bench_$c.json 2> gpurun_out/r3a/bench_$c.err || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a/c4prof -o run --output-format csv -- python bench.py --config c4 --steps 5 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r3a/bench_c4.json 2> gpurun_out/r3a/bench_c4.err || exit $?
exit 0
