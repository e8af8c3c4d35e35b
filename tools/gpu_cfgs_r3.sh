#!/bin/bash
# bench lines of C1, C3, C4 and C5 (per-GPU share) with the current build, and the
# k_scan section profile (CLY_PROF experiment build) on C2 and C3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c1 --steps 10 --warmup 2 --no-host-path > gpurun_out/cfg/bench_c1.json 2> gpurun_out/cfg/bench_c1.err || exit $?
for c in c3 c5 c4; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/cfg/bench_$c.json 2> gpurun_out/cfg/bench_$c.err || exit $?
done
if [[ -f couloydb_amd/libclyscan_prof.so ]]; then
  timeout -k 10 200 python -u tools/prof_sections.py c2 libclyscan_prof.so > gpurun_out/cfg/prof_c2.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/prof_sections.py c3 libclyscan_prof.so > gpurun_out/cfg/prof_c3.log 2>&1 || exit $?
fi
exit 0
