#!/bin/bash
# GPU suite, same-box scan-only store experiments, C2/C3 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -4 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_xpcmp.sh c2 libclyscan.so libexp_base.so libexp_nocomp.so libexp_noseg.so libexp_nostore.so || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
head -c 900 $D/bench_c2.json; echo
timeout -k 10 400 python -u bench.py --config c3 --no-host-path --no-cpu-baseline > $D/bench_c3.json 2> $D/bench_c3.err || exit $?
head -c 900 $D/bench_c3.json; echo
