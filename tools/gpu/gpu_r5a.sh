#!/bin/bash
# round 5, first call: GPU suite, default bench, and the self-launched N=2 rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5a
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
head -c 600 $D/bench_c2.json; echo
CLY_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --config c2 --steps 10 --warmup 2 > $D/rehearse_n2.json 2> $D/rehearse_n2.err || exit $?
head -c 600 $D/rehearse_n2.json; echo
echo done
