#!/bin/bash
# round 6: link / k_emit / k_fin markers only on request: GPU suite, wall-clock
# A/B against 82f6533 (C2, C1 both orders; C5), and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ad
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in c2 c1 c5; do
  timeout -k 10 300 python -u tools/wall_ab.py $c libclyscan.so libexp_82f6533.so > $D/wall_$c.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/wall_ab.py $c libexp_82f6533.so libclyscan.so > $D/wall_${c}_ba.log 2>&1 || exit $?
done
grep -h "wall" $D/wall_*.log
timeout -k 10 400 python -u bench.py --no-host-path --no-cpu-baseline --no-c5-leg > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
tail -c 700 $D/bench_c2.json
