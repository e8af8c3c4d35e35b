#!/bin/bash
# round 6: timing events without system fences: GPU suite, wall-clock A/B
# against 419bf65 (C2, C5, C3), and the C2 bench's kernel trace (gaps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ac
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in c2 c5 c3; do
  timeout -k 10 300 python -u tools/wall_ab.py $c libclyscan.so libexp_419bf65.so > $D/wall_$c.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/wall_ab.py $c libexp_419bf65.so libclyscan.so > $D/wall_${c}_ba.log 2>&1 || exit $?
done
grep -h "wall" $D/wall_*.log
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_stats -o run -- python3 bench.py --no-host-path --no-cpu-baseline --no-c5-leg > $D/bench_under_rocprof.json 2> $D/bench_stats.err || exit $?
echo done
