#!/bin/bash
# round 6: GPU suite of this build, the default bench line, then the store-placement
# skeleton and k_scan alone with HBM vs L2-resident loads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6c
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
cat $D/bench_c2.json
timeout -k 10 120 ./tools/xp/skel > $D/skel.log 2>&1 || exit $?
cat $D/skel.log
for lib in libexp_base.so libexp_l2.so; do
  for cfg in c2 c3; do
    timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}.log 2>&1 || exit $?
    echo "$cfg $lib $(tail -1 $D/${cfg}_${lib}.log | grep -o "'k_scan': [0-9.]*")"
  done
done
