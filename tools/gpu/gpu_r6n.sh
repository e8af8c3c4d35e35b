#!/bin/bash
# round 6: index winners as a bitmap (after gpu_r6m.sh): GPU suite, index A/B
# against the previous commit's library on C4 and C2, kernel stats of both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${TAG:-r6n}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/index_once.py c4 libclyscan.so libexp_fd8e900.so > $D/ix_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/index_once.py c2 libclyscan.so libexp_fd8e900.so > $D/ix_c2.log 2>&1 || exit $?
grep index_ms $D/ix_c4.log $D/ix_c2.log
for c in c4 c2; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ix_stats_$c -o run -- python3 tools/index_once.py $c libclyscan.so > $D/ix_stats_$c.log 2>&1 || exit $?
done
echo done
