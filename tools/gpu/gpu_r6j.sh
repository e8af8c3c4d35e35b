#!/bin/bash
# round 6: keys-only index sort (packed hash|del|index keys, fewer radix passes)
# and winner flags: GPU suite, then the index A/B against the previous commit's
# library on C4 and C2 (index_ms, identical per-record states)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6j
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/index_once.py c4 libclyscan.so libexp_fd8e900.so > $D/ix_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/index_once.py c2 libclyscan.so libexp_fd8e900.so > $D/ix_c2.log 2>&1 || exit $?
grep index_ms $D/ix_c4.log $D/ix_c2.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ix_stats -o run -- python3 tools/index_once.py c4 libclyscan.so > $D/ix_stats.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --config c4 --no-host-path --no-cpu-baseline > $D/bench_c4.json 2> $D/bench_c4.err || exit $?
tail -c 1500 $D/bench_c4.json
echo done
