#!/bin/bash
# One GPU call, steps chained: smoke, selected pytest files (TESTS, marker
# expression MARK), then optionally bench runs (BENCH="c2 c3 ..." with
# BENCH_ARGS).  Each step runs under its own time limit; the first failure ends
# the call.  Logs land in gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ -z "$NOSMOKE" ]]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ -n "$TESTS" ]]; then
  timeout -k 10 ${TLIM:-900} python -u -m pytest $TESTS -m "${MARK:-gpu}" -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  [[ $rc -ne 0 ]] && exit $rc
fi
for cfg in $BENCH; do
  timeout -k 10 ${BLIM:-400} python -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['kernel'], d['roofline']['frac'], d['parity_ok'])"
done
exit 0
