#!/bin/bash
# round-6 final build, call B (after call A's traffic passes are committed):
# the bench lines C2 (default), C1, C3, C4, C5, the one-GPU rehearsal of
# --gpus 2 (C5 per rank), and the default line under rocprofv3 --stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/finB
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
tail -c 400 $D/bench_c2.json
for cfg in c1 c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-host-path --no-cpu-baseline > $D/bench_$cfg.json 2> $D/bench_$cfg.err || exit $?
  echo "$cfg $(python3 -c "import json,sys; d=json.loads(open('$D/bench_$cfg.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel']['k_scan_ms'], d['roofline']['frac'], d['roofline']['traffic'])")"
done
CLY_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --no-cpu-baseline > $D/rehearse_n2.json 2> $D/rehearse_n2.err || exit $?
tail -c 300 $D/rehearse_n2.json
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_stats -o run -- python3 bench.py --no-host-path --no-cpu-baseline --no-c5-leg > $D/bench_under_rocprof.json 2> $D/bench_stats.err || exit $?
echo done
