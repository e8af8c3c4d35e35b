#!/bin/bash
# the default bench line twice on one box (box-to-box and run-to-run spread of the final build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/bench2
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 400 python -u bench.py > $D/bench_$k.json 2> $D/bench_$k.err || exit $?
  python3 -c "import json; b=json.loads(open('$D/bench_$k.json').read().strip().splitlines()[-1]); print(b['value'], b['ms_per_step'], b['kernel']['k_scan_ms'], b['kernel']['k_emit_ms'], b['roofline']['frac'], b['roofline']['traffic'], b['index_load_wall_ms'], b['small_records']['value'])"
done
