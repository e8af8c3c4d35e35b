#!/bin/bash
# default bench line (C2 + host path + index load + small records), C4 bench (merge + hint scan)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5e
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
python3 -c "import json; d=json.loads(open('$D/bench_c2.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel'], d.get('small_records'), d.get('index_load'), d.get('host_path'), sep='\n')"
timeout -k 10 500 python -u bench.py --config c4 --no-host-path --no-cpu-baseline > $D/bench_c4.json 2> $D/bench_c4.err || exit $?
python3 -c "import json; d=json.loads(open('$D/bench_c4.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel'], d.get('merge'), sep='\n')"
