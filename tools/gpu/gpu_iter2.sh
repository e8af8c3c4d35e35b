#!/bin/bash
# GPU suite on the product build, the fresh-process open probe, the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-iter2}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_open2.sh || exit $?
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
python3 -c "import json,sys; b=json.loads(open('$D/bench_c2.json').read().strip().splitlines()[-1]); print(b['value'], b['kernel'], b.get('small_records'), b.get('index_load'))"
