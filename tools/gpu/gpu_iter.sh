#!/bin/bash
# one iteration: the GPU suite on the product build, a same-box A/B of a
# baseline build ($1) against the product (C2, C3, small records), and the
# default bench line; $2 = output dir name
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${2:-iter}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_ab.sh $1 libclyscan.so || exit $?
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
python3 -c "import json,sys; b=json.loads(open('$D/bench_c2.json').read().strip().splitlines()[-1]); print(b['value'], b['kernel'], b.get('small_records'), b.get('index_load'))"
