#!/bin/bash
# skeleton microbench, then the index/load GPU tests (ordered enumeration)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 ./tools/xp/skel > $D/skel.log 2>&1 || exit $?
cat $D/skel.log
timeout -k 10 400 python -u -m pytest tests/test_index_keys.py tests/test_load_driver.py -q -x --timeout 120 --timeout-method thread -m gpu > $D/pytest_ix.log 2>&1
rc=$?; tail -15 $D/pytest_ix.log; exit $rc
