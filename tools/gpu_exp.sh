#!/bin/bash
# experiment: parity of the small + product builds on corpora, then per-kernel times of LIBS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/check_lib.py libclyscan_small.so --corpora=8 > gpurun_out/check_small.log 2>&1 || exit $?
timeout -k 10 200 python tools/check_lib.py libclyscan.so --corpora=8 > gpurun_out/check.log 2>&1 || exit $?
timeout -k 10 300 python tools/exp_kms.py ${LIBS:-libclyscan.so} > gpurun_out/exp.log 2>&1 || exit $?
if [[ -n "$TESTS" ]]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
fi
exit 0
