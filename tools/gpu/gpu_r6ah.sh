#!/bin/bash
# round 6: no guess at a block's first 4 bytes whose first two bytes are <= 4
# (the structural false start after a record straddling the block start):
# guess probes, GPU suite, same-box A/B against fc16b32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ah
mkdir -p $D
export TMPDIR=/tmp
for c in small c3 c2; do
  timeout -k 10 300 python -u tools/guess_probe.py $c > $D/guess_$c.log 2>&1 || exit $?
done
grep -h "wrong run-start" $D/guess_*.log
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ABDIR=r6ah_ab bash tools/gpu/gpu_ab.sh libclyscan.so libexp_fc16b32.so
