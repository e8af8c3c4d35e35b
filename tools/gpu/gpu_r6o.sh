#!/bin/bash
# round 6: the part-view test (both builds), then C5's own traffic passes and
# its bench line (traffic filled from them)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6o
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 150 --timeout-method thread -m gpu -k "past_part_view" > $D/pytest_view.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $D/pytest_view.log
[ $rc -eq 0 ] || exit $rc
i=2
for s in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d $D/c5_p$i -o run -- python3 tools/scan_once.py c5 2 > $D/c5_p$i.log 2>&1 || exit $?
done
echo done
