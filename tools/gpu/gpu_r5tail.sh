#!/bin/bash
# C2 kernel stats over 20 scans (the committed average then reflects the
# steady state, not the first call), and the one-GPU N=2 rehearsal of bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/tail
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2_stats20 -o run -- python3 tools/scan_once.py c2 20 > $D/c2_stats20.log 2>&1 || exit $?
CLY_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 2 --config c2 --steps 10 --warmup 2 --no-host-path --no-cpu-baseline > $D/rehearse_n2.json 2> $D/rehearse_n2.err || exit $?
tail -1 $D/rehearse_n2.json
