#!/bin/bash
# round 4: full GPU suite; C2 kernel stats + SQ counters; C4 merge bench + stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4c/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -8 gpurun_out/r4c/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-host-path --no-cpu-baseline > gpurun_out/r4c/bench_c2.json 2> gpurun_out/r4c/bench_c2.err || exit $?
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
i=0
for s in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $s --kernel-trace --output-format csv -d gpurun_out/r4c/c2_p$i -o run -- python3 tools/scan_once.py c2 2 > gpurun_out/r4c/c2_p$i.log 2>&1 || exit $?
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/c2_stats -o run -- python3 tools/scan_once.py c2 10 > gpurun_out/r4c/c2_stats.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config c4 --no-host-path --no-cpu-baseline > gpurun_out/r4c/bench_c4.json 2> gpurun_out/r4c/bench_c4.err || exit $?
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/c4_stats -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r4c/c4_stats.log 2>&1 || exit $?
i=0
for s in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d gpurun_out/r4c/c4_p$i -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r4c/c4_p$i.log 2>&1 || exit $?
done
echo done
