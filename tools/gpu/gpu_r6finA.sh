#!/bin/bash
# round-6 final build, call A: GPU suite, then kernel stats, SQ passes and HBM
# traffic passes (C2 / C3 / C4 scans, C4 merge kernels; SQ passes of the merge kernels) -> tools/collect_artifacts.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/fin
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_cmp.sh > $D/cmp.log 2>&1 || exit $?
cp gpurun_out/cmp/bench_c2.json $D/bench_c2.json
timeout -k 10 400 python -u bench.py --config c4 --no-host-path --no-cpu-baseline --no-post-merge-open > $D/bench_c4.json 2> $D/bench_c4.err || exit $?
timeout -k 10 400 python -u bench.py --config c3 --no-host-path --no-cpu-baseline > $D/bench_c3.json 2> $D/bench_c3.err || exit $?
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
for cfg in c2 c3 c4 c5; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/${cfg}_stats -o run -- python3 tools/scan_once.py $cfg 5 > $D/${cfg}_stats.log 2>&1 || exit $?
  i=0
  for s in "$S1" "$S2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d $D/${cfg}_p$i -o run -- python3 tools/scan_once.py $cfg 2 > $D/${cfg}_p$i.log 2>&1 || exit $?
  done
  echo "$cfg passes done"
done
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c4m_stats -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-host-path --no-cpu-baseline --no-post-merge-open > $D/c4m_stats.log 2>&1 || exit $?
i=0
for s in "FETCH_SIZE" "WRITE_SIZE" "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d $D/c4m_p$i -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-host-path --no-cpu-baseline --no-post-merge-open > $D/c4m_p$i.log 2>&1 || exit $?
done
echo done
