#!/bin/bash
# Round artifacts of the current build: full GPU tests + smoke, the default
# bench line (CPU baseline included), rocprofv3 kernel stats of the same bench
# command, HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one --pmc pass each)
# for C2 and C3, and one SQ counter pass of k_scan.  Each GPU step has its own
# limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/art gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/art/bench.json 2> gpurun_out/art/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/art/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/art/bench_prof.json 2> gpurun_out/art/prof.err || exit $?
i=0
for counter in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counter --kernel-trace --output-format csv -d gpurun_out/art/pmc$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/art/pmc$i.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --pmc $counter --kernel-trace --output-format csv -d gpurun_out/art/c3pmc$i -o run -- python bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/art/c3pmc$i.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/pmc/p1.log 2>&1 || exit $?
exit 0
