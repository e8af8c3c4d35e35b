#!/bin/bash
# Round artifacts of the current build: full GPU tests + smoke, bench with the
# CPU baseline, rocprofv3 kernel stats of the same bench command, HBM traffic
# passes (FETCH_SIZE / WRITE_SIZE, one --pmc pass each) and the SQ counter
# passes of k_crc / k_spec.  Each GPU step has its own limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/art gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/art/bench.json 2> gpurun_out/art/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/art/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > gpurun_out/art/bench_prof.json 2> gpurun_out/art/prof.err || exit $?
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/art/pmc$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/art/pmc$i.log 2>&1 || exit $?
done < tools/pmc_traffic.txt
i=0
while read -r set; do
  [[ -z "$set" ]] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done < tools/pmc_sets_r2d.txt
exit 0
