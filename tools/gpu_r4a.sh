#!/bin/bash
# round 4: full GPU test suite, smoke, default bench (C2) and the C3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4a_pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/r4a_pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 && echo smoke ok
timeout -k 10 300 python -u bench.py --no-host-path > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err && echo bench ok
timeout -k 10 300 python -u bench.py --config c3 --no-host-path --no-cpu-baseline > gpurun_out/r4a_bench_c3.json 2> gpurun_out/r4a_bench_c3.err && echo bench c3 ok
