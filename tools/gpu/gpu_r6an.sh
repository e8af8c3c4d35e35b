#!/bin/bash
# round 6: the scan call's final wait polls the stream instead of blocking:
# same-box wall-clock A/B of whole scan calls against e99ced4 (C2, C1, C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6an
mkdir -p $D
export TMPDIR=/tmp
for cfg in c2 c1 c3; do
  timeout -k 10 300 python -u tools/wall_ab.py $cfg libclyscan.so libexp_e99ced4.so > $D/wall_$cfg.log 2>&1 || exit $?
  grep wall $D/wall_$cfg.log
done
timeout -k 10 400 python -u bench.py --no-host-path --no-cpu-baseline > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
python3 -c "import json; d=json.loads(open('$D/bench_c2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel']['all_ms'])"
