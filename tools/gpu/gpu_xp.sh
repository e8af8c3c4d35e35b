#!/bin/bash
# timing experiments: kernel stats of scan_once over the libraries named in $@ (C2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${CFG:-c2}
mkdir -p gpurun_out/xp
for lib in "$@"; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xp/${CFG}_$lib -o run -- \
    python3 tools/scan_once.py $CFG 10 $lib > gpurun_out/xp/${CFG}_$lib.log 2>&1 || exit $?
  tail -1 gpurun_out/xp/${CFG}_$lib.log
done
echo done
