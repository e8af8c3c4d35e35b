#!/bin/bash
# rocprofv3 PMC passes (one per line of $1) over tools/ktime.py c2 1; each pass
# under its own time limit, the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
while read -r C; do
  [[ -z "$C" || "$C" == \#* ]] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc/p$i -o run -- python tools/ktime.py c2 1 > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done < "$1"
exit 0
