#!/bin/bash
# gpurun a command, waiting while the pool has no free box (exit 3 / "transient":
# nothing ran, nothing charged); any other outcome is returned as it is
out=${OUT:-/tmp/gpurun_wait.out}
for i in $(seq 1 ${TRIES:-20}); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out; then sleep ${WAIT:-90}; continue; fi
  cat $out; exit $rc
done
cat $out; exit $rc
