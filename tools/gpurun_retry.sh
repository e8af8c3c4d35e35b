#!/bin/bash
# Re-submit a gpurun call only when the infrastructure failed before the command
# ran (status=transient / exit 3: no box, nothing executed, nothing charged).
# A command that ran and failed is never re-run.
T=${GPU_TIMEOUT:-900}
for i in 1 2 3 4 5 6; do
  rm -f gpurun_out/.last_call.json
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if [[ $rc -eq 3 ]] || echo "$out" | grep -q "status=transient"; then
    echo "[retry] infrastructure transient, attempt $i; sleeping 60s"; sleep 60; continue
  fi
  exit $rc
done
exit 3
