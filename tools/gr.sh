#!/bin/bash
# local helper: run a command on the GPU box via gpurun (retrying transient
# failures up to 3 times); stale gpurun_out/*.log are removed first.
# usage: tools/gr.sh TIMEOUT 'command'
T=$1; shift
rm -f gpurun_out/*.log
for i in 1 2 3; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gr.out 2>&1
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  grep -E "^\[gpurun\] (status|GPU-minutes)" /tmp/gr.out | tail -2
  if [[ "$st" != "transient" ]]; then break; fi
  sleep 20
done
