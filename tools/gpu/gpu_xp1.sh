#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xp1
timeout -k 10 120 ./tools/xp/${XP:-stream_depth} > gpurun_out/xp1/${XP:-stream_depth}.log 2>&1; rc=$?
cat gpurun_out/xp1/${XP:-stream_depth}.log
exit $rc
