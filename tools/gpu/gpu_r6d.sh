#!/bin/bash
# round 6: the small-record leg (1 GiB of 19-30-B records) with the product
# build, k_scan alone, without compact-entry stores, without any store, and
# with section clocks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6d
mkdir -p $D
for lib in libclyscan.so libexp_base.so libexp_nocomp.so libexp_nostore.so libexp_prof.so; do
  timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_${lib}.log 2>&1 || exit $?
  echo "$lib: $(grep -o "'k_scan_ms': [0-9.]*\|'value': [0-9.]*\|'k_scan': [0-9.]*" $D/small_${lib}.log | tr '\n' ' ')"
  grep "^xp:" $D/small_${lib}.log | tail -2
done
