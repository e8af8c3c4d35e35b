#!/bin/bash
# round 6, final build: the small-record leg (1 GiB of 19-30-B records) under
# rocprofv3: kernel stats, two SQ passes, FETCH_SIZE and WRITE_SIZE passes
# (tools/pmc_agg.py gpurun_out/r6am small)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6am
mkdir -p $D
export TMPDIR=/tmp
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/small_stats -o run -- python3 tools/small_once.py libclyscan.so > $D/small_stats.log 2>&1 || exit $?
i=0
for s in "$S1" "$S2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d $D/small_p$i -o run -- python3 tools/small_once.py libclyscan.so > $D/small_p$i.log 2>&1 || exit $?
done
echo done
