#!/bin/bash
# k_scan with stores vs without (SCAN_ONLY builds), the deferred-snapshot build
# against the baseline (C2, C3, small records), then the open probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/gpu_xpns.sh || exit $?
bash tools/gpu/gpu_ab.sh libclyscan_xbase.so libclyscan_xsnap.so || exit $?
bash tools/gpu/gpu_open2.sh
