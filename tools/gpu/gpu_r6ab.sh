#!/bin/bash
# round 6: C3's longest repair walk (tile 523292): LOCALs before repair and final TileIns
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ab
mkdir -p $D
timeout -k 10 300 python -u tools/guess_probe.py c3 523292 > $D/guess_c3.log 2>&1 || exit $?
grep -v "amdgpu.ids" $D/guess_c3.log | tail -14 | cut -c1-400
