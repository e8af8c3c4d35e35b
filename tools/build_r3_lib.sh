#!/bin/bash
# Rebuild couloydb_amd/libclyscan_r3.so (the round-3 library the same-box
# comparisons in tools/gpu/gpu_cmp.sh time beside the current build) from commit
# d15e466, whose product sources hash to e028212b75f3 (cly_build_info).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$ROOT" archive d15e466 couloydb_amd/csrc include | tar -x -C "$T"
make -C "$T/couloydb_amd/csrc" -j4 ../libclyscan.so > /dev/null
cp "$T/couloydb_amd/libclyscan.so" "$ROOT/couloydb_amd/libclyscan_r3.so"
rm -rf "$T"
python3 - "$ROOT" <<'PY'
import ctypes, sys
lib = ctypes.CDLL(sys.argv[1] + "/couloydb_amd/libclyscan_r3.so")
lib.cly_build_info.restype = ctypes.c_char_p
info = lib.cly_build_info().decode()
assert "src=e028212b75f3" in info, info
print(info)
PY
