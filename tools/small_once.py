"""Experiment target: bench.py's small-record leg (1 GiB of 19-30-B records,
one file) with libclyscan build argv[1]; prints the leg's line.  argv[2]:
cly_dbg_set flags (2: print each host repair round)."""
import ctypes
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import small_records_leg  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else "libclyscan.so"
sc = Scanner(0, lib=lib)
sc.lib.cly_dbg_set(sc.ctx, 4 | (int(sys.argv[2]) if len(sys.argv) > 2 else 0))   # per-kernel markers
print(lib, small_records_leg(sc, torch), sc.kernel_ms(), flush=True)
