"""Debug: scan one fixture (or a mixed corpus) and compare the per-sub-tile
results (descriptor, records before the sub-tile) with the oracle's chain.
Usage: python tools/dbg_sums.py LIB NAME|corpus:SEED:J [rows] [first_row] [sub_tile_bytes]"""
import bisect
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from couloydb_amd import DataFile, Scanner  # noqa: E402
from oracle import cly_oracle as co  # noqa: E402
from gpu_util import mixed_corpus  # noqa: E402

lib, name = sys.argv[1], sys.argv[2]
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lo = int(sys.argv[4]) if len(sys.argv) > 4 else 0
TS = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
if name.startswith("corpus:"):
    _, seed, j = name.split(":")
    data = np.frombuffer(mixed_corpus(int(seed) * 7 + int(j), [40_000, 300_000, 1_500_000][int(j)],
                                      corrupt=(int(seed) % 4 == 3) * (int(j) + 1)), np.uint8).copy()
else:
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", name + ".cly"), dtype=np.uint8)
sc = Scanner(0, lib=lib)
try:
    r = sc.scan([DataFile(data, 7)])
    print("gpu: st=%d end=%d n=%d" % (r.status[0], r.end_offset[0], r.n_records[0]))
except Exception as e:
    print("gpu error", e)
t, st, end = co.scan_file(data, 7)
print("oracle: st=%d end=%d n=%d len=%d" % (st, end, len(t), len(data)))
st4 = (ctypes.c_uint32 * 4)()
sc.lib.cly_dbg_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
sc.lib.cly_dbg_stats(sc.ctx, st4)
print("fixes %d grid %d lds %d" % (st4[0], st4[2], st4[3]))
ddt = np.dtype([("x", "<i8"), ("cnt", "<u4"), ("entry", "<i2"), ("mode", "u1"), ("flags", "u1")])
n = min(rows + lo, (len(data) + TS - 1) // TS or 1)
desc = np.zeros(n, ddt)
sc.lib.cly_dbg_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_descs(sc.ctx, desc.ctypes.data, n)
sp = np.zeros(n, np.uint64)
sc.lib.cly_dbg_subp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_subp(sc.ctx, sp.ctypes.data, n)
sdt = np.dtype([("evt_off", "<i8"), ("evt_gidx", "<u8"), ("open_pos", "<i8"), ("evt_status", "<i4"),
                ("cnt", "<u4"), ("open_state", "<u4"), ("open_crc", "<u4"), ("head_raw", "<u4"), ("head_shift", "<u4"),
                ("first4", "<u4"), ("head_len", "<u4"), ("flags", "<u4"), ("head_z", "<u4")])
assert sdt.itemsize == sc.lib.cly_dbg_sumsize(), (sdt.itemsize, sc.lib.cly_dbg_sumsize())
sums = np.zeros(n, sdt)
sc.lib.cly_dbg_sums.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_sums(sc.ctx, sums.ctypes.data, n)
for i in range(lo, n):
    print("sum %4d" % i, {k: (hex(int(sums[i][k])) if k in ("open_state", "open_crc", "head_raw", "first4") else int(sums[i][k]))
                          for k in sdt.names})
offs = [int(x["offset"]) for x in t]
for i in range(lo, n):
    d = desc[i]
    s0 = i * TS
    j = bisect.bisect_left(offs, s0)
    oe = (offs[j] - s0) if j < len(offs) and offs[j] < s0 + TS else -1
    on = bisect.bisect_left(offs, s0 + TS) - j
    ok = int(sp[i]) == j and (d["mode"] != 1 or (d["entry"] == oe and d["cnt"] == on))
    print("sub %4d mode %d entry %5d cnt %3d flags %d P %6d | oracle entry %5d cnt %3d P %6d %s" % (
        i, d["mode"], d["entry"], d["cnt"], d["flags"], sp[i], oe, on, j, "OK" if ok else "DIFF"))
