"""Debug: scan one fixture (or a mixed corpus) and dump the per-sub-tile summaries.
Usage: python tools/dbg_sums.py LIB NAME|corpus:SEED:J [max_rows]"""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from couloydb_amd import DataFile, Scanner  # noqa: E402
from oracle import cly_oracle as co  # noqa: E402
from gpu_util import mixed_corpus  # noqa: E402
lib, name = sys.argv[1], sys.argv[2]
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lo = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if name.startswith("corpus:"):
    _, seed, j = name.split(":")
    data = np.frombuffer(mixed_corpus(int(seed) * 7 + int(j), [40_000, 300_000, 1_500_000][int(j)],
                                      corrupt=(int(seed) % 4 == 3) * (int(j) + 1)), np.uint8).copy()
else:
    data = np.fromfile(os.path.join(ROOT, "tests", "golden", name + ".cly"), dtype=np.uint8)
sc = Scanner(0, lib=lib)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_enable(sc.ctx, 1)
try:
    r = sc.scan([DataFile(data, 7)])
    print("gpu: st=%d end=%d n=%d" % (r.status[0], r.end_offset[0], r.n_records[0]))
except Exception as e:
    print("gpu error", e)
t, st, end = co.scan_file(data, 7)
print("oracle: st=%d end=%d n=%d len=%d" % (st, end, len(t), len(data)))
sz = sc.lib.cly_dbg_sumsize()
st4 = (ctypes.c_uint32 * 4)()
sc.lib.cly_dbg_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
sc.lib.cly_dbg_stats(sc.ctx, st4)
print("redo_units %d redo_subs %d grid %d lds %d" % tuple(st4))
dt = np.dtype([("evt_off", "<i8"), ("evt_gidx", "<u8"), ("p_excl", "<u8"), ("open_pos", "<i8"), ("evt_status", "<i4"),
               ("cnt", "<u4"), ("open_state", "<u4"), ("open_crc", "<u4"), ("head_raw", "<u4"), ("head_shift", "<u4"),
               ("first4", "<u4"), ("head_len", "<u4"), ("flags", "<u4"), ("head_z", "<u4")])
assert dt.itemsize == sz, (dt.itemsize, sz)
buf = np.zeros(rows, dt)
sc.lib.cly_dbg_sums.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_sums(sc.ctx, buf.ctypes.data, rows)
offs = [int(x["offset"]) for x in t]
for i, b in enumerate(buf):
    if i < lo: continue
    print(i, {k: (int(b[k]) if k not in ("open_state", "open_crc", "head_raw", "head_shift", "first4") else hex(int(b[k])))
              for k in dt.names})
ddt = np.dtype([(n, "<i4") for n in "mode E cnt term tst last lterm eof_exit k0 guess bad bpos".split()] + [("tpos", "<i8"), ("xrel", "<i8")])
dbuf = np.zeros(rows, ddt)
sc.lib.cly_dbg_subs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_subs(sc.ctx, dbuf.ctypes.data, rows)
TS = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
import bisect
for i, b in enumerate(dbuf):
    if i < lo: continue
    d = {k: int(b[k]) for k in ddt.names}
    # oracle: first record start >= sub-tile start, records starting in the sub-tile
    s0 = i * TS
    j = bisect.bisect_left(offs, s0)
    oe = (offs[j] - s0) if j < len(offs) else -1
    on = bisect.bisect_left(offs, s0 + TS) - j
    print("sub", i, "E", d["E"], "guess", d["guess"], "cnt", d["cnt"], "mode", d["mode"], "| oracle E", oe, "cnt", on,
          "OK" if (d["mode"] != 1 or (d["E"] == oe and d["cnt"] == on)) else "DIFF")
UNIT = int(sys.argv[6]) if len(sys.argv) > 6 else 2048
nu = (len(data) + UNIT - 1) // UNIT
up = (ctypes.c_uint64 * nu)()
sc.lib.cly_dbg_unitp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_unitp(sc.ctx, up, nu)
for u in range(nu):
    print("unit", u, "P", up[u], "oracle", bisect.bisect_left(offs, u * UNIT))
