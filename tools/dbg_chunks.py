"""Per-chunk trace of one scan (debug): python tools/dbg_chunks.py LIB FIXTURE [max_chunks]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from couloydb_amd import DataFile, Scanner  # noqa: E402

DBG = np.dtype([("entry_g", "<i8"), ("p_excl", "<u8"), ("xrel", "<i8"), ("tpos", "<i8"), ("mode", "<i4"),
                ("guess", "<i4"), ("E", "<i4"), ("cnt", "<i4"), ("term", "<i4"), ("tst", "<i4"),
                ("in_dead", "<i4"), ("k0", "<i4")])
SUM = np.dtype([("evt_off", "<i8"), ("evt_gidx", "<u8"), ("p_excl", "<u8"), ("open_pos", "<i8"),
                ("evt_status", "<i4"), ("cnt", "<u4"), ("open_state", "<u4"), ("open_crc", "<u4"),
                ("head_raw", "<u4"), ("head_shift", "<u4"), ("first4", "<u4"), ("head_len", "<u4"),
                ("flags", "<u4"), ("_pad", "<u4")])
lib, fx = sys.argv[1], sys.argv[2]
mx = int(sys.argv[3]) if len(sys.argv) > 3 else 64
sc = Scanner(0, lib=lib)
L = sc.lib
L.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.cly_dbg_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
L.cly_dbg_sizes.argtypes = [ctypes.c_void_p]
sizes = (ctypes.c_int * 3)()
sc.lib.cly_dbg_sizes(sizes)
assert sizes[0] == DBG.itemsize and sizes[1] == SUM.itemsize, list(sizes)
sc.lib.cly_dbg_enable(sc.ctx, int(os.environ.get("CLY_DBG", "1")))
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
data = np.fromfile(os.path.join(ROOT, "tests", "golden", fx + ".cly"), dtype=np.uint8)
import threading
def dump_trace():
    if hasattr(L, "cly_dbg_trace"):
        L.cly_dbg_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        NL = int(os.environ.get("CLY_NT", "64"))
        tr = (ctypes.c_int * (2048 + 4 * NL * 8))()
        L.cly_dbg_trace(sc.ctx, tr, 2048 + 4 * NL * 8)
        print("trace (mark, chunk):", [(tr[2 * i], tr[2 * i + 1]) for i in range(8)], flush=True)
        for t in range(int(os.environ.get("CLY_LANES", "0"))):
            o = tr[2048 + t * 8: 2048 + t * 8 + 8]
            print("  lane %3d sp_s=%d sp_x=%d sp_cnt=%d ws=%d wx=%d wc=%d pk=%d base=%d wterm=%d fail_k=%d" % (
                t, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7] & 0xffff, (o[7] >> 16) & 15, o[7] >> 20), flush=True)
t = threading.Timer(10.0, dump_trace)
t.daemon = True
t.start()
try:
    r = sc.scan([DataFile(data, gold[fx]["fid"])])
    print("result st=%d end=%d n=%d | gold st=%d end=%d n=%d" % (r.status[0], r.end_offset[0], r.n_records[0],
          gold[fx]["status"], gold[fx]["end_offset"], gold[fx]["n_records"]))
except Exception as e:
    print("scan error:", e)
t.cancel()
dump_trace()
if hasattr(L, "cly_dbg_fout"):
    L.cly_dbg_fout.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    fo = np.zeros(1, np.dtype([("n", "<u8"), ("end", "<i8"), ("st", "<i4"), ("ok", "<i4"), ("first", "<u8")]))
    L.cly_dbg_fout(sc.ctx, fo.ctypes.data, 1)
    print("fout:", fo)
d = np.zeros(mx, DBG)
s = np.zeros(mx, SUM)
n = sc.lib.cly_dbg_chunks(sc.ctx, d.ctypes.data, s.ctypes.data, mx)
only = os.environ.get("CLY_DBG_ONLY")
for i in range(n):
    if only and not (d[i]["mode"] != 1 or d[i]["entry_g"] < i * 0 ):
        pass
    print(i, {k: int(d[i][k]) for k in DBG.names})
    print("  ", {k: int(s[i][k]) for k in SUM.names if k != "_pad"})
