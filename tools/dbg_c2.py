"""Debug: C2 workload, list sub-tiles whose final entry differs from their guess."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
wl = make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_enable(sc.ctx, 1)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
st4 = (ctypes.c_uint32 * 4)()
sc.lib.cly_dbg_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
sc.lib.cly_dbg_stats(sc.ctx, st4)
print("passes", st.passes, "redo_units %d redo_subs %d grid %d lds %d" % tuple(st4), "scan_ms", st.scan_ms)
ddt = np.dtype([(n, "<i4") for n in "mode E cnt term tst last lterm eof_exit k0 guess bad bpos".split()] + [("tpos", "<i8"), ("xrel", "<i8")])
n = sum((ln + 73727) // 73728 for (_, ln, _) in wl.dev_files) * 8
dbuf = np.zeros(n, ddt)
sc.lib.cly_dbg_subs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_subs(sc.ctx, dbuf.ctypes.data, n)
bad = np.nonzero((dbuf["mode"] == 1) & (dbuf["E"] != dbuf["guess"]))[0]
print("sub-tiles with E != guess:", len(bad))
for i in bad[:20]:
    print(i, "unit", i // 8, {k: int(dbuf[i][k]) for k in ddt.names})
    for j in range(max(0, i - 1), i + 2):
        print("   ", j, {k: int(dbuf[j][k]) for k in ("mode", "E", "guess", "cnt", "xrel")})
