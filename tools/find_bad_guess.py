"""Device diagnostic: run a bench workload with the per-chunk trace on, list
chunks whose speculative guess differed from the true entry, and dump the file
bytes around the first few to gpurun_out/badguess_*.bin for CPU replay."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner, build_info  # noqa: E402

CHUNK = int(build_info().split("CHUNK=")[1].split()[0])
DBG = np.dtype([("entry_g", "<i8"), ("p_excl", "<u8"), ("xrel", "<i8"), ("tpos", "<i8"), ("mode", "<i4"),
                ("guess", "<i4"), ("E", "<i4"), ("cnt", "<i4"), ("term", "<i4"), ("tst", "<i4"),
                ("in_dead", "<i4"), ("k0", "<i4")])
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
wl = make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_enable(sc.ctx, 1)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
n = st.n_chunks
d = np.zeros(n, DBG)
sc.lib.cly_dbg_chunks(sc.ctx, d.ctypes.data, None, n)
ok_normal = (d["mode"] == 0) & (d["guess"] == d["E"])
ok_pass = (d["mode"] == 1) & (d["guess"] < 0)
bad = np.nonzero(~(ok_normal | ok_pass | (d["mode"] == 2)))[0]
print("chunks %d, wrong guesses %d" % (n, len(bad)))
# chunk -> file
nch = [(ln + CHUNK - 1) // CHUNK for (_, ln, _) in wl.dev_files]
starts = np.cumsum([0] + nch)
for k, c in enumerate(bad[:6]):
    f = int(np.searchsorted(starts, c, side="right") - 1)
    cl = int(c - starts[f])
    print("chunk %d (file %d local %d): mode %d guess %d true E %d cnt %d xrel %d" % (
        c, f, cl, d[c]["mode"], d[c]["guess"], d[c]["E"], d[c]["cnt"], d[c]["xrel"]))
    lo = max(0, (cl - 2) * CHUNK)
    hi = min(wl.dev_files[f][1], (cl + 3) * CHUNK)
    b = wl.file_bytes(f)[lo:hi]
    path = os.path.join(ROOT, "gpurun_out", "badguess_%d.bin" % k)
    b.tofile(path)
    print("   dumped file bytes [%d, %d) -> %s (chunk starts at offset %d in the dump)" % (
        lo, hi, os.path.basename(path), cl * CHUNK - lo))
