"""Which tiles of a C2 scan did k_scan's entry guess get wrong?  Snapshots the
tile LOCALs before repair (cly_dbg_set bit 0) and compares each tile's guess G
with the true first record start (C2: records of 276 B from offset 0)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
wl = make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_set.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_tiles.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
sc.lib.cly_dbg_set(sc.ctx, 1)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
TILE = 65536
nt = [(ln + TILE - 1) // TILE for _, ln, _ in wl.dev_files]
N = sum(nt)
loc = np.zeros((N, 4), np.uint64)
tin = np.zeros((N, 8), np.uint32)
sc.lib.cly_dbg_tiles(sc.ctx, loc.ctypes.data, tin.ctypes.data, N)
print("passes", st.passes, "need", need, "expect", wl.expect_records, "kms", sc.kernel_ms())
base = 0
bad = 0
for f, (ptr, ln, fid) in enumerate(wl.dev_files):
    out = wl.d_out[first[f] * 48:(first[f] + res[f].n_records) * 48].cpu().numpy().view(np.int64).reshape(-1, 6)
    starts = out[:, 0]
    for tt in range(nt[f]):
        l0, l1 = int(loc[base + tt, 0]), int(loc[base + tt, 1])
        G = l1 & 0xFFFFFFFF
        tb = tt * TILE
        i = np.searchsorted(starts, tb)
        true_g = int(starts[i]) if i < len(starts) else ln
        if tt > 0 and G != true_g and not (l0 & 4):
            bad += 1
            if bad <= 12:
                print("file %d tile %d: G=%d true=%d (rel %d vs %d) flags=%#x cnt=%d X=%d" % (
                    f, tt, G, true_g, G - tb, true_g - tb, l0 & 0xFF, l0 >> 32, l1 >> 32))
    base += nt[f]
print("wrong guesses:", bad, "of", N)
if bad:
    # bytes around the first wrong guess's tile start
    pass
