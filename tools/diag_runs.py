"""Diagnostic (not a product): k_scan's guesses against the final chain on a
workload (argv[1], default c3): per tile the LOCAL k_scan wrote (before any
repair, cly_dbg_set bit 0) and the TileIn the link settled on; counts the
tiles whose first boundary disagrees, split into a run's first tile (guessed)
and the carried ones, and the longest stretch of consecutive disagreeing tiles."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
RUN = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wl = make_workload(cfg, torch)
sc = Scanner(0)
lib = sc.lib
if len(sys.argv) > 3:
    sc.close()
    sc = Scanner(0, lib=sys.argv[3])
    lib = sc.lib
lib.cly_dbg_set.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.cly_dbg_tiles.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
lib.cly_dbg_set(sc.ctx, 3)
import os
import tempfile
errf = tempfile.TemporaryFile()
saved = os.dup(2)
os.dup2(errf.fileno(), 2)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
os.dup2(saved, 2)
errf.seek(0)
elog = errf.read().decode()
print(elog, flush=True)
import re
m = re.findall(r"from tile (\d+)", elog)
print("passes", st.passes, sc.kernel_ms(), flush=True)
TILE = 65536
ntiles = sum((ln + TILE - 1) // TILE for _, ln, _ in wl.dev_files)
loc = np.zeros((ntiles, 4), np.uint64)
tin = np.zeros((ntiles, 8), np.uint32)
lib.cly_dbg_tiles(sc.ctx, loc.ctypes.data, tin.ctypes.data, ntiles)
t0 = 0
bad = np.zeros(ntiles, bool)
kind = np.zeros(ntiles, np.int8)          # 0 file's first, 1 run's first (guessed), 2 carried
for _, ln, _ in wl.dev_files:
    nt = (ln + TILE - 1) // TILE
    for u in range(nt):
        t = t0 + u
        l0, l1, l3 = int(loc[t, 0]), int(loc[t, 1]), int(loc[t, 3])
        X, dead = int(tin[t, 2]), bool(tin[t, 3] & 1)
        kind[t] = 0 if u == 0 else (1 if u % RUN == 0 else 2)
        if u == 0 or dead:
            continue
        if l0 & 4:                                   # DF_NONE
            bad[t] = X < (l3 & 0xFFFFFFFF)
        else:
            bad[t] = X != (l1 & 0xFFFFFFFF)
    t0 += nt
longest, cur = 0, 0
for b in bad:
    cur = cur + 1 if b else 0
    longest = max(longest, cur)
print("tiles", ntiles, "bad", int(bad.sum()), "bad guessed", int((bad & (kind == 1)).sum()),
      "bad carried", int((bad & (kind == 2)).sum()), "longest bad stretch", longest, flush=True)

ws = int(m[-1]) if m else -1
if ws >= 0:
    for t in range(ws - 1, ws + 8):
        l0, l1 = int(loc[t, 0]), int(loc[t, 1])
        print(" tile", t, "kind", kind[t], "k_scan flags", hex(l0 & 0xff), "n", l0 >> 32, "G", hex(l1 & 0xFFFFFFFF),
              "exit", hex(l1 >> 32), "| final entry X", hex(int(tin[t, 2])), "dead", int(tin[t, 3] & 1), flush=True)
listed = np.nonzero(tin[:, 3] & 2)[0]
print("listed in the last round", len(listed), flush=True)
for t in listed[:20]:
    print(" tile", t, "kind", kind[t], "loc", [hex(int(x)) for x in loc[t]], "tin X", hex(int(tin[t, 2])), "dead", tin[t, 3] & 1)
