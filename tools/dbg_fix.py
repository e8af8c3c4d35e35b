"""Debug: trace the link / fix rounds of one scan (cly_dbg_enable flag 4).
Usage: python tools/dbg_fix.py [LIB] [corpus:SEED | c1 | c2 | c3] [--force]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from couloydb_amd import DataFile, Scanner  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
lib = args[0] if args else "libclyscan_small.so"
what = args[1] if len(args) > 1 else "corpus:0"
if not what.startswith("corpus:") and what != "tiny":
    import torch
    from bench import make_workload
    wl = make_workload(what, torch)
sc = Scanner(0, lib=lib)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_enable(sc.ctx, 4 | (8 if "--descs" in sys.argv else 0) | (2 if "--force" in sys.argv else 0))
if what == "tiny":
    from gpu_util import fixed_records_file
    data = fixed_records_file(200000, 0, seed=13)
    try:
        r = sc.scan([DataFile(data, 0)])
        print("ok", r.n_records[0])
    except Exception as e:
        print("ERR", e)
elif what.startswith("corpus:"):
    from gpu_util import mixed_corpus
    seed = int(what.split(":")[1])
    files = []
    for j in range(3):
        data = mixed_corpus(seed * 7 + j, [40_000, 300_000, 1_500_000][j], corrupt=(seed % 4 == 3) * (j + 1))
        files.append(DataFile(np.frombuffer(data, np.uint8).copy(), 1000 + j))
    try:
        sc.scan(files)
    except Exception as e:
        print("ERR", e)
else:
    for it in range(2):
        first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        print("iter %d: scan %.3f ms resolve %.3f ms passes %d" % (it, st.scan_ms, st.resolve_ms, st.passes), flush=True)
