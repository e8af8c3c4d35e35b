"""Index-load probe: `gen DIR [cfg]` writes a configuration's data files as
%09d.cly into DIR; `open DIR LIB` opens DIR twice with libclyscan LIB in this
process (first / second open) and prints the load stats."""
import os
import sys
import time

sys.path.insert(0, ".")

if sys.argv[1] == "gen":
    import torch
    from bench import make_workload
    d = sys.argv[2]
    wl = make_workload(sys.argv[3] if len(sys.argv) > 3 else "c2", torch)
    os.makedirs(d, exist_ok=True)
    for i, (_, ln, fid) in enumerate(wl.dev_files):
        wl.file_bytes(i).tofile(os.path.join(d, "%09d.cly" % fid))
    print("wrote", len(wl.dev_files), "files", flush=True)
else:
    from couloydb_amd import Scanner
    d, lib = sys.argv[2], sys.argv[3]
    t0 = time.perf_counter()
    sc = Scanner(0, lib=lib)
    print("ctx %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
    for k in range(2):
        t0 = time.perf_counter()
        db = sc.open_db(d)
        w = (time.perf_counter() - t0) * 1e3
        s = db.stats
        print("%s open%d wall %.1f h2d %.1f scan %.1f index %.1f insert %.1f" % (
            lib, k, w, s.h2d_ms, s.scan_ms, s.index_ms, s.insert_ms), flush=True)
        db.close()
