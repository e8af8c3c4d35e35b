"""Index-load experiment: the C2 files written to /dev/shm once, then
cly_db_open under each CLY_H2D_MODE / CLY_LOAD_OVERLAP setting (2 opens each)."""
import os
import shutil
import sys
import tempfile

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

wl = make_workload("c2", torch)
sc = Scanner(0)
d = tempfile.mkdtemp(prefix="clyload_", dir="/dev/shm")
try:
    for i, (_, ln, fid) in enumerate(wl.dev_files):
        wl.file_bytes(i).tofile(os.path.join(d, "%09d.cly" % fid))
    for mode in ("0", "1", "2"):
        for ov in ("0", "1"):
            os.environ["CLY_H2D_MODE"], os.environ["CLY_LOAD_OVERLAP"] = mode, ov
            for rep in range(2):
                db = sc.open_db(d)
                s = db.stats
                print("h2d_mode", mode, "overlap", ov, "rep", rep, "wall %.1f h2d %.1f scan %.1f index %.1f insert %.1f keys %d" % (
                    s.total_ms, s.h2d_ms, s.scan_ms, s.index_ms, s.insert_ms, s.str_keys), flush=True)
                db.close()
finally:
    shutil.rmtree(d, ignore_errors=True)
