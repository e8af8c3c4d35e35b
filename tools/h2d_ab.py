"""Experiment: the open's H2D modes (CLY_XP_H2D 0 staging, 1 direct from the
mapping, 2 direct after MADV_POPULATE_READ, 3 staging after populate) on the C2
files in /dev/shm, each mode's first and second open in a fresh process."""
import os
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload, index_load_leg  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

os.environ["CLY_XP_H2D"] = sys.argv[1]
wl = make_workload("c2", torch)
sc = Scanner(0)
r = index_load_leg(wl, sc)
print("mode", sys.argv[1], {k: r[k] for k in ("wall_ms", "list_map_ms", "h2d_ms", "scan_ms", "index_ms", "host_insert_ms")},
      r["second_open"], flush=True)
