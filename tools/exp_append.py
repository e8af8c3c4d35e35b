"""The bench's append leg alone (C2 re-appended by cly_append_device), for
rocprofv3 kernel stats: python tools/exp_append.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

wl = bench.make_workload("c2", torch)
with Scanner(0) as sc:
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    print(bench.append_leg(wl, sc, first, torch, reps=5))
