"""Debug: raw k_scan guesses (no fix rounds) of one bench workload file against
the oracle's record starts.  Usage: python tools/dbg_guess.py [c2|c3] [file] [n]"""
import bisect
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402
from oracle import cly_oracle as co  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
fi = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 20
wl = make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_enable(sc.ctx, 16)
ptr, ln, fid = wl.dev_files[fi]
try:
    sc.scan_device([(ptr, ln, fid)], wl.d_out.data_ptr(), wl.out_cap)
except Exception as e:
    print("scan:", e)
TS = 9216
n = (ln + TS - 1) // TS
ddt = np.dtype([("x", "<i8"), ("cnt", "<u4"), ("entry", "<i2"), ("mode", "u1"), ("flags", "u1")])
desc = np.zeros(n, ddt)
sc.lib.cly_dbg_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
sc.lib.cly_dbg_descs(sc.ctx, desc.ctypes.data, n)
data = wl.file_bytes(fi)
t, st, end = co.scan_file(data, fid)
offs = t["offset"].astype(np.int64)
sizes = t["size"].astype(np.int64)
wrong = 0
for s in range(n):
    s0 = s * TS
    j = bisect.bisect_left(offs, s0)
    if j < len(offs) and offs[j] < s0 + TS:
        tm, te = 1, int(offs[j] - s0)
    else:
        tm, te = 2, 0
    d = desc[s]
    ok = d["mode"] == tm and (tm != 1 or d["entry"] == te)
    if not ok:
        wrong += 1
        if wrong <= nshow:
            # records around
            k = bisect.bisect_right(offs, s0) - 1
            recs = [(int(offs[i] - s0), int(sizes[i])) for i in range(max(k, 0), min(k + 4, len(offs)))]
            print("sub %d: guess mode %d entry %d cnt %d | true mode %d entry %d | records(rel,size) %s" % (
                s, d["mode"], d["entry"], d["cnt"], tm, te, recs))
print("file %d: %d sub-tiles, %d wrong guesses" % (fi, n, wrong))


# ---- emulate the speculation of the first few wrong sub-tiles (kernel logic)
def govarint(b):
    x, s = 0, 0
    for i in range(min(len(b), 11)):
        c = int(b[i])
        if i == 10:
            return 0, -11
        if c < 0x80:
            if i == 9 and c > 1:
                return 0, -10
            ux = x | (c << s)
            v = ux >> 1
            return (~v if ux & 1 else v), i + 1
        x |= (c & 0x7f) << s
        s += 7
    return 0, 0


def hdr(pos):
    m = min(26, ln - pos)
    if m <= 5:
        return False, 0
    b = data[pos:pos + m]
    typ, dt = int(b[4]), int(b[5])
    idx = 6
    ks, na = govarint(b[idx:m]); idx += na
    if idx < 0 or na <= 0:
        return False, 0
    vs, nb = govarint(b[idx:m]); idx += nb
    if nb <= 0:
        return False, 0
    ex, nc = govarint(b[idx:m]); idx += nc
    if nc <= 0:
        return False, 0
    ks32, vs32 = ks & 0xffffffff, vs & 0xffffffff
    good = typ <= 4 and dt <= 4 and ks >= 1 and vs >= 0
    return good, idx + ks32 + vs32


SUB = 144
shown = 0
for s in range(n):
    if shown >= 3:
        break
    s0 = s * TS
    j = bisect.bisect_left(offs, s0)
    tm = 1 if (j < len(offs) and offs[j] < s0 + TS) else 2
    d = desc[s]
    if d["mode"] != 1 or tm != 2:
        continue
    shown += 1
    nrel = ln - s0
    win = min(TS + 320, nrel)
    print("== sub %d guess %d (true PASS)" % (s, d["entry"]))
    for lane in range(64):
        a, b = lane * SUB, min(lane * SUB + SUB, TS)
        fb = None
        res = None
        for q in range(a, b):
            if s0 + q + 6 >= ln:
                break
            if data[s0 + q + 4] > 4 or data[s0 + q + 5] > 4:
                continue
            kb = data[s0 + q + 6]
            if kb == 0 or kb & 1:
                continue
            g, sz = hdr(s0 + q)
            if not g:
                continue
            p, x, ok = q, q + sz, True
            while x < b:
                g2, sz2 = hdr(s0 + x)
                if not g2:
                    ok = False
                    break
                p, x = x, x + sz2
            if not ok or x > nrel:
                continue
            if x < nrel and x + 26 > win:
                if fb is None:
                    fb = (q, x, 0)
                continue
            if x < nrel:
                g3, _ = hdr(s0 + x)
                if not g3:
                    continue
            res = (q, x, 1)
            break
        r = res or fb
        if r:
            q, x, v = r
            dc = None
            if x < nrel:
                g4, sz4 = hdr(s0 + x)
                dc = g4 and (x + sz4 >= nrel and x + sz4 == nrel or (x + sz4 < nrel and hdr(s0 + x + sz4)[0]))
            print("   lane %2d spec q=%d x=%d verified=%d deep_check=%s" % (lane, q, x, v, dc))
