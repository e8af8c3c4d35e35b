"""Debug (GPU box): scan a mixed corpus with CLY_DUMP set and compare every lane's
chain with the oracle's record boundaries.  Usage: dbg_chain.py SEED [lib]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
seed = int(sys.argv[1]); lib = sys.argv[2] if len(sys.argv) > 2 else "libclyscan.so"
CH = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
dump = "/tmp/cly_dump.bin"
if os.path.exists(dump): os.remove(dump)
os.environ["CLY_DUMP"] = dump
from tests.gpu_util import mixed_corpus
from oracle import cly_oracle as co
from couloydb_amd import DataFile, Scanner
files = []
for j in range(3):
    data = mixed_corpus(seed * 7 + j, [40_000, 300_000, 1_500_000][j], corrupt=(seed % 4 == 3) * (j + 1))
    files.append(DataFile(np.frombuffer(data, np.uint8).copy(), 1000 + j))
with Scanner(0, lib=lib) as sc:
    try:
        sc.scan(files)
    except Exception as e:
        print("scan error", e)
d = np.fromfile(dump, np.uint32).reshape(-1, 64, 8)
TILE = 64 * CH
tile0 = 0
for fi, f in enumerate(files):
    t, st, end = co.scan_file(f.data, f.fid)
    offs = [int(x["offset"]) for x in t] if len(t) else []
    bset = sorted(offs) + [int(end)]
    n = len(f.data)
    nt = max(1, (n + TILE - 1) // TILE)
    print("file", fi, "len", n, "records", len(offs), "status", st, "end", end, "tiles", nt)
    bad = 0
    for tt in range(nt):
        for l in range(64):
            cb = tt * TILE + l * CH
            if cb >= n and cb != 0: continue
            ce = min(cb + CH, n); last = cb + CH >= n
            inb = [b for b in bset if (cb <= b < ce) or (last and b == n)]
            mode, E, x, term, cnt, sx, G, ff = [int(v) for v in d[tile0 + tt, l]]; m0 = e0 = m1 = e1 = -1
            dead = cb > end
            exp_mode = 2 if dead else (1 if inb else 0)
            ok = mode == exp_mode and (mode != 1 or (E == inb[0] and cnt == len([b for b in inb if b != end]) ))
            if not ok and bad < 12:
                print("  tile %d lane %d cb %d: got mode %d E %d x %d term %d cnt %d | entry %#x G %d file %d | want mode %d bnds %s | A %d/%d R1 %d/%d" %
                      (tt, l, cb, mode, E, x, term, cnt, sx, G, ff, exp_mode, inb[:6], m0, e0, m1, e1))
                bad += 1
    tile0 += nt
