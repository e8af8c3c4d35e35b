"""Debug: scan every golden fixture with the given libraries, report failures."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import json  # noqa: E402
import numpy as np  # noqa: E402
from couloydb_amd import DataFile, Scanner  # noqa: E402
GOLD = os.path.join(ROOT, "tests", "golden")
GOLDEN = json.load(open(os.path.join(GOLD, "golden.json")))
FIXTURES = sorted(k for k in GOLDEN if not k.startswith("_"))


def fixture_file(name):
    with open(os.path.join(GOLD, name + ".cly"), "rb") as f:
        return DataFile(np.frombuffer(f.read(), np.uint8).copy(), GOLDEN[name]["fid"])
for lib in sys.argv[1].split(","):
    sc = Scanner(0, lib=lib)
    bad = []
    for n in FIXTURES:
        g = GOLDEN[n]
        try:
            r = sc.scan([fixture_file(n)])
            ok = (r.status[0], r.end_offset[0], r.n_records[0]) == (g["status"], g["end_offset"], g["n_records"])
        except Exception as e:
            ok = False
        if not ok:
            bad.append(n)
    print(lib, "fail:", bad, flush=True)

# stored record starts of the first tiles vs the golden offsets
import ctypes  # noqa: E402
for lib, tile_bytes in [("libclyscan.so", 65536), ("libclyscan_small.so", 4096)]:
    sc = Scanner(0, lib=lib)
    for n in sys.argv[2].split(","):
        g = GOLDEN[n]
        try:
            sc.scan([fixture_file(n)])
        except Exception:
            pass
        offs = [t[0] for t in g["tuples"]]
        for t in range(min(4, len(fixture_file(n).data) // tile_bytes + 1)):
            pos = (ctypes.c_uint16 * 2048)()
            loc = (ctypes.c_uint64 * 4)()
            sc.lib.cly_dbg_tile(sc.ctx, t, pos, loc)
            cnt = loc[0] >> 32
            mine = [t * tile_bytes + pos[i] for i in range(min(cnt, 2048))]
            want = [o for o in offs if t * tile_bytes <= o < (t + 1) * tile_bytes]
            print(lib, n, "tile", t, "flags %#x cnt %d" % (loc[0] & 0xff, cnt), "match" if mine == want else "DIFF",
                  "" if mine == want else (mine[:12], want[:12]), flush=True)
