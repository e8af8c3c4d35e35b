"""Guess probe: one scan of a bench workload (argv[1], default c3) keeping the
LOCALs before any repair (cly_dbg_set bit 0); lists the run-start tiles whose
guessed entry differs from the true one (the final TileIn), with the bytes at
the guess and at the true entry."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402
from bench import make_workload  # noqa: E402
from couloydb_amd import Scanner  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
TILE, PART = 65536, 32768 * 65536
FOCUS = int(sys.argv[2]) if len(sys.argv) > 2 else -100    # a global tile index to show (e.g. the longest walk's)
class _Small:
    pass


def small_workload():
    """bench.small_records_leg's file (1 GiB of 19-30-B records), kept in HBM"""
    from couloydb_amd import _abi
    gen = _abi.load_gen_lib()
    seed = 0x434C59 + 7
    rng = np.random.default_rng(seed)
    n = int((1 << 30) / 24.5)
    recs = np.zeros(n, dtype=_abi.GEN_DTYPE)
    recs["value_len"] = rng.integers(0, 12, n)
    recs["key_index"] = np.arange(n, dtype=np.int64) % 1_000_000_000
    recs["type"] = (rng.random(n) < 0.25).astype(np.uint8)
    recs["value_len"][recs["type"] == 1] = 0
    fo = (ctypes.c_uint64 * 4)()
    fl = (ctypes.c_uint64 * 4)()
    nf = ctypes.c_uint32()
    total = gen.cly_gen_layout(recs.ctypes.data, n, 1 << 62, 4096, fo, fl, 4, ctypes.byref(nf))
    w = _Small()
    w.d_buf = torch.empty(int(total) + 4096, dtype=torch.uint8, device="cuda")
    d_recs = torch.from_numpy(recs.view(np.uint8)).to("cuda")
    gen.cly_gen_encode(ctypes.c_void_p(w.d_buf.data_ptr()), ctypes.c_void_p(d_recs.data_ptr()), n, seed)
    w.dev_files = [(w.d_buf.data_ptr() + int(fo[0]), int(fl[0]), 1)]
    w.file_off = [int(fo[0])]
    w.out_cap = n + 1024
    w.d_out = torch.empty(w.out_cap * 48, dtype=torch.uint8, device="cuda")
    return w


wl = small_workload() if cfg == "small" else make_workload(cfg, torch)
sc = Scanner(0)
sc.lib.cly_dbg_set(sc.ctx, 3)
first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
nt = [max(1, (ln + TILE - 1) // TILE) for _, ln, _ in wl.dev_files]
ntiles = sum(nt)
loc = np.zeros((ntiles, 4), np.uint64)
tin = np.zeros((ntiles, 8), np.uint32)
sc.lib.cly_dbg_tiles(sc.ctx, ctypes.c_void_p(loc.ctypes.data), ctypes.c_void_p(tin.ctypes.data), ctypes.c_int64(ntiles))
rt = 4
wrong, shown, t0 = 0, 0, 0
kinds = {}
for f, (ptr, ln, fid) in enumerate(wl.dev_files):
    fo = wl.file_off[f]
    for u in range(0, nt[f], rt):
        if u == 0:
            continue
        t = t0 + u
        l0, l1 = int(loc[t, 0]), int(loc[t, 1])
        dead = tin[t, 3] & 1
        X = int(tin[t, 2]) | ((int(tin[t, 7]) & 0xFFFF) << 32)
        x0 = (u // 32768) * PART
        ts = u * TILE
        none = (l0 & 4) != 0
        G = x0 + (l1 & 0xFFFFFFFF)
        if dead:
            continue
        true_in = X < ts + TILE
        if none and not true_in:
            continue
        if not none and G == X:
            continue
        wrong += 1
        k = "none-but-start" if none else ("guess-after-true" if G > X else "guess-before-true")
        kinds[k] = kinds.get(k, 0) + 1
        if shown < 12 or abs(t - FOCUS) <= 4:
            shown += 1
            gb = wl.d_buf[fo + G: fo + G + 16].cpu().numpy().tobytes().hex() if not none else "-"
            xb = wl.d_buf[fo + X: fo + X + 16].cpu().numpy().tobytes().hex() if true_in else "-"
            print("file %d tile %d: %s guess %s (+%d) true %d (+%d) | guess bytes %s | true bytes %s" % (
                f, u, k, "NONE" if none else str(G), (G - ts) if not none else -1, X, X - ts, gb, xb), flush=True)
    t0 += nt[f]
if FOCUS >= 0:
    for t in range(FOCUS - 1, FOCUS + 5):
        print("tile %d LOCAL %s TileIn %s" % (t, [hex(int(v)) for v in loc[t]], [hex(int(v)) for v in tin[t]]), flush=True)
print(cfg, "passes", st.passes, "wrong run-start guesses", wrong, kinds, flush=True)
