#!/usr/bin/env python3
"""Benchmark: device-resident CouloyDB log-record scan (decode + CRC -> index tuples).

Contract (see task spec): `python bench.py --gpus N --steps K --warmup W` prints ONE
JSON line on rank 0.  A step = one full scan (k_scan, k_link, k_emit,
k_fin and the result read-back) of the configuration's data files, already resident in HBM.  For N>1
each rank (one per GPU) scans its own fid range of the same per-GPU size
(weak scaling, no collective on the data path; the barrier and the
max-over-ranks timing use torch.distributed).  Ranks: either an outer
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
(WORLD_SIZE must equal --gpus), or plain `python bench.py --gpus N`, which
starts the N ranks itself (a torch.distributed.run child, 127.0.0.1) before any
GPU call and exits with their status.

Workloads (BASELINE.json configs):
  c2 (default): 16 files x 256 MiB, key 0x00||%09d, 256-B random values -> 276-B records
  c1: one 64 MiB file of 1 KiB values (CPU plumbing config; also runnable here)
  c3: 32 GiB, Zipf(1.1) value lengths 64 B-64 KiB
  c5: BASELINE config 5's per-GPU share: 32 GiB of the C2/C3 mix (one fid range
      per rank; 8 ranks = 256 GiB)
  c4: merge.go path, 32 GiB: keys 0..K-1 put, then k%4==0 overwritten and
      k%4==2 deleted (50 % of the records dead); a step = scan + merge rewrite
      (live filter, NO_TX_ID re-encode + CRC, file rotation, hint records)
Data is synthetic (splitmix64 values), written on the GPU by libclygen.so, a
restatement of EncodeLogRecord + appendLogRecord's file rotation.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident log-record decode+CRC; Mrecords/s; index-load wall time"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
DATA_FILE_SIZE = 256 << 20   # options.go:32


class Workload:
    pass


def _zipf_lengths(n, rng, s=1.1, nmax=65473):
    ranks = np.arange(1, nmax + 1, dtype=np.float64)
    w = ranks ** (-s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    r = np.searchsorted(cdf, rng.random(n)) + 1
    return (63 + r).astype(np.uint32)


def make_workload(name, torch, rank=0, device=0, seed=0x434C59, size=32 * 2**30):
    """Build the config's data files in HBM on `device`.  Returns a Workload with
    dev_files [(ptr, len, fid)], d_buf, d_out (uint8 tensor), out_cap, expect_records."""
    from couloydb_amd import _abi
    gen = _abi.load_gen_lib()
    if name == "c2":
        nrec_file = DATA_FILE_SIZE // 276
        nfiles_target = 16
        vl = np.full(nrec_file * nfiles_target, 256, np.uint32)
    elif name == "c1":
        nfiles_target = 1
        vl = np.full(64280, 1024, np.uint32)
    elif name == "c3":
        rng = np.random.default_rng(seed + 3)
        nfiles_target = 128
        # enough draws for 32 GiB, cut where the records fill 128 files of
        # DataFileSize (each file loses less than one record to the rotation)
        vl = _zipf_lengths(int(size / 2000), rng)
        cum = np.cumsum(vl.astype(np.int64) + 20)
        vl = vl[: int(np.searchsorted(cum, size - nfiles_target * 40000))]
    elif name == "c5":
        # BASELINE config 5 per GPU: a 32-GiB fid range of the C2/C3 mix (16 GiB of
        # 256-B values, then 16 GiB of Zipf value sizes); 8 GPUs -> 256 GiB
        rng = np.random.default_rng(seed + 5)
        nfiles_target = 128
        half = size // 2
        n2 = int(half // 276)
        vz = _zipf_lengths(int(half / 2000), rng)
        cum = np.cumsum(vz.astype(np.int64) + 20)
        vz = vz[: int(np.searchsorted(cum, half - 64 * 40000))]
        vl = np.concatenate([np.full(n2, 256, np.uint32), vz])
    elif name == "c4":
        nfiles_target = 128
        K = int(size / (276 + 276 / 4 + 19 / 4))
        K -= K % 4
        ph2 = np.arange(0, K, 2, dtype=np.int64)             # k%4==0 put, k%4==2 Del
        keys = np.concatenate([np.arange(K, dtype=np.int64), ph2])
        vl = np.concatenate([np.full(K, 256, np.uint32), np.where(ph2 % 4 == 0, 256, 0).astype(np.uint32)])
        typ = np.concatenate([np.zeros(K, np.uint8), np.where(ph2 % 4 == 0, 0, 1).astype(np.uint8)])
        live = np.concatenate([(np.arange(K) % 2 == 1), ph2 % 4 == 0]).astype(np.uint8)
    else:
        raise ValueError(name)
    n = len(vl)
    recs = np.zeros(n, dtype=_abi.GEN_DTYPE)
    recs["value_len"] = vl
    if name == "c4":
        recs["key_index"] = (keys + rank * K) % 1_000_000_000
        recs["type"] = typ
    else:
        recs["key_index"] = (np.arange(n, dtype=np.int64) + rank * n) % 1_000_000_000
    maxf = 4096
    fo = (ctypes.c_uint64 * maxf)()
    fl = (ctypes.c_uint64 * maxf)()
    nf = ctypes.c_uint32()
    limit = DATA_FILE_SIZE if name != "c1" else 64 << 20
    total = gen.cly_gen_layout(recs.ctypes.data, n, limit, 4096, fo, fl, maxf, ctypes.byref(nf))
    dev = torch.device("cuda", device)
    d_buf = torch.empty(int(total) + 4096, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
    base_dst = 0
    rc = gen.cly_gen_encode(ctypes.c_void_p(d_buf.data_ptr() + base_dst), ctypes.c_void_p(d_recs.data_ptr()), n,
                            seed + rank)
    if rc != 0:
        raise RuntimeError("cly_gen_encode failed: %d" % rc)
    del d_recs
    wl = Workload()
    wl.name = name
    wl.d_buf = d_buf
    wl.dev_files = [(d_buf.data_ptr() + fo[i], int(fl[i]), rank * maxf + i) for i in range(nf.value)]
    wl.file_off = [int(fo[i]) for i in range(nf.value)]
    wl.bytes = int(sum(fl[i] for i in range(nf.value)))
    wl.expect_records = n
    wl.out_cap = n + 1024
    if name == "c4":
        wl.live_np = live
        wl.live = torch.from_numpy(live).to(dev)
        wl.n_live = int(live.sum())
        live_bytes = int((recs["value_len"][live != 0].astype(np.int64) + 20).sum())
        wl.merge_max_files = live_bytes // (DATA_FILE_SIZE - 65536) + 4
        wl.d_merge = torch.empty(wl.merge_max_files * DATA_FILE_SIZE, dtype=torch.uint8, device=dev)
        wl.hint_cap = wl.n_live * 40 + 4096
        wl.d_hint = torch.empty(wl.hint_cap, dtype=torch.uint8, device=dev)
    wl.d_out = torch.empty(wl.out_cap * 48, dtype=torch.uint8, device=dev)

    def file_bytes(i):
        o, ln = wl.file_off[i], wl.dev_files[i][1]
        return wl.d_buf[o:o + ln].cpu().numpy()
    wl.file_bytes = file_bytes
    torch.cuda.synchronize(dev)
    return wl


def measured_traffic(config):
    """k_scan HBM bytes per launch (read + write) from the newest committed
    profiles/*_traffic.json whose build and config match this library."""
    import glob
    from couloydb_amd import build_info
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            t = json.load(open(f))
        except ValueError:
            continue
        k = t.get("kernels", {}).get("k_scan")
        if t.get("build") == build_info() and t.get("config") == config and k:
            best = k.get("fetch_bytes", 0) + k.get("write_bytes", 0)
    return best


MT_THREADS = 16                 # the GPU box's CPU share per GPU


def cpu_baseline(wl, budget_s=12.0):
    """Oracle (C restatement) on the host cores over a bounded sample of the same
    workload: 'ref-algorithm' single thread over whole files; 'ref-faithful' =
    the reference's per-record fstat+mmap/munmap pattern over a bounded record
    count of one file."""
    from oracle import cly_oracle as co
    files, t_alg, nbytes, nrec = [], 0.0, 0, 0
    i = 0
    while i < len(wl.dev_files) and t_alg < budget_s * 0.6:
        arr = wl.file_bytes(i)
        t0 = time.perf_counter()
        r = co.scan_files_mt([arr], [wl.dev_files[i][2]], 1)
        t_alg += time.perf_counter() - t0
        nbytes += len(arr)
        nrec += int(r)
        files.append(i)
        i += 1
    alg_gibs = nbytes / t_alg / 2**30
    # the same restatement with the files spread over MT_THREADS threads (the
    # box's CPU share), over ALL the configuration's files: groups of
    # MT_THREADS files (one file per thread), only the scans timed
    t_mt, mt_rec, mt_bytes = 0.0, 0, 0
    nf_all = len(wl.dev_files)
    for g0 in range(0, nf_all, MT_THREADS):
        grp = list(range(g0, min(g0 + MT_THREADS, nf_all)))
        arrs = [wl.file_bytes(i) for i in grp]
        t0 = time.perf_counter()
        mt_rec += int(co.scan_files_mt(arrs, [wl.dev_files[i][2] for i in grp], MT_THREADS))
        t_mt += time.perf_counter() - t0
        mt_bytes += sum(len(a) for a in arrs)
        del arrs
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    multi = {"value": round(mt_bytes / t_mt / 2**30, 4), "unit": "GiB/s", "cores": MT_THREADS,
             "cores_note": "the GPU box's CPU share per GPU (OMP_NUM_THREADS/MAX_JOBS are 16 there; nproc and "
                           "the affinity mask report the whole host, %s CPUs)" % affinity,
             "mrecords_per_s": round(mt_rec / t_mt / 1e6, 3),
             "sample": "all %d files (%.2f GiB) in groups of %d, one file per thread, %d threads, clyo_scan_files_mt" % (
                 nf_all, mt_bytes / 2**30, MT_THREADS, MT_THREADS)}
    merge_part = None
    if wl.name == "c4":
        # scan + merge rewrite of the sampled files (file i's live bytes follow the
        # scan order of the records before it)
        t_m, mb, first_rec = 0.0, 0, 0
        for i in range(min(len(files), 4)):
            arr = wl.file_bytes(i)
            t0 = time.perf_counter()
            tt, _, _ = co.scan_file(arr, wl.dev_files[i][2])
            rc, _, _, r = co.merge([arr], tt, np.zeros(len(tt), np.uint32), wl.live_np[first_rec:first_rec + len(tt)],
                                   DATA_FILE_SIZE)
            t_m += time.perf_counter() - t0
            first_rec += len(tt)
            mb += len(arr)
        merge_part = {"value": round(mb / t_m / 2**30, 4), "unit": "GiB/s",
                      "sample": "%d files: oracle scan + clyo_merge (merge.go:90-143 restated), 1 thread" % min(len(files), 4)}
    index_part = None
    if wl.name == "c2":
        # db.loadIndex (String index, tx buffering, TTL pass) over all of the
        # configuration's files in memory, one thread as the reference: the CPU
        # side of index_load_wall_ms
        arrs = [wl.file_bytes(i) for i in range(len(wl.dev_files))]
        t0 = time.perf_counter()
        rc, lr = co.load_index(arrs, [f for _, _, f in wl.dev_files], time.time_ns())
        t_li = time.perf_counter() - t0
        index_part = {"wall_ms": round(t_li * 1e3, 1), "rc": rc, "records": int(lr.records),
                      "str_keys": int(lr.str_keys), "cores": 1,
                      "sample": "all %d files (%.2f GiB) in memory; oracle clyo_load_index (db.go:487-651 String/"
                                "ListMeta restated, open-addressing tables keyed into the file bytes)"
                                % (len(arrs), sum(len(a) for a in arrs) / 2**30)}
        del arrs
    # ref-faithful on a bounded number of records of file 0
    arr = wl.file_bytes(0)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "000000000.cly")
        arr.tofile(p)
        t0 = time.perf_counter()
        nf, st, end = co.scan_path_faithful(p, 0, 20000)
        tf = time.perf_counter() - t0
    faithful_gibs = end / tf / 2**30
    return {"value": round(alg_gibs, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": "%d of %d files (%.2f GiB, %d records) scanned by oracle/cly_oracle.c clyo_scan_files_mt, 1 thread"
                      % (len(files), len(wl.dev_files), nbytes / 2**30, nrec),
            "mrecords_per_s": round(nrec / t_alg / 1e6, 3),
            "ref_faithful": {"value": round(faithful_gibs, 5), "unit": "GiB/s",
                             "mrecords_per_s": round(nf / tf / 1e6, 4),
                             "sample": "first %d records of one file; per record fstat + 2x (open, mmap whole file, copy, munmap)" % nf},
            "host_nproc": os.cpu_count(),
            **({"index_load": index_part} if index_part else {}),
            "multi_thread": multi,
            **({"value": merge_part["value"], "sample": merge_part["sample"], "scan_only_value": round(alg_gibs, 4)}
               if merge_part else {})}


def host_path(wl, sc, max_files=16):
    """End-to-end rate of the host-memory entry cly_scan (the cgo path: mmap'd
    files in, index tuples out): H2D of the file bytes, the scan, D2H of the
    tuples.  Bounded to the first `max_files` files of the workload; pageable
    buffers (what an mmap hands over) and page-locked buffers."""
    import torch
    from couloydb_amd import TUPLE_DTYPE, _abi
    n = min(max_files, len(wl.dev_files))
    pageable = [np.ascontiguousarray(wl.file_bytes(i)) for i in range(n)]
    out_rec = {}
    for kind in ("pageable", "pinned"):
        bufs = pageable if kind == "pageable" else [torch.from_numpy(a).pin_memory().numpy() for a in pageable]
        arr = (_abi.ClyFile * n)()
        for i, a in enumerate(bufs):
            arr[i].base, arr[i].len, arr[i].fid = a.ctypes.data, len(a), wl.dev_files[i][2]
        cap = sum(len(a) for a in bufs) // 200 + 1024 if wl.name == "c2" else wl.expect_records + 1024
        out = np.empty(cap, dtype=TUPLE_DTYPE)
        first = (ctypes.c_uint64 * n)()
        res = (_abi.ClyFileResult * n)()
        need = ctypes.c_uint64()
        st = _abi.ClyStats()
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            rc = sc.lib.cly_scan(sc.ctx, arr, n, out.ctypes.data, cap, first, res, ctypes.byref(need), ctypes.byref(st))
            times.append(time.perf_counter() - t0)
            if rc != 0:
                return {"error": rc}
        nbytes = sum(len(a) for a in bufs)
        t = min(times[1:])
        out_rec[kind] = {"value": round(nbytes / t / 2**30, 3), "unit": "GiB/s", "ms": round(t * 1e3, 2),
                         "records": int(need.value), "tuple_bytes_d2h": int(need.value) * 48}
        del bufs
    out_rec["sample"] = "%d files, %.2f GiB; cly_scan (H2D + scan + D2H of the tuples), best of 2 after 1 warm-up" % (
        n, sum(len(a) for a in pageable) / 2**30)
    return out_rec


def index_load_leg(wl, sc):
    """NewCouloyDB's index load from files on disk through the device
    (cly_db_open, include/clyload.h): the configuration's files written as
    `%09d.cly` to a temporary directory, then list + mmap, H2D, scan, index
    rebuild on the device, and the host String-index inserts (timed apart)."""
    d = tempfile.mkdtemp(prefix="clyload_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        for i, (_, ln, fid) in enumerate(wl.dev_files):
            wl.file_bytes(i).tofile(os.path.join(d, "%09d.cly" % fid))
        # the application's start-up step (cly_load_prepare: page-locked staging),
        # outside the timed open, as before round 6 when contexts allocated it
        t0 = time.perf_counter()
        prep_rc = sc.prepare_load()
        prep_ms = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        db = sc.open_db(d)
        wall = (time.perf_counter() - t0) * 1e3
        s = db.stats
        # a second open in the same process (page-locked staging allocated, files
        # in the page cache): the steady state of an open, reported beside
        db.close()
        t0 = time.perf_counter()
        db2 = sc.open_db(d)
        wall2 = (time.perf_counter() - t0) * 1e3
        s2 = db2.stats
        db2.close()
        out = {"wall_ms": round(wall, 2), "list_map_ms": round(s.list_map_ms, 2), "h2d_ms": round(s.h2d_ms, 2),
               "scan_ms": round(s.scan_ms, 2), "index_ms": round(s.index_ms, 2),
               "host_insert_ms": round(s.insert_ms, 2), "files": int(s.n_files), "records": int(s.records),
               "string_keys": int(s.str_keys),
               "device_part_ms": round(s.h2d_ms + s.scan_ms + s.index_ms, 2),
               "prepare_ms": round(prep_ms, 2), "prepare_rc": prep_rc,
               "second_open": {"wall_ms": round(wall2, 2), "h2d_ms": round(s2.h2d_ms, 2),
                               "index_ms": round(s2.index_ms, 2), "host_insert_ms": round(s2.insert_ms, 2)},
               "sample": "%d files (%.2f GiB) in %s; host index = hash-sharded open-addressing tables, 16 threads" % (
                   s.n_files, s.bytes / 2**30, os.path.dirname(d))}
        return out
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)


def _record_bytes(key, value):
    """One NORMAL String LogRecord without expiration (EncodeLogRecord,
    data/logRecord.go:55-84): crc32 IEEE over the header's type/dataType and the
    three zig-zag varints, the key and the value."""
    import zlib

    def varint(x):
        ux, out = x << 1, bytearray()
        while ux >= 0x80:
            out.append((ux & 0x7F) | 0x80)
            ux >>= 7
        out.append(ux)
        return bytes(out)
    body = bytes([0, 0]) + varint(len(key)) + varint(len(value)) + varint(0) + key + value
    return (zlib.crc32(body) & 0xFFFFFFFF).to_bytes(4, "little") + body


def post_merge_open_leg(wl, sc, torch, lens, hint_bytes, n_live):
    """NewCouloyDB after a merge (db.go:442-485, merge.go:182-287): the C4
    merge's output files `%09d.cly` (fids 0..k-1), its hint-index and a
    merge-finished record naming the first fid the merge did not cover (the
    old files' count: every later write would go there) in a /dev/shm
    directory, as loadMergeFiles leaves it; then cly_db_open: the hint preload
    (every live key's String Put from the hint file) and the scan of the data
    files, index rebuild, host inserts.  Timed first and second open."""
    import shutil
    d = tempfile.mkdtemp(prefix="clymerged_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        for k, ln in enumerate(lens):
            base = k * DATA_FILE_SIZE
            wl.d_merge[base:base + ln].cpu().numpy().tofile(os.path.join(d, "%09d.cly" % k))
        wl.d_hint[:hint_bytes].cpu().numpy().tofile(os.path.join(d, "hint-index"))
        with open(os.path.join(d, "merge-finished"), "wb") as f:
            f.write(_record_bytes(b"\x07", str(len(wl.dev_files)).encode()))   # MergeFinishedKey, merge.go:154-168
        walls, stats = [], []
        for _ in range(2):
            t0 = time.perf_counter()
            db = sc.open_db(d)
            walls.append((time.perf_counter() - t0) * 1e3)
            stats.append(db.stats)
            db.close()
        s = stats[0]
        nbytes = int(sum(lens)) + hint_bytes
        return {"wall_ms": round(walls[0], 2), "second_open_wall_ms": round(walls[1], 2),
                "h2d_ms": round(s.h2d_ms, 2), "scan_ms": round(s.scan_ms, 2), "index_ms": round(s.index_ms, 2),
                "host_insert_ms": round(s.insert_ms, 2), "list_map_ms": round(s.list_map_ms, 2),
                "files": int(s.n_files), "bytes": nbytes, "records": int(s.records),
                "hint_records": int(s.hint_records), "string_keys": int(s.str_keys),
                "gib_per_s_second_open": round(nbytes / (walls[1] / 1e3) / 2**30, 2),
                "ok": bool(int(s.hint_records) == n_live and int(s.str_keys) == n_live),
                "sample": "%d merged files + hint-index (%.2f GiB) + merge-finished in %s" % (
                    len(lens), nbytes / 2**30, os.path.dirname(d))}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def c5_leg(sc, torch, device, steps=5):
    """BASELINE config 5 on one GPU: one rank's 32-GiB fid range of the C2/C3
    mix, the same step as the --gpus N > 1 lines time (their per-GPU share), so
    that the driver's 1/2/4/8-GPU lines have a c5 reference at N = 1."""
    wl = make_workload("c5", torch, rank=0, device=device)
    best, kscan, need, res = timed_scans(sc, wl.dev_files, wl.d_out.data_ptr(), wl.out_cap, reps=steps)
    out = {"workload": "c5", "bytes": wl.bytes, "files": len(wl.dev_files), "records": int(need),
           "value": round(wl.bytes / best / 2**30, 2), "unit": "GiB/s", "ms": round(best * 1e3, 3),
           "k_scan_ms": round(kscan, 3), "k_scan_frac": round(wl.bytes / (kscan / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
           "ok": bool(need == wl.expect_records and all(r.status == 0 for r in res)),
           "note": "best of %d device-resident scans (the N>1 lines' per-rank step)" % steps}
    del wl
    torch.cuda.empty_cache()
    return out


def timed_scans(sc, files, d_out, cap, reps=5):
    """reps device-resident scans of files (after one untimed): best wall time
    per scan, the k_scan time, the record count and the statuses."""
    import torch
    sc.scan_device(files, d_out, cap)
    best, kscan, need, res = None, None, 0, None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        first, res, st, need = sc.scan_device(files, d_out, cap)
        dt = time.perf_counter() - t0
        if best is None or dt < best:
            best, kscan = dt, sc.kernel_ms()["k_scan"]
    return best, kscan, need, res


def small_records_leg(sc, torch, nbytes=1 << 30, seed=0x434C59 + 7):
    """One device-resident data file of 19-30-B records (0x00||%09d keys,
    values of 0-11 B, a quarter of them tombstones): every 64-KiB tile holds
    more than CAP_T records, the spill-chunk path (ReadLogRecord's loop over
    commit markers / short KVs, data/dataFile.go:64-111)."""
    from couloydb_amd import _abi
    gen = _abi.load_gen_lib()
    rng = np.random.default_rng(seed)
    n = int(nbytes / 24.5)
    recs = np.zeros(n, dtype=_abi.GEN_DTYPE)
    recs["value_len"] = rng.integers(0, 12, n)
    recs["key_index"] = np.arange(n, dtype=np.int64) % 1_000_000_000
    recs["type"] = (rng.random(n) < 0.25).astype(np.uint8)
    recs["value_len"][recs["type"] == 1] = 0
    fo = (ctypes.c_uint64 * 4)()
    fl = (ctypes.c_uint64 * 4)()
    nf = ctypes.c_uint32()
    total = gen.cly_gen_layout(recs.ctypes.data, n, 1 << 62, 4096, fo, fl, 4, ctypes.byref(nf))
    d_buf = torch.empty(int(total) + 4096, dtype=torch.uint8, device="cuda")
    d_recs = torch.from_numpy(recs.view(np.uint8)).to("cuda")
    if gen.cly_gen_encode(ctypes.c_void_p(d_buf.data_ptr()), ctypes.c_void_p(d_recs.data_ptr()), n, seed) != 0:
        return {"error": "gen"}
    del d_recs
    files = [(d_buf.data_ptr() + int(fo[0]), int(fl[0]), 1)]
    d_out = torch.empty((n + 1024) * 48, dtype=torch.uint8, device="cuda")
    t, kscan, need, res = timed_scans(sc, files, d_out.data_ptr(), n + 1024)
    out = {"value": round(int(fl[0]) / t / 2**30, 2), "unit": "GiB/s", "ms": round(t * 1e3, 3),
           "k_scan_ms": round(kscan, 3), "bytes": int(fl[0]), "records": int(need),
           "mean_record_bytes": round(int(fl[0]) / max(1, need), 2),
           "ok": bool(need == n and res[0].status == 0)}
    del d_out, d_buf
    return out


def append_leg(wl, sc, first, torch, reps=3):
    """The write path over the whole configuration: every scanned record
    re-appended by cly_append_device (appendLogRecord over a batch, db.go:368-413)
    into fresh data files; GiB/s of records written (device-resident)."""
    from couloydb_amd import REC_IN_DTYPE
    n = wl.expect_records
    t = wl.d_out[: n * 48].view(torch.int64).view(n, 6)
    off, fid = t[:, 0], (t[:, 3] & 0xFFFFFFFF)
    u32 = wl.d_out[: n * 48].view(torch.int32).view(n, 12)
    ks, vs = u32[:, 8].to(torch.int64), u32[:, 9].to(torch.int64)
    b8 = wl.d_out[: n * 48].view(n, 48)
    hsz, tl = b8[:, 42].to(torch.int64), b8[:, 43].to(torch.int64)
    bases = torch.tensor([p for p, _, _ in wl.dev_files], dtype=torch.int64, device="cuda")
    fids = torch.tensor([f for _, _, f in wl.dev_files], dtype=torch.int64, device="cuda")
    fidx = torch.searchsorted(fids, fid)
    kp = bases[fidx] + off + hsz + tl
    ri = torch.zeros((n, 5), dtype=torch.int64, device="cuda")
    ri[:, 0] = kp
    ri[:, 1] = kp + (ks - tl)
    ri[:, 2] = (ks - tl) | (vs << 32)
    ri[:, 3] = t[:, 1]
    ri[:, 4] = b8[:, 40].to(torch.int64) | (b8[:, 41].to(torch.int64) << 8)
    dfs = DATA_FILE_SIZE
    rc, lens, q = sc.append_device(ri.data_ptr(), n, 0, False, 0, 0, dfs, None, 0, None)
    nreg = q.n_out_files
    out = torch.empty(nreg * int(q.out_stride), dtype=torch.uint8, device="cuda")
    pos = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    ms = []
    for i in range(reps + 1):
        rc, lens, r = sc.append_device(ri.data_ptr(), n, 0, False, 0, 0, dfs, out.data_ptr(), nreg, pos.data_ptr())
        if rc != 0:
            return {"error": rc}
        if i:
            ms.append(r.append_ms)
    # the records re-encode to the input's bytes (NO_TX_ID keys, canonical headers)
    same = all(torch.equal(out[k * int(q.out_stride):k * int(q.out_stride) + lens[k]],
                           wl.d_buf[wl.file_off[k]:wl.file_off[k] + lens[k]]) for k in range(nreg))
    res = {"append_ms": round(min(ms), 3), "value": round(int(r.bytes) / (min(ms) / 1e3) / 2**30, 2), "unit": "GiB/s",
           "records": n, "bytes": int(r.bytes), "files": nreg, "identical_to_input": bool(same)}
    del out, pos, ri
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """`bench.py --gpus N` run without an outer launcher: start N rank
    processes (one per GPU) through torch.distributed.run as a CHILD process
    (this process never touches the GPU, so no exec after GPU init), let rank 0
    print the JSON line on the inherited stdout, and return the launcher's exit
    status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dry_protocol(args, rank, world):
    """--dry-protocol: the rank protocol alone on the CPU (gloo; no GPU, no
    workload): warmup, barrier, K timed no-op steps, barrier, MAX over ranks,
    one line from rank 0 carrying n_gpus and every rank's pid.  The CPU tests
    use it to check the launcher (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(backend="gloo")
    for _ in range(args.warmup):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    pids = [os.getpid()]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(float(t[0]) / max(1, args.steps) * 1e3, 4),
                          "dry_protocol": True, "rank_pids": pids}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=["c1", "c2", "c3", "c4", "c5"],
                    help="default: c2 at --gpus 1 (BASELINE config 2), c5 at --gpus N > 1 (config 5: a 32-GiB "
                         "fid range per GPU, 256 GiB at 8)")
    ap.add_argument("--no-post-merge-open", action="store_true",
                    help="c4: skip the open of the merge's output (hint preload + merged files)")
    ap.add_argument("--no-c5-leg", action="store_true", help="skip the N=1 line's C5 reference leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--verify", action="store_true", help="check one file against the oracle after timing")
    ap.add_argument("--dry-protocol", action="store_true", help="rank protocol only, on the CPU (launcher tests)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    # Ranks: under torch.distributed.run WORLD_SIZE is set and must equal
    # --gpus; without it, --gpus N > 1 starts its own N ranks (before any GPU
    # call in this process) and exits with their status.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (env_world, args.gpus), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_protocol:
        dry_protocol(args, rank, world)
        return
    if args.config is None:
        args.config = "c5" if world > 1 else "c2"

    import torch
    import torch.distributed as dist
    # CLY_BENCH_REHEARSE=1: every rank on GPU 0 over gloo (rehearses the N>1
    # path on a one-GPU box; the driver's multi-GPU runs use RCCL, one GPU per rank)
    rehearse = os.environ.get("CLY_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        if rehearse:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    from couloydb_amd import Scanner, build_info
    wl = make_workload(args.config, torch, rank=rank, device=local)
    sc = Scanner(local)

    merge_ms = [0.0]
    merge_info = {}

    def step():
        r = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
        if args.config == "c4":
            first, res, st, need = r
            rc, lens, m = sc.merge_device(wl.dev_files, wl.d_out.data_ptr(), first, res, wl.live.data_ptr(),
                                          DATA_FILE_SIZE, wl.d_merge.data_ptr(), wl.merge_max_files,
                                          wl.d_hint.data_ptr(), wl.hint_cap)
            if rc != 0:
                raise RuntimeError("cly_merge_device failed: %d (need %d files, %d hint bytes)"
                                   % (rc, m.n_out_files, m.hint_bytes))
            merge_ms[0] += m.merge_ms
            merge_info.update(n_live=int(m.n_live), n_reencoded=int(m.n_reencoded), n_out_files=int(m.n_out_files),
                              hint_bytes=int(m.hint_bytes), out_bytes=int(sum(lens)), out_lens=lens)
        return r

    # index rebuild (db.loadIndex's String/ListMeta indexes) over the scanned
    # tuples on the device, before the timed steps: the device-resident
    # index-load time = scan + index; for c4 its live bytes drive the merge
    first, res, st, need = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    st = sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)[2]
    d_state = torch.empty(max(1, need), dtype=torch.uint8, device="cuda")
    ixr = sc.index_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr())
    ixr = sc.index_device(wl.dev_files, wl.d_out.data_ptr(), first, res, d_state.data_ptr())
    index_info = {"index_ms": round(ixr.index_ms, 3), "scan_ms": round(st.total_ms, 3),
                  "device_index_load_ms": round(st.total_ms + ixr.index_ms, 3),
                  "keys_live": int(ixr.n_live), "records_applied": int(ixr.n_applied),
                  "hash_collisions": int(ixr.n_collisions)}
    if args.config == "c4":
        # the merge's live bytes are the index's; they must equal the workload's
        index_info["matches_workload_live"] = bool((d_state[:need].cpu().numpy() == wl.live_np).all())
        wl.live = d_state
    else:
        del d_state

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    merge_ms[0] = 0.0
    t0 = time.perf_counter()
    scan_ms, res_ms, passes, recs = 0.0, 0.0, 0, 0
    kms = dict.fromkeys(Scanner.KERNELS, 0.0)
    for _ in range(args.steps):
        first, res, st, need = step()
        scan_ms += st.total_ms
        res_ms += st.resolve_ms
        passes = max(passes, st.passes)
        recs = sum(r.n_records for r in res)
        for k, v in sc.kernel_ms().items():
            kms[k] += v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt, scan_ms / args.steps, kms["k_scan"] / args.steps], dtype=torch.float64,
                     device="cpu" if rehearse else "cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, scan_dev_ms, crc_ms = float(t[0]), float(t[1]), float(t[2])
    # the link / k_emit / k_fin split from one more scan call with per-kernel
    # markers (cly_dbg_set bit 2: a marker between kernels costs ~5 us, so the
    # timed steps keep only the k_scan and whole-call ones)
    sc.lib.cly_dbg_set(sc.ctx, 4)
    sc.scan_device(wl.dev_files, wl.d_out.data_ptr(), wl.out_cap)
    kdiag = sc.kernel_ms()
    sc.lib.cly_dbg_set(sc.ctx, 0)
    ms = dt / args.steps * 1e3
    total_bytes = wl.bytes * world
    total_recs = recs * world
    value = total_bytes / (ms / 1e3) / 2**30
    achieved = wl.bytes / (crc_ms / 1e3) / 1e9           # the dominant kernel, k_scan
    step_gbs = wl.bytes / (ms / 1e3) / 1e9
    ok = all(r.status == 0 for r in res) and recs == wl.expect_records
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 values, written in HBM by libclygen)",
        "config": {"workload": args.config, "files_per_gpu": len(wl.dev_files),
                   "bytes_per_gpu": wl.bytes, "records_per_gpu": recs,
                   "parallelism": "files sharded by fid range, %d GPU(s), no collective" % world},
        "mrecords_per_s": round(total_recs / (ms / 1e3) / 1e6, 2),
        "kernel": {"k_scan_ms": round(kms["k_scan"] / args.steps, 4), "all_ms": round(kms["all"] / args.steps, 4),
                   **{k + "_ms": round(kdiag[k], 4) for k in ("link", "k_emit", "k_fin", "retry")},
                   "device_ms": round(scan_dev_ms, 4), "passes": passes, "build": build_info(),
                   "note": "k_scan_ms, all_ms: the timed steps' averages (HIP events); link/k_emit/k_fin: one more "
                           "call with per-kernel markers"},
        "roofline": {"bound": "hbm", "kernel": "k_scan", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": measured_traffic(args.config),
                     "step_achieved": round(step_gbs, 1), "step_frac": round(step_gbs / HBM_PEAK_GBS, 4),
                     "note": "achieved = input bytes per k_scan launch (it reads every byte of every file once) / "
                             "its HIP-event duration; step_* = the same bytes / the whole step's wall time; "
                             "traffic = k_scan HBM read+write bytes per launch from the committed rocprofv3 "
                             "FETCH_SIZE/WRITE_SIZE passes of this build (profiles/*_traffic.json), null if none"},
        "parity_ok": ok,
    }
    out["index"] = index_info
    if args.config == "c2" and rank == 0 and world == 1 and not args.no_host_path:
        out["append"] = append_leg(wl, sc, first, torch)
        out["small_records"] = small_records_leg(sc, torch)
    if args.config == "c4":
        mi = dict(merge_info)
        lens = mi.pop("out_lens")
        mms = merge_ms[0] / args.steps
        mi["merge_ms"] = round(mms, 4)
        mi["merge_io_gbs"] = round((mi["out_bytes"] * 2 + mi["hint_bytes"]) / (mms / 1e3) / 1e9, 1)
        # size-independent checks: the live count, and a rescan of the merge output
        # (every merged record decodes, keys carry NO_TX_ID, files end cleanly) and of the hint file
        mfiles = [(wl.d_merge.data_ptr() + k * DATA_FILE_SIZE, lens[k], k) for k in range(len(lens))]
        cap = mi["n_live"] + 1024
        d2 = torch.empty(cap * 48, dtype=torch.uint8, device="cuda")
        f2, r2, _, n2 = sc.scan_device(mfiles, d2.data_ptr(), cap)
        hf = [(wl.d_hint.data_ptr(), mi["hint_bytes"], 0)]
        f3, r3, _, n3 = sc.scan_device(hf, d2.data_ptr(), cap)
        # loadIndexFromHintFile's scan (merge.go:257-287) of the merge's hint
        # file: ~24-B records, every tile past CAP_T (spill chunks)
        ht, hk, hn, hres = timed_scans(sc, hf, d2.data_ptr(), cap)
        mi["hint_scan"] = {"value": round(mi["hint_bytes"] / ht / 2**30, 2), "unit": "GiB/s",
                           "ms": round(ht * 1e3, 3), "k_scan_ms": round(hk, 3), "records": int(hn),
                           "tb_per_s": round(mi["hint_bytes"] / ht / 1e12, 3)}
        mi["rescan_ok"] = bool(n2 == mi["n_live"] and all(r.status == 0 for r in r2) and n3 == mi["n_live"]
                               and r3[0].status == 0)
        out["merge"] = mi
        del d2
        if rank == 0 and world == 1 and not args.no_post_merge_open:
            torch.cuda.empty_cache()
            try:
                out["post_merge_open"] = post_merge_open_leg(wl, sc, torch, lens, mi["hint_bytes"], mi["n_live"])
            except Exception as e:     # reported in the line, not fatal to it
                out["post_merge_open"] = {"error": repr(e)}
        out["parity_ok"] = bool(ok and mi["n_live"] == wl.n_live and mi["rescan_ok"]
                                and index_info["matches_workload_live"])
    if args.verify and rank == 0:
        from oracle import cly_oracle as co
        from couloydb_amd import TUPLE_DTYPE
        first, res, st, need = step()
        o = wl.d_out[: need * 48].cpu().numpy().view(TUPLE_DTYPE)
        tt, so, eo = co.scan_file(wl.file_bytes(0), wl.dev_files[0][2])
        g = o[first[0]:first[0] + res[0].n_records]
        out["verify_file0"] = bool(len(g) == len(tt) and (g.view(np.uint8) == tt.view(np.uint8)).all()
                                   and so == res[0].status and eo == res[0].end_offset)
    if rank == 0 and world == 1 and not args.no_host_path:
        out["host_path"] = host_path(wl, sc)
        hp = out["host_path"].get("pageable", {})
        if hp and len(wl.dev_files) <= 16:
            # the record source of db.loadIndex (db.go:582-637) from mmap'd files to
            # index tuples in host memory (the cgo path's rate)
            out["host_scan_wall_ms"] = hp["ms"]
    if args.config == "c2" and world == 1 and not args.no_c5_leg:
        # the N = 1 point of config 5's scaling curve (the --gpus N > 1 lines run c5)
        out["c5_n1"] = c5_leg(sc, torch, local)
    if args.config == "c2" and rank == 0 and world == 1 and not args.no_host_path:
        out["index_load"] = index_load_leg(wl, sc)
        out["index_load_wall_ms"] = out["index_load"]["wall_ms"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl)
    if rank == 0:
        print(json.dumps(out), flush=True)
    sc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
