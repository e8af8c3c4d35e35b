"""Multi-GPU scan: the files of a data directory are split into
contiguous fid ranges balanced by bytes (shard.partition_by_bytes), one context
(and host thread) per device scans its range, and the tuples are concatenated
in fid order, the order db.loadIndex consumes them (db.go:582).  Records never
span files (db.go:376-385), so the shards need no exchange: tx markers that
fall into another shard are resolved by the consumer's ordered tx buffering
over the concatenated tuples, as in the single-device scan."""
import threading

import numpy as np

from . import ScanResult, Scanner, TUPLE_DTYPE, _abi
from .shard import partition_by_bytes


class MultiScanner:
    """One Scanner per device in `devices` (a device may repeat: several
    contexts on one GPU)."""

    def __init__(self, devices):
        self.scanners = [Scanner(d) for d in devices]

    def close(self):
        for s in self.scanners:
            s.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def scan(self, files):
        files = list(files)
        ranges = partition_by_bytes([len(f.data) for f in files], len(self.scanners))
        out = [None] * len(ranges)
        err = []

        def run(k):
            lo, hi = ranges[k]
            try:
                out[k] = self.scanners[k].scan(files[lo:hi]) if hi > lo else None
            except Exception as e:      # re-raised in the caller's thread
                err.append(e)

        th = [threading.Thread(target=run, args=(k,)) for k in range(len(ranges))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise err[0]
        parts = [r for r in out if r is not None]
        tuples = np.concatenate([p.tuples for p in parts]) if parts else np.zeros(0, TUPLE_DTYPE)
        first, res, base = [], [], 0
        for p in parts:
            for i in range(len(p.files)):
                first.append(base + int(p.file_first[i]))
                r = _abi.ClyFileResult()
                r.n_records, r.end_offset, r.status = p.n_records[i], p.end_offset[i], p.status[i]
                res.append(r)
            base += len(p.tuples)
        st = _abi.ClyStats()
        for p in parts:
            st.total_ms = max(st.total_ms, p.stats.total_ms)
            st.records += p.stats.records
            st.bytes += p.stats.bytes
        return ScanResult(files, tuples, first, res, st)
