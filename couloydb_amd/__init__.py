"""couloydb_amd — MI355X-native log-record scan for CouloyDB data files.

Host-side mirror of the reference interface for the scan path
(data/dataFile.go, data/logRecord.go, db.go:582-637), over the C-ABI of
include/clyscan.h.  The decode + CRC runs in HIP kernels on gfx950; this module
only moves buffers and shapes results.

    from couloydb_amd import Scanner, DataFile
    with Scanner(device=0) as sc:
        res = sc.scan([DataFile.from_path("000000000.cly", fid=0)])
        for rec, size in res.records(0): ...
"""
import ctypes
import os

import numpy as np

from . import _abi
from ._abi import (END_EOF, END_TORN, END_ZERO, ERR_CRC, ERR_OFFSET, ERR_TRUNC5, ERR_VARINT,
                   POS_DTYPE, REC_IN_DTYPE, TUPLE_DTYPE)

__all__ = ["POS_DTYPE", "Scanner", "DataFile", "LogRecord", "LogPos", "ScanResult", "ScanError", "MergeResult",
           "ErrInvalidCRC", "TUPLE_DTYPE", "STATUS_NAMES"]

# data/logRecord.go:10-16 / :20-26
LogRecordNormal, LogRecordDeleted, LogRecordTxnCommit, LogRecordTxnRollback, LogRecordTxnBegin = range(5)
String, Hash, List, ListMeta, Set = range(5)

STATUS_NAMES = {END_EOF: "EOF", END_ZERO: "EOF(zero header)", END_TORN: "EOF(torn record)",
                ERR_CRC: "ErrInvalidCRC", ERR_TRUNC5: "panic(5-byte tail)",
                ERR_VARINT: "panic(varint overflow)", ERR_OFFSET: "mmap: invalid ReadAt offset"}


class ScanError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__("clyscan error %d: %s %s" % (code, STATUS_NAMES.get(code, ""), msg))


class ErrInvalidCRC(ScanError):
    """public.ErrInvalidCRC (public/errors.go:13)."""


class LogPos(tuple):
    """data.LogPos{Fid, Offset} (data/logRecord.go:52-55)."""
    __slots__ = ()

    def __new__(cls, fid, offset):
        return tuple.__new__(cls, (fid, offset))

    fid = property(lambda s: s[0])
    offset = property(lambda s: s[1])


class LogRecord:
    """data.LogRecord (data/logRecord.go:43-49); Key/Value are views of the file bytes."""
    __slots__ = ("key", "value", "type", "data_type", "expiration")

    def __init__(self, key, value, type, data_type, expiration):
        self.key, self.value, self.type, self.data_type, self.expiration = key, value, type, data_type, expiration


class DataFile:
    """A data file's bytes (host memory) plus its file id (data/dataFile.go:12-17)."""

    def __init__(self, data, fid=0):
        self.data = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        self.fid = fid

    @classmethod
    def from_path(cls, path, fid=None):
        if fid is None:
            fid = int(os.path.basename(path).split(".")[0])    # "%09d.cly", db.go:452-458
        arr = np.fromfile(path, dtype=np.uint8) if os.path.getsize(path) else np.zeros(0, np.uint8)
        return cls(arr, fid)


class ScanResult:
    """Output of one scan call: tuples (numpy structured array, TUPLE_DTYPE) in
    file order, per-file first index, n_records, end_offset and status."""

    def __init__(self, files, tuples, file_first, res, stats):
        self.files = files
        self.tuples = tuples
        self.file_first = file_first
        self.n_records = [r.n_records for r in res]
        self.end_offset = [r.end_offset for r in res]
        self.status = [r.status for r in res]
        self.stats = stats

    def file_tuples(self, i):
        a = self.file_first[i]
        return self.tuples[a:a + self.n_records[i]]

    def records(self, i):
        """Yield (LogRecord, size) exactly as repeated ReadLogRecord calls do; raise
        ErrInvalidCRC / ScanError where the reference returns an error."""
        f = self.files[i]
        buf = f.data
        for t in self.file_tuples(i):
            o, h, ks, vs = int(t["offset"]), int(t["header_size"]), int(t["key_size"]), int(t["value_size"])
            key = buf[o + h:o + h + ks].tobytes()
            val = buf[o + h + ks:o + h + ks + vs].tobytes()
            yield LogRecord(key, val, int(t["type"]), int(t["data_type"]), int(t["expiration"])), int(t["size"])
        st = self.status[i]
        if st == ERR_CRC:
            raise ErrInvalidCRC(st, "at offset %d" % self.end_offset[i])
        if st < 0:
            raise ScanError(st, "at offset %d" % self.end_offset[i])


class MergeResult:
    """Output of Scanner.merge: the merge DB's data files (fid k = files[k]), the
    hint-index file, and the counters of cly_merge_result."""

    def __init__(self, files, hint, r):
        self.files = files
        self.hint = hint
        self.n_live = r.n_live
        self.n_reencoded = r.n_reencoded
        self.n_out_files = r.n_out_files


class Scanner:
    """One GPU context (cly_ctx).  Not thread-safe; one per device."""

    def __init__(self, device=0, lib="libclyscan.so"):
        self.lib_name = lib
        self.lib = _abi.load_scan_lib(lib)
        self._dev_key, self._dev_arr = None, None      # scan_device's last file array (reused when equal)
        self.ctx = ctypes.c_void_p()
        rc = self.lib.cly_ctx_create(device, ctypes.byref(self.ctx))
        if rc != 0:
            raise ScanError(rc, "cly_ctx_create(device=%d)" % device)

    def close(self):
        if self.ctx:
            self.lib.cly_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _file_array(files, device_ptrs=None):
        arr = (_abi.ClyFile * max(1, len(files)))()
        for i, f in enumerate(files):
            if device_ptrs is None:
                arr[i].base = f.data.ctypes.data if len(f.data) else None
                arr[i].len = len(f.data)
            else:
                arr[i].base, arr[i].len = device_ptrs[i]
            arr[i].fid = f.fid if hasattr(f, "fid") else f[2]
        return arr

    def scan(self, files):
        """Host-memory path (cly_scan): H2D, scan, D2H."""
        files = list(files)
        arr = self._file_array(files)
        cap = int(self.lib.cly_scan_capacity(arr, len(files)))
        out = np.zeros(max(cap, 1), dtype=TUPLE_DTYPE)
        first = (ctypes.c_uint64 * max(1, len(files)))()
        res = (_abi.ClyFileResult * max(1, len(files)))()
        need = ctypes.c_uint64()
        st = _abi.ClyStats()
        rc = self.lib.cly_scan(self.ctx, arr, len(files), out.ctypes.data, cap, first, res,
                               ctypes.byref(need), ctypes.byref(st))
        if rc == _abi.ERR_CAPACITY:
            out = np.zeros(int(need.value), dtype=TUPLE_DTYPE)
            rc = self.lib.cly_scan(self.ctx, arr, len(files), out.ctypes.data, int(need.value), first, res,
                                   ctypes.byref(need), ctypes.byref(st))
        if rc != 0:
            raise ScanError(rc, self.lib.cly_strerror(rc).decode())
        n = len(files)
        return ScanResult(files, out[:int(need.value)], [int(first[i]) for i in range(n)],
                          [res[i] for i in range(n)], st)

    def merge(self, files, live, data_file_size):
        """db.merge's rewrite loop (merge.go:90-143) on the device, host buffers
        in and out (cly_merge).  live[i]: the index still points at the i-th
        record of scan(files) (merge.go:104-132).  Returns a MergeResult."""
        files = list(files)
        arr = self._file_array(files)
        lv = np.ascontiguousarray(live, dtype=np.uint8)
        r = _abi.ClyMergeResult()
        rc = self.lib.cly_merge(self.ctx, arr, len(files), lv.ctypes.data if len(lv) else None, len(lv),
                                data_file_size, None, 0, None, None, 0, ctypes.byref(r))
        if rc not in (0, _abi.ERR_CAPACITY):
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, "cly_merge")
        nf = max(1, int(r.n_out_files))
        stride = int(r.out_stride)
        out = np.zeros(nf * stride, np.uint8)
        lens = (ctypes.c_uint64 * nf)()
        hint = np.zeros(max(1, int(r.hint_bytes)), np.uint8)
        rc = self.lib.cly_merge(self.ctx, arr, len(files), lv.ctypes.data if len(lv) else None, len(lv),
                                data_file_size, out.ctypes.data, nf, lens, hint.ctypes.data, len(hint),
                                ctypes.byref(r))
        if rc != 0:
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, "cly_merge")
        outs = [out[k * stride:k * stride + int(lens[k])].tobytes() for k in range(int(r.n_out_files))]
        return MergeResult(outs, hint[:int(r.hint_bytes)].tobytes(), r)

    def load_hint(self, hint_file):
        """loadIndexFromHintFile (merge.go:257-287): scan the hint-index file and
        decode each record's LogPos (DecodeLogRecordPos).  Returns (tuples,
        positions[POS_DTYPE], status, end_offset); raises ScanError(ERR_VARINT)
        where the reference's decode panics and ErrInvalidCRC on a corrupt record."""
        arr = self._file_array([hint_file])
        cap = int(self.lib.cly_scan_capacity(arr, 1)) + 16
        out = np.zeros(cap, dtype=TUPLE_DTYPE)
        pos = np.zeros(cap, dtype=POS_DTYPE)
        n = ctypes.c_uint64()
        res = _abi.ClyFileResult()
        rc = self.lib.cly_hint_scan(self.ctx, arr, out.ctypes.data, pos.ctypes.data, cap, ctypes.byref(n),
                                    ctypes.byref(res))
        if rc != 0:
            raise ScanError(rc, "cly_hint_scan (after %d records)" % n.value)
        if res.status == ERR_CRC:
            raise ErrInvalidCRC(res.status, "at offset %d" % res.end_offset)
        if res.status < 0:
            raise ScanError(res.status, "at offset %d" % res.end_offset)
        k = int(n.value)
        return out[:k], pos[:k], res.status, res.end_offset

    def index(self, files):
        """db.loadIndex's rebuild of the five indexes (db.go:511-651) on the
        device, host buffers in (cly_index).  Returns (state per record in scan
        order: IX_DEAD / IX_LIVE / IX_LOADONLY, ClyIndexResult)."""
        files = list(files)
        arr = self._file_array(files)
        cap = int(self.lib.cly_scan_capacity(arr, len(files))) + 16
        state = np.zeros(cap, np.uint8)
        n = ctypes.c_uint64()
        r = _abi.ClyIndexResult()
        rc = self.lib.cly_index(self.ctx, arr, len(files), state.ctypes.data, cap, ctypes.byref(n), ctypes.byref(r))
        if rc != 0:
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, "cly_index")
        return state[:int(n.value)], r

    def index_device(self, dev_files, d_tuples, file_first, results, d_state, stream=None):
        """Device-resident index rebuild over a scan_device result -> ClyIndexResult."""
        n = len(dev_files)
        arr = (_abi.ClyFile * max(1, n))()
        for i, (ptr, ln, fid) in enumerate(dev_files):
            arr[i].base, arr[i].len, arr[i].fid = ptr, ln, fid
        first = (ctypes.c_uint64 * max(1, n))(*file_first)
        res = (_abi.ClyFileResult * max(1, n))(*results)
        r = _abi.ClyIndexResult()
        rc = self.lib.cly_index_device(self.ctx, arr, n, d_tuples, first, res, d_state, ctypes.byref(r), stream)
        if rc != 0:
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, "cly_index_device")
        return r

    def append(self, records, tx_id=0, commit=False, active_fid=0, write_off=0, data_file_size=256 << 20):
        """appendLogRecord over a batch from host memory (cly_append): records =
        [(key, value, type, data_type, expiration)].  Returns ([region bytes,
        region 0 from write_off on], [(fid, offset)], ClyAppendResult)."""
        n = len(records)
        keep = []
        ri = np.zeros(max(1, n), REC_IN_DTYPE)
        for i, (k, v, typ, dt, exp) in enumerate(records):
            kb, vb = np.frombuffer(k, np.uint8), np.frombuffer(v, np.uint8)
            keep += [kb, vb]
            ri[i]["key"], ri[i]["key_len"] = (kb.ctypes.data if len(kb) else 0), len(kb)
            ri[i]["value"], ri[i]["value_len"] = (vb.ctypes.data if len(vb) else 0), len(vb)
            ri[i]["type"], ri[i]["data_type"], ri[i]["expiration"] = typ, dt, exp
        r = _abi.ClyAppendResult()
        args = (self.ctx, ri.ctypes.data, n, tx_id, 1 if commit else 0, active_fid, write_off, data_file_size)
        rc = self.lib.cly_append(*args, None, 0, None, None, ctypes.byref(r))
        if rc not in (0, _abi.ERR_CAPACITY):
            raise ScanError(rc, "cly_append")
        nreg, stride = int(r.n_out_files), int(r.out_stride)
        out = np.zeros(max(1, nreg) * stride, np.uint8)
        lens = (ctypes.c_uint64 * max(1, nreg))()
        pos = np.zeros(n + 2, POS_DTYPE)
        rc = self.lib.cly_append(*args, out.ctypes.data, nreg, lens, pos.ctypes.data, ctypes.byref(r))
        if rc != 0:
            raise ScanError(rc, "cly_append")
        regions = [out[k * stride + (write_off if k == 0 else 0):k * stride + int(lens[k])].tobytes()
                   for k in range(nreg)]
        nt = n + (1 if commit else 0)
        return regions, [(int(p["fid"]), int(p["offset"])) for p in pos[:nt]], r

    def append_device(self, d_recs, n, tx_id, commit, active_fid, write_off, data_file_size, d_out, out_max_files,
                      d_pos, stream=None):
        """Batched append (db.appendLogRecord over a batch, db.go:368-413; WriteBatch
        with commit=True): d_recs = device array of n REC_IN_DTYPE records.
        Returns (rc, region lengths, ClyAppendResult)."""
        lens = (ctypes.c_uint64 * max(1, out_max_files))()
        r = _abi.ClyAppendResult()
        rc = self.lib.cly_append_device(self.ctx, d_recs, n, tx_id, 1 if commit else 0, active_fid, write_off,
                                        data_file_size, d_out, out_max_files, lens, d_pos, ctypes.byref(r), stream)
        return rc, [int(lens[k]) for k in range(min(out_max_files, int(r.n_out_files)))], r

    def merge_device(self, dev_files, d_tuples, file_first, results, d_live, data_file_size, d_out, out_max_files,
                     d_hint, hint_cap, stream=None):
        """Device-resident merge (cly_merge_device) over a scan_device result.
        Returns (rc, out_file_lens, ClyMergeResult); rc CLY_ERR_CAPACITY leaves the
        needs in the result."""
        n = len(dev_files)
        arr = (_abi.ClyFile * max(1, n))()
        for i, (ptr, ln, fid) in enumerate(dev_files):
            arr[i].base, arr[i].len, arr[i].fid = ptr, ln, fid
        first = (ctypes.c_uint64 * max(1, n))(*file_first)
        res = (_abi.ClyFileResult * max(1, n))(*results)
        lens = (ctypes.c_uint64 * max(1, out_max_files))()
        r = _abi.ClyMergeResult()
        rc = self.lib.cly_merge_device(self.ctx, arr, n, d_tuples, first, res, d_live, data_file_size, d_out,
                                       out_max_files, lens, d_hint, hint_cap, ctypes.byref(r), stream)
        return rc, [int(lens[k]) for k in range(min(out_max_files, int(r.n_out_files)))], r

    def set_clock(self, now_ns):
        """loadIndex's time.Now() for the TTL sweep of the index entries
        (UnixNano; 0 = the wall clock at each call)."""
        self.lib.cly_ctx_set_clock(self.ctx, int(now_ns))

    def prepare_load(self):
        """cly_load_prepare: allocate the load driver's page-locked staging now
        (an application's start-up step; the first open then does not pay for
        it).  Returns the status (CLY_OK, or CLY_ERR_DEVICE: opens allocate lazily)."""
        return int(self.lib.cly_load_prepare())

    def open_db(self, path, data_file_size=0, apply_sweep=False):
        """NewCouloyDB's index load (db.go:442-655, merge.go:240-287) from the
        `*.cly`, hint-index and merge-finished files of directory `path`, on
        this scanner's device (cly_db_open_opts).  apply_sweep: append the TTL
        sweep's tombstones to the active file on disk, as db.Del does."""
        return LoadedDB(self, path, data_file_size, apply_sweep)

    KERNELS = ("k_scan", "link", "k_emit", "k_fin", "retry", "all")

    def kernel_ms(self):
        """Per-kernel HIP-event times (ms) of the last scan_device call: k_scan,
        the link rounds (k_link, the device repair round, host-driven repairs), k_emit, k_fin,
        the attempts run again with a larger spill pool (0 unless a tile held more than CAP_T
        records and the pool was short), all."""
        k = (ctypes.c_double * 6)()
        self.lib.cly_dbg_kernel_ms(self.ctx, k)
        return dict(zip(self.KERNELS, list(k)))

    def scan_device(self, dev_files, d_out, out_cap, stream=None):
        """Device-resident path: dev_files = [(device_ptr, len, fid)], d_out =
        device pointer of out_cap tuples.  Returns (file_first, results, stats, needed)."""
        n = len(dev_files)
        key = tuple(dev_files)
        if key != self._dev_key:           # (a repeated call over the same files builds no array)
            arr = (_abi.ClyFile * max(1, n))()
            for i, (ptr, ln, fid) in enumerate(dev_files):
                arr[i].base, arr[i].len, arr[i].fid = ptr, ln, fid
            self._dev_key, self._dev_arr = key, arr
        arr = self._dev_arr
        first = (ctypes.c_uint64 * max(1, n))()
        res = (_abi.ClyFileResult * max(1, n))()
        need = ctypes.c_uint64()
        st = _abi.ClyStats()
        rc = self.lib.cly_scan_device(self.ctx, arr, n, d_out, out_cap, first, res, ctypes.byref(need),
                                      ctypes.byref(st), stream)
        if rc != 0:
            raise ScanError(rc, self.lib.cly_strerror(rc).decode())
        return list(first)[:n], list(res)[:n], st, int(need.value)


def build_info(lib="libclyscan.so"):
    return _abi.load_scan_lib(lib).cly_build_info().decode()


class LoadedDB:
    """The indexes NewCouloyDB holds after loadIndex (include/clyload.h):
    String / ListMeta key -> LogPos, Hash (key, field), List (key, seq gob
    bytes) and Set (key, member) -> LogPos, and values by position
    (getLogRecordByPos).  get/hget/lget/sget return the value bytes, or raise
    KeyError for public.ErrKeyNotFound."""

    def __init__(self, scanner, path, data_file_size=0, apply_sweep=False):
        scanners = list(scanner) if isinstance(scanner, (list, tuple)) else [scanner]
        self.lib = scanners[0].lib
        self.db = ctypes.c_void_p()
        self.stats = _abi.ClyLoadStats()
        opt = _abi.ClyDbOptions()
        opt.data_file_size = data_file_size
        opt.flags = _abi.DB_APPLY_SWEEP if apply_sweep else 0
        if len(scanners) == 1:
            rc = self.lib.cly_db_open_opts(scanners[0].ctx, os.fsencode(path), ctypes.byref(opt),
                                           ctypes.byref(self.db), ctypes.byref(self.stats))
        else:
            ctxs = (ctypes.c_void_p * len(scanners))(*[sc.ctx.value for sc in scanners])
            rc = self.lib.cly_db_open_multi(ctxs, len(scanners), os.fsencode(path), ctypes.byref(opt),
                                            ctypes.byref(self.db), ctypes.byref(self.stats))
        if rc != 0:
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, self.lib.cly_strerror(rc).decode())

    def entries(self, kind):
        """cly_db_entries of one kind (_abi.IT_*): [(key, sub, LogPos, expiration)]."""
        n = int(self.lib.cly_db_count(self.db, kind))
        arr = (_abi.ClyDbEntry * max(1, n))()
        got = int(self.lib.cly_db_entries(self.db, kind, 0, arr, n))
        out = []
        for e in arr[:got]:
            key = ctypes.string_at(e.key, e.key_len) if e.key_len else b""
            sub = ctypes.string_at(e.sub, e.sub_len) if e.sub_len else b""
            out.append((key, sub, LogPos(e.pos.fid, e.pos.offset), int(e.expiration)))
        return out

    def close(self):
        if self.db:
            self.lib.cly_db_close(self.db)
            self.db = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _pos(self, rc, pos, what):
        if rc == _abi.DB_NOT_FOUND:
            raise KeyError(what)
        if rc != 0:
            raise ScanError(rc, self.lib.cly_strerror(rc).decode())
        return LogPos(pos.fid, pos.offset)

    def pos(self, key):
        p = _abi.ClyPos()
        return self._pos(self.lib.cly_db_get(self.db, key, len(key), ctypes.byref(p)), p, key)

    def hpos(self, key, field):
        p = _abi.ClyPos()
        return self._pos(self.lib.cly_db_hget(self.db, key, len(key), field, len(field), ctypes.byref(p)), p,
                         (key, field))

    def lpos(self, key, seq):
        p = _abi.ClyPos()
        return self._pos(self.lib.cly_db_lget(self.db, key, len(key), seq, len(seq), ctypes.byref(p)), p, (key, seq))

    def spos(self, key, member):
        p = _abi.ClyPos()
        return self._pos(self.lib.cly_db_sget(self.db, key, len(key), member, len(member), ctypes.byref(p)), p,
                         (key, member))

    def listmeta_pos(self, key):
        p = _abi.ClyPos()
        return self._pos(self.lib.cly_db_listmeta(self.db, key, len(key), ctypes.byref(p)), p, key)

    def value(self, pos):
        p = _abi.ClyPos()
        p.fid, p.offset = pos.fid, pos.offset
        n = ctypes.c_uint64()
        rc = self.lib.cly_db_value(self.db, ctypes.byref(p), None, 0, ctypes.byref(n))
        if rc == _abi.DB_NOT_FOUND:
            raise KeyError(pos)
        if rc != 0:
            raise (ErrInvalidCRC if rc == ERR_CRC else ScanError)(rc, self.lib.cly_strerror(rc).decode())
        buf = ctypes.create_string_buffer(max(1, n.value))
        rc = self.lib.cly_db_value(self.db, ctypes.byref(p), buf, n.value, ctypes.byref(n))
        if rc != 0:
            raise ScanError(rc, self.lib.cly_strerror(rc).decode())
        return buf.raw[:n.value]

    def get(self, key):
        return self.value(self.pos(key))

    def hget(self, key, field):
        return self.value(self.hpos(key, field))

    def lget(self, key, seq):
        return self.value(self.lpos(key, seq))

    def sget(self, key, member):
        return self.value(self.spos(key, member))


def index_key(lib, dtype, data):
    """cly_index_key: the index key updateIndex derives from decoded key bytes
    -> (P, R) bytes, or raises ValueError('panic') / returns None (no index)."""
    out = ctypes.create_string_buffer(len(data) + 32)
    plen = ctypes.c_uint32()
    n = lib.cly_index_key(dtype, bytes(data), len(data), out, len(data) + 32, ctypes.byref(plen))
    if n == -1:
        raise ValueError("panic")
    if n == -2:
        return None
    return out.raw[:plen.value], out.raw[plen.value:n]


def open_db_multi(scanners, path, data_file_size=0, apply_sweep=False):
    """The index load with the files sharded by fid range over several scanners
    (one per GPU, or several on one): cly_db_open_multi; the index is rebuilt on
    scanners[0]'s device."""
    return LoadedDB(list(scanners), path, data_file_size, apply_sweep)
