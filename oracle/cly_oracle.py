"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU restatement (oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.  The product path
(couloydb_amd, libclyscan.so) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libclyoracle.so")

TUPLE_DTYPE = np.dtype([
    ("offset", "<i8"), ("expiration", "<i8"), ("tx_id", "<i8"),
    ("fid", "<u4"), ("size", "<u4"), ("key_size", "<u4"), ("value_size", "<u4"),
    ("type", "u1"), ("data_type", "u1"), ("header_size", "u1"), ("txid_len", "u1"),
    ("crc", "<u4")])
REC = 100

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        L.clyo_uvarint.argtypes = [ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_int)]
        L.clyo_uvarint.restype = ctypes.c_uint64
        L.clyo_varint.argtypes = [ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_int)]
        L.clyo_varint.restype = ctypes.c_int64
        L.clyo_put_varint.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.clyo_put_varint.restype = ctypes.c_int
        L.clyo_crc32_update.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.clyo_crc32_update.restype = ctypes.c_uint32
        L.clyo_read_log_record.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.clyo_read_log_record.restype = ctypes.c_int
        L.clyo_scan_file.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_uint64, P(ctypes.c_int64), P(ctypes.c_int32)]
        L.clyo_scan_file.restype = ctypes.c_uint64
        L.clyo_encode_record.argtypes = [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64]
        L.clyo_encode_record.restype = ctypes.c_uint64
        L.clyo_scan_path_faithful.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64,
                                              P(ctypes.c_int64), P(ctypes.c_int32)]
        L.clyo_scan_path_faithful.restype = ctypes.c_int64
        L.clyo_scan_files_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int]
        L.clyo_scan_files_mt.restype = ctypes.c_uint64
        L.clyo_merge.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint64, ctypes.c_void_p]
        L.clyo_merge.restype = ctypes.c_int
        L.clyo_decode_pos.argtypes = [ctypes.c_void_p, ctypes.c_uint64, P(ctypes.c_uint32), P(ctypes.c_int64)]
        L.clyo_decode_pos.restype = ctypes.c_int
        L.clyo_load_index.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_int64, ctypes.c_void_p]
        L.clyo_load_index.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(buf):
    a = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    return a, (a.ctypes.data if a.size else None)


def varint(b):
    a, p = _ptr(bytes(b) if b else b"\0")
    n = ctypes.c_int()
    v = lib().clyo_varint(p, len(b), ctypes.byref(n))
    return v, n.value


def crc32(b):
    a, p = _ptr(bytes(b) if b else b"\0")
    return lib().clyo_crc32_update(0, p, len(b))


def scan_file(data, fid=0):
    """-> (tuples ndarray, status, end_offset): the db.loadIndex inner loop."""
    a, p = _ptr(data)
    end = ctypes.c_int64()
    st = ctypes.c_int32()
    cap = len(a) // 4 + 2
    out = np.zeros(cap, dtype=TUPLE_DTYPE)
    n = lib().clyo_scan_file(p, len(a), fid, out.ctypes.data, cap, ctypes.byref(end), ctypes.byref(st))
    return out[:n], st.value, end.value


def encode_record(key, value, typ=0, dtype=0, exp=0):
    out = np.zeros(26 + len(key) + len(value), dtype=np.uint8)
    k = np.frombuffer(key, np.uint8) if key else np.zeros(1, np.uint8)
    v = np.frombuffer(value, np.uint8) if value else np.zeros(1, np.uint8)
    n = lib().clyo_encode_record(out.ctypes.data, typ, dtype, k.ctypes.data, len(key), v.ctypes.data,
                                 len(value), exp)
    return out[:n].tobytes()


def scan_path_faithful(path, fid=0, max_records=0):
    end = ctypes.c_int64()
    st = ctypes.c_int32()
    n = lib().clyo_scan_path_faithful(path.encode(), fid, max_records, ctypes.byref(end), ctypes.byref(st))
    return n, st.value, end.value


def scan_files_mt(arrays, fids, nthreads):
    n = len(arrays)
    bases = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrays])
    lens = (ctypes.c_uint64 * n)(*[len(a) for a in arrays])
    fa = (ctypes.c_uint32 * n)(*fids)
    return lib().clyo_scan_files_mt(bases, lens, fa, n, nthreads)


class LoadResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("records", "applied", "str_keys", "listmeta_keys", "expired",
                                               "with_ttl", "tx_pending")] + \
               [("write_off", ctypes.c_int64), ("status", ctypes.c_int32), ("_pad", ctypes.c_int32)]


LI_UNSUPPORTED = -20


def load_index(arrays, fids, now_ns):
    """clyo_load_index: db.loadIndex (String/ListMeta) over the files in fid
    order -> (rc, LoadResult)."""
    n = len(arrays)
    bases = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrays])
    lens = (ctypes.c_uint64 * n)(*[len(a) for a in arrays])
    fa = (ctypes.c_uint32 * n)(*fids)
    r = LoadResult()
    rc = lib().clyo_load_index(bases, lens, fa, n, now_ns, ctypes.byref(r))
    return rc, r


class MergeResult(ctypes.Structure):
    _fields_ = [("n_live", ctypes.c_uint64), ("n_reencoded", ctypes.c_uint64), ("hint_bytes", ctypes.c_uint64),
                ("n_out_files", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


def merge(arrays, tuples, tuple_file, live, data_file_size):
    """db.merge rewrite (merge.go:90-143) -> (rc, [output file bytes], hint bytes, MergeResult)."""
    tuples = np.ascontiguousarray(tuples, dtype=TUPLE_DTYPE)
    tf = np.ascontiguousarray(tuple_file, dtype=np.uint32)
    lv = np.ascontiguousarray(live, dtype=np.uint8)
    n = len(tuples)
    keep = [np.ascontiguousarray(a) if len(a) else np.zeros(1, np.uint8) for a in arrays]
    bases = (ctypes.c_void_p * max(1, len(keep)))(*[a.ctypes.data for a in keep])
    live_bytes = int(tuples["size"][lv != 0].astype(np.int64).sum()) if n else 0
    max_files = live_bytes // max(1, data_file_size // 2) + 2
    out = np.zeros(max_files * data_file_size, np.uint8)
    out_len = np.zeros(max_files, np.uint64)
    hint_cap = int(n * 48 + tuples["key_size"].astype(np.int64).sum()) + 64 if n else 64
    hint = np.zeros(hint_cap, np.uint8)
    r = MergeResult()
    rc = lib().clyo_merge(bases, tf.ctypes.data if n else None, tuples.ctypes.data if n else None, n,
                          lv.ctypes.data if n else None, data_file_size, out.ctypes.data, max_files,
                          out_len.ctypes.data, hint.ctypes.data, hint_cap, ctypes.byref(r))
    files = [out[k * data_file_size:k * data_file_size + int(out_len[k])].tobytes() for k in range(r.n_out_files)] \
        if rc == 0 else []
    return rc, files, hint[:r.hint_bytes].tobytes() if rc == 0 else b"", r


def decode_pos(value):
    """DecodeLogRecordPos -> (rc, fid, offset)."""
    a, p = _ptr(bytes(value) if value else b"\0")
    f = ctypes.c_uint32()
    o = ctypes.c_int64()
    rc = lib().clyo_decode_pos(p, len(value), ctypes.byref(f), ctypes.byref(o))
    return rc, f.value, o.value


def hint_positions(data, tuples):
    """loadIndexFromHintFile's per-record step (merge.go:272-284) over scanned
    hint tuples -> (rc, fids uint32[], offsets int64[])."""
    fids = np.zeros(len(tuples), np.uint32)
    offs = np.zeros(len(tuples), np.int64)
    for i, t in enumerate(tuples):
        o = int(t["offset"]) + int(t["header_size"]) + int(t["key_size"])
        rc, f, off = decode_pos(bytes(data[o:o + int(t["value_size"])]))
        if rc:
            return rc, fids[:i], offs[:i]
        fids[i], offs[i] = f, off
    return 0, fids, offs
