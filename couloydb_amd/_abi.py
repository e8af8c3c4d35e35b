"""ctypes declarations of the C-ABI in include/clyscan.h and include/clygen.h.

The shared libraries are built in-tree by ``__graft_entry__.build()`` (or
``make -C couloydb_amd/csrc``).  Loading fails loudly when they are missing:
there is no CPU fallback for the scan.
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))

# status codes (include/clyscan.h)
END_EOF, END_ZERO, END_TORN = 0, 1, 2
ERR_CRC, ERR_TRUNC5, ERR_VARINT, ERR_OFFSET = -1, -2, -3, -4
OK, ERR_CAPACITY, ERR_DEVICE, ERR_ARG, ERR_NOREPAIR = 0, -10, -11, -12, -13


class ClyFile(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_uint64),
                ("fid", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


class ClyFileResult(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("end_offset", ctypes.c_int64),
                ("status", ctypes.c_int32), ("_pad", ctypes.c_int32)]


class ClyStats(ctypes.Structure):
    _fields_ = [("scan_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("passes", ctypes.c_uint32),
                ("n_chunks", ctypes.c_uint32), ("bytes", ctypes.c_uint64),
                ("records", ctypes.c_uint64)]


class ClyGenRec(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_uint64), ("key_index", ctypes.c_uint32),
                ("value_len", ctypes.c_uint32), ("tx_id", ctypes.c_int64),
                ("type", ctypes.c_uint8), ("dtype", ctypes.c_uint8),
                ("value_mode", ctypes.c_uint8), ("_pad", ctypes.c_uint8),
                ("_pad2", ctypes.c_int32)]


class ClyIndexResult(ctypes.Structure):
    _fields_ = [("n_live", ctypes.c_uint64), ("n_applied", ctypes.c_uint64), ("n_host", ctypes.c_uint64),
                ("n_collisions", ctypes.c_uint64), ("index_ms", ctypes.c_double),
                ("n_loadonly", ctypes.c_uint64), ("n_merge_panic", ctypes.c_uint64)]


IX_DEAD, IX_LIVE, IX_HOST, IX_LOADONLY = 0, 1, 2, 3


class ClyAppendResult(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_uint64), ("out_stride", ctypes.c_uint64), ("final_write_off", ctypes.c_uint64),
                ("final_fid", ctypes.c_uint32), ("n_out_files", ctypes.c_uint32), ("append_ms", ctypes.c_double)]


# numpy view of cly_rec_in (40 bytes)
REC_IN_DTYPE = np.dtype([("key", "<u8"), ("value", "<u8"), ("key_len", "<u4"), ("value_len", "<u4"),
                         ("expiration", "<i8"), ("type", "u1"), ("data_type", "u1"), ("_pad", "u1", (6,))])
assert REC_IN_DTYPE.itemsize == 40


class ClyMergeResult(ctypes.Structure):
    _fields_ = [("n_live", ctypes.c_uint64), ("n_reencoded", ctypes.c_uint64),
                ("hint_bytes", ctypes.c_uint64), ("out_stride", ctypes.c_uint64),
                ("n_out_files", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("merge_ms", ctypes.c_double)]


# numpy view of cly_pos (16 bytes)
POS_DTYPE = np.dtype([("offset", "<i8"), ("fid", "<u4"), ("_pad", "<u4")])


# numpy view of cly_tuple (48 bytes)
TUPLE_DTYPE = np.dtype([
    ("offset", "<i8"), ("expiration", "<i8"), ("tx_id", "<i8"),
    ("fid", "<u4"), ("size", "<u4"), ("key_size", "<u4"), ("value_size", "<u4"),
    ("type", "u1"), ("data_type", "u1"), ("header_size", "u1"), ("txid_len", "u1"),
    ("crc", "<u4")])
assert TUPLE_DTYPE.itemsize == 48

GEN_DTYPE = np.dtype([("dst", "<u8"), ("key_index", "<u4"), ("value_len", "<u4"),
                      ("tx_id", "<i8"), ("type", "u1"), ("dtype", "u1"),
                      ("value_mode", "u1"), ("_pad", "u1"), ("_pad2", "<i4")])
assert GEN_DTYPE.itemsize == 32

SCAN_SYMBOLS = ["cly_ctx_create", "cly_ctx_destroy", "cly_ctx_set_clock", "cly_scan_capacity", "cly_scan",
                "cly_scan_device", "cly_merge_device", "cly_merge", "cly_hint_positions_device", "cly_hint_scan",
                "cly_index_device", "cly_index", "cly_append_device", "cly_append",
                "cly_strerror", "cly_build_info"]
GEN_SYMBOLS = ["cly_gen_record_size", "cly_gen_layout", "cly_gen_encode"]
LOAD_SYMBOLS = ["cly_db_open", "cly_db_open_opts", "cly_db_open_multi", "cly_db_close", "cly_db_get", "cly_db_listmeta", "cly_db_hget",
                "cly_db_lget", "cly_db_sget", "cly_db_value", "cly_index_key", "cly_db_count", "cly_db_entries",
                "cly_load_prepare"]
DB_NOT_FOUND, DB_EOF = 1, 2
ERR_DIR, ERR_MERGE_FIN, ERR_KEY_EMPTY = -14, -15, -16
IT_STRING, IT_LISTMETA, IT_HASH, IT_LIST, IT_SET, IT_EXPIRED = range(6)
DB_APPLY_SWEEP = 1


class ClyPos(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("fid", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


class ClyLoadStats(ctypes.Structure):
    _fields_ = [("list_map_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("scan_ms", ctypes.c_double),
                ("index_ms", ctypes.c_double), ("insert_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("n_files", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("records", ctypes.c_uint64),
                ("str_keys", ctypes.c_uint64), ("listmeta_keys", ctypes.c_uint64), ("hash_fields", ctypes.c_uint64),
                ("list_items", ctypes.c_uint64), ("set_members", ctypes.c_uint64),
                ("active_fid", ctypes.c_uint32), ("_pad", ctypes.c_uint32), ("write_off", ctypes.c_int64),
                ("hint_records", ctypes.c_uint64), ("n_expired", ctypes.c_uint64),
                ("write_off_loaded", ctypes.c_int64), ("active_fid_loaded", ctypes.c_uint32),
                ("sweep_files", ctypes.c_uint32), ("n_shards", ctypes.c_uint32), ("_pad2", ctypes.c_uint32),
                ("tuple_slots", ctypes.c_uint64), ("order_ms", ctypes.c_double), ("order_rounds", ctypes.c_uint32),
                ("_pad3", ctypes.c_uint32)]


class ClyDbOptions(ctypes.Structure):
    _fields_ = [("data_file_size", ctypes.c_uint64), ("flags", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


class ClyDbEntry(ctypes.Structure):
    _fields_ = [("key", ctypes.c_void_p), ("key_len", ctypes.c_uint64), ("sub", ctypes.c_void_p),
                ("sub_len", ctypes.c_uint64), ("pos", ClyPos), ("expiration", ctypes.c_int64)]

_libs = {}


def lib_path(name="libclyscan.so"):
    """In-package library by name; an absolute path is taken as is."""
    return name if os.path.isabs(name) else os.path.join(PKG_DIR, name)


def load_scan_lib(name="libclyscan.so"):
    """Load (once) and type the scan library; raises if it is not built."""
    if name in _libs:
        return _libs[name]
    path = lib_path(name)
    if not os.path.exists(path):
        raise RuntimeError("%s is not built (run __graft_entry__.build()); the scan has no CPU fallback" % path)
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    lib.cly_ctx_create.argtypes = [ctypes.c_int, P(ctypes.c_void_p)]
    lib.cly_ctx_create.restype = ctypes.c_int
    lib.cly_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.cly_ctx_destroy.restype = None
    if hasattr(lib, "cly_dbg_kernel_ms"):
        lib.cly_dbg_kernel_ms.argtypes = [ctypes.c_void_p, P(ctypes.c_double)]
        lib.cly_dbg_kernel_ms.restype = ctypes.c_int
    lib.cly_db_open.argtypes = [ctypes.c_void_p, ctypes.c_char_p, P(ctypes.c_void_p), ctypes.c_void_p]
    lib.cly_db_open.restype = ctypes.c_int
    lib.cly_db_open_opts.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, P(ctypes.c_void_p),
                                     ctypes.c_void_p]
    lib.cly_db_open_opts.restype = ctypes.c_int
    lib.cly_db_open_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p,
                                      P(ctypes.c_void_p), ctypes.c_void_p]
    lib.cly_db_open_multi.restype = ctypes.c_int
    lib.cly_db_count.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.cly_db_count.restype = ctypes.c_uint64
    lib.cly_db_entries.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
    lib.cly_db_entries.restype = ctypes.c_uint64
    lib.cly_db_close.argtypes = [ctypes.c_void_p]
    lib.cly_db_close.restype = None
    if hasattr(lib, "cly_load_prepare"):          # (libraries of earlier builds, tools/build_r3_lib.sh)
        lib.cly_load_prepare.argtypes = []
        lib.cly_load_prepare.restype = ctypes.c_int
    for fn in ("cly_db_get", "cly_db_listmeta"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p]
        getattr(lib, fn).restype = ctypes.c_int
    for fn in ("cly_db_hget", "cly_db_lget", "cly_db_sget"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                     ctypes.c_uint64, ctypes.c_void_p]
        getattr(lib, fn).restype = ctypes.c_int
    lib.cly_index_key.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                  P(ctypes.c_uint32)]
    lib.cly_index_key.restype = ctypes.c_int64
    lib.cly_db_value.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                 P(ctypes.c_uint64)]
    lib.cly_db_value.restype = ctypes.c_int
    lib.cly_ctx_set_clock.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.cly_ctx_set_clock.restype = None
    lib.cly_scan_capacity.argtypes = [P(ClyFile), ctypes.c_int]
    lib.cly_scan_capacity.restype = ctypes.c_uint64
    lib.cly_scan.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                             P(ctypes.c_uint64), P(ClyFileResult), P(ctypes.c_uint64), P(ClyStats)]
    lib.cly_scan.restype = ctypes.c_int
    lib.cly_scan_device.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                    P(ctypes.c_uint64), P(ClyFileResult), P(ctypes.c_uint64), P(ClyStats),
                                    ctypes.c_void_p]
    lib.cly_scan_device.restype = ctypes.c_int
    lib.cly_merge_device.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, P(ctypes.c_uint64),
                                     P(ClyFileResult), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint32, P(ctypes.c_uint64), ctypes.c_void_p, ctypes.c_uint64,
                                     P(ClyMergeResult), ctypes.c_void_p]
    lib.cly_merge_device.restype = ctypes.c_int
    lib.cly_merge.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, P(ctypes.c_uint64),
                              ctypes.c_void_p, ctypes.c_uint64, P(ClyMergeResult)]
    lib.cly_merge.restype = ctypes.c_int
    lib.cly_hint_positions_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_void_p, P(ctypes.c_uint64), ctypes.c_void_p]
    lib.cly_hint_positions_device.restype = ctypes.c_int
    lib.cly_hint_scan.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                  P(ctypes.c_uint64), P(ClyFileResult)]
    lib.cly_hint_scan.restype = ctypes.c_int
    lib.cly_index_device.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, P(ctypes.c_uint64),
                                     P(ClyFileResult), ctypes.c_void_p, P(ClyIndexResult), ctypes.c_void_p]
    lib.cly_index_device.restype = ctypes.c_int
    lib.cly_index.argtypes = [ctypes.c_void_p, P(ClyFile), ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                              P(ctypes.c_uint64), P(ClyIndexResult)]
    lib.cly_index.restype = ctypes.c_int
    lib.cly_append_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_uint32, P(ctypes.c_uint64), ctypes.c_void_p, P(ClyAppendResult),
                                      ctypes.c_void_p]
    lib.cly_append_device.restype = ctypes.c_int
    lib.cly_append.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int,
                               ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                               P(ctypes.c_uint64), ctypes.c_void_p, P(ClyAppendResult)]
    lib.cly_append.restype = ctypes.c_int
    lib.cly_strerror.argtypes = [ctypes.c_int]
    lib.cly_strerror.restype = ctypes.c_char_p
    lib.cly_build_info.argtypes = []
    lib.cly_build_info.restype = ctypes.c_char_p
    _libs[name] = lib
    return lib


def load_gen_lib():
    if "gen" in _libs:
        return _libs["gen"]
    path = lib_path("libclygen.so")
    if not os.path.exists(path):
        raise RuntimeError("%s is not built (run __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    lib.cly_gen_record_size.argtypes = [ctypes.c_int64, ctypes.c_uint32]
    lib.cly_gen_record_size.restype = ctypes.c_uint64
    lib.cly_gen_layout.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                   P(ctypes.c_uint64), P(ctypes.c_uint64), ctypes.c_uint32, P(ctypes.c_uint32)]
    lib.cly_gen_layout.restype = ctypes.c_uint64
    lib.cly_gen_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    lib.cly_gen_encode.restype = ctypes.c_int
    _libs["gen"] = lib
    return lib
