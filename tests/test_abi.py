"""CPU tests of the drop-in boundary: the C-ABI libraries load, export every
function include/*.h declares, keep the struct layouts, and the host-only
pieces (capacity bound, writer layout, GF(2) CRC algebra) are correct.
No kernel is launched here."""
import ctypes
import os
import re
import subprocess
import sys
import tempfile
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_golden as mg  # noqa: E402

from couloydb_amd import _abi  # noqa: E402


def declared_functions(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(cly_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.mark.parametrize("header,lib", [("clyscan.h", "libclyscan.so"), ("clyscan.h", "libclyscan_small.so"),
                                        ("clyload.h", "libclyscan.so"), ("clygen.h", "libclygen.so")])
def test_library_exports_header_symbols(header, lib):
    path = _abi.lib_path(lib)
    assert os.path.exists(path), "build the libraries first (__graft_entry__.build())"
    h = ctypes.CDLL(path)
    names = declared_functions(header)
    assert len(names) >= 3
    for n in names:
        assert hasattr(h, n), "%s missing from %s" % (n, lib)
    expect = {"clyscan.h": _abi.SCAN_SYMBOLS, "clyload.h": _abi.LOAD_SYMBOLS}.get(header, _abi.GEN_SYMBOLS)
    assert sorted(expect) == names


def test_struct_layouts():
    assert ctypes.sizeof(_abi.ClyFile) == 24
    assert ctypes.sizeof(_abi.ClyFileResult) == 24
    assert _abi.TUPLE_DTYPE.itemsize == 48
    assert ctypes.sizeof(_abi.ClyGenRec) == 32
    # the C compiler agrees
    src = r'''
    #include <stdio.h>
    #include <stddef.h>
    #include "clyscan.h"
    #include "clygen.h"
    int main(void){ printf("%zu %zu %zu %zu %zu %zu\n", sizeof(cly_file), sizeof(cly_tuple),
      sizeof(cly_file_result), offsetof(cly_tuple, type), offsetof(cly_tuple, crc), sizeof(cly_gen_rec)); return 0; }
    '''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split()
    assert out == ["24", "48", "24", "40", "44", "32"]
    assert _abi.TUPLE_DTYPE.fields["type"][1] == 40 and _abi.TUPLE_DTYPE.fields["crc"][1] == 44


def test_capacity_bound():
    lib = _abi.load_scan_lib()
    arr = (_abi.ClyFile * 3)()
    for i, ln in enumerate([0, 9, 1 << 20]):
        arr[i].len = ln
    assert lib.cly_scan_capacity(arr, 3) == (0 // 9 + 1) + (9 // 9 + 1) + ((1 << 20) // 9 + 1)


def test_build_info():
    s = _abi.load_scan_lib().cly_build_info().decode()
    assert "gfx950" in s and "SEG=" in s and "TILE=" in s and "src=" in s


def test_gen_record_size_and_layout():
    g = _abi.load_gen_lib()
    for tx, vl in [(0, 0), (0, 256), (0, 1024), (1_697_000_000_000_000_017, 70000), (5, 63)]:
        rec = mg.encode_record(mg.key_tx(mg.test_key(3), tx), b"\0" * vl)
        assert g.cly_gen_record_size(tx, vl) == len(rec)
    n = 1000
    recs = np.zeros(n, dtype=_abi.GEN_DTYPE)
    recs["value_len"] = 256
    fo = (ctypes.c_uint64 * 64)()
    fl = (ctypes.c_uint64 * 64)()
    nf = ctypes.c_uint32()
    total = g.cly_gen_layout(recs.ctypes.data, n, 276 * 100 + 275, 4096, fo, fl, 64, ctypes.byref(nf))
    assert nf.value == 10 and all(fl[i] == 27600 for i in range(10))
    assert recs["dst"][100] == 28672 and total == 10 * 28672


GF_TEST = r'''
#include <stdio.h>
#include <stdint.h>
#include "crc_gf.h"
static uint32_t T0[256];
int main(void) {
  for (uint32_t i = 0; i < 256; i++) { uint32_t c = i; for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CLY_POLY : c >> 1; T0[i] = c; }
  uint32_t s = 0x12345678u; int bad = 0;
  for (int L = 0; L < 3000; L++) {
    uint32_t z = s; for (int k = 0; k < L; k++) z = T0[z & 0xff] ^ (z >> 8);
    if (cly_shift(s, L) != z) bad++;
    if (cly_crc_byte_bitwise(s, (uint8_t)L) != (T0[(s ^ (uint8_t)L) & 0xff] ^ (s >> 8))) bad++;
    s = s * 2654435761u + 12345u;
  }
  /* combine: crc(AB) from pieces */
  const char* A = "hello, "; const char* B = "world - couloydb log record";
  uint32_t r = 0xFFFFFFFFu; for (const char* p = A; *p; p++) r = T0[(r ^ (uint8_t)*p) & 0xff] ^ (r >> 8);
  uint32_t q = 0; int nb = 0; for (const char* p = B; *p; p++, nb++) q = T0[(q ^ (uint8_t)*p) & 0xff] ^ (q >> 8);
  printf("%d %08x\n", bad, ~(cly_shift(r, nb) ^ q));
  return 0;
}
'''


def test_gf_shift_algebra():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "gf.c")
        open(c, "w").write(GF_TEST)
        exe = os.path.join(d, "gf")
        subprocess.check_call(["gcc", "-O2", "-I", os.path.join(ROOT, "couloydb_amd", "csrc"), c, "-o", exe])
        bad, crc = subprocess.check_output([exe]).decode().split()
    assert bad == "0"
    assert int(crc, 16) == zlib.crc32(b"hello, world - couloydb log record")


def test_path_struct_layouts():
    """The merge / hint / index / append structs: ctypes and numpy views agree with the C compiler."""
    src = r'''
    #include <stdio.h>
    #include <stddef.h>
    #include "clyscan.h"
    int main(void){ printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(cly_merge_result),
      offsetof(cly_merge_result, merge_ms), sizeof(cly_pos), sizeof(cly_index_result), sizeof(cly_rec_in),
      offsetof(cly_rec_in, expiration), offsetof(cly_rec_in, type), sizeof(cly_append_result),
      offsetof(cly_append_result, append_ms)); return 0; }
    '''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        out = [int(x) for x in subprocess.check_output([exe]).decode().split()]
    assert out[0] == ctypes.sizeof(_abi.ClyMergeResult) and out[1] == _abi.ClyMergeResult.merge_ms.offset
    assert out[2] == _abi.POS_DTYPE.itemsize == 16
    assert out[3] == ctypes.sizeof(_abi.ClyIndexResult)
    assert out[4] == _abi.REC_IN_DTYPE.itemsize == 40
    assert out[5] == _abi.REC_IN_DTYPE.fields["expiration"][1] and out[6] == _abi.REC_IN_DTYPE.fields["type"][1]
    assert out[7] == ctypes.sizeof(_abi.ClyAppendResult) and out[8] == _abi.ClyAppendResult.append_ms.offset
