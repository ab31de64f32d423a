"""CPU tests of the C-ABI boundary: the HIP library loads without a GPU,
exports every function include/*.h declares, and its host-only helpers
(tables, sizing) behave.  No compute call is made here (no GPU)."""
import ctypes
import glob
import hashlib
import json
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_api():
    names = declared_functions()
    assert "nghttp2_amd_hd_huff_encode_batch" in names
    assert "nghttp2_amd_hd_huff_decode_batch" in names


def test_library_exports_every_declared_symbol():
    import nghttp2_amd
    path = nghttp2_amd.lib_path()
    assert os.path.exists(path), "build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True,
                         capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    L = ctypes.CDLL(path)
    for n in declared_functions():
        getattr(L, n)


def test_library_exports_nothing_else():
    """The dynamic symbol table is exactly the declared C ABI: no kernel
    stubs, template instantiations or retired A/B entry points."""
    import nghttp2_amd
    out = subprocess.run(["nm", "-D", "--defined-only", nghttp2_amd.lib_path()], check=True,
                         capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    assert exported == set(declared_functions()), sorted(exported ^ set(declared_functions()))


def test_library_is_gfx950_code_object():
    """The .so carries a HIP fat binary with a gfx950 code object."""
    import nghttp2_amd
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", nghttp2_amd.lib_path()],
                         check=True, capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(nghttp2_amd.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_engine_tables_match_reference_without_gpu():
    import nghttp2_amd
    ref = json.load(open(os.path.join(REPO, "tests", "golden", "reference_tables.json")))
    sym, dec = nghttp2_amd.tables_ref_layout()
    assert hashlib.sha256(sym).hexdigest() == ref["sym_sha256"]
    assert hashlib.sha256(dec).hexdigest() == ref["dec_sha256"]


def test_sizing_helpers():
    import nghttp2_amd
    L = nghttp2_amd.lib()
    assert L.nghttp2_amd_hd_huff_encode_bound(0, 0) >= 16
    # worst case 30 bits per byte + one pad byte per string
    b = L.nghttp2_amd_hd_huff_encode_bound(1000, 10)
    assert b >= (1000 * 30 + 7) // 8 + 10 and b % 16 == 0
    assert L.nghttp2_amd_hd_huff_workspace_size(1 << 20) >= 4 * ((1 << 20) // 4096)
    assert b"gfx950" in L.nghttp2_amd_hd_version()


def test_invalid_arguments_rejected_without_gpu():
    import nghttp2_amd
    L = nghttp2_amd.lib()
    # NULL pointers are rejected before any HIP call
    rv = L.nghttp2_amd_hd_huff_decode_batch(None, None, 5, None, None, None, None, None, None)
    assert rv == nghttp2_amd.NGHTTP2_ERR_INVALID_ARGUMENT
    rv = L.nghttp2_amd_hd_huff_encode_batch(None, None, 5, None, 0, None, None, 0, None)
    assert rv == nghttp2_amd.NGHTTP2_ERR_INVALID_ARGUMENT
