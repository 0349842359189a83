"""CPU tests of the C-ABI boundary: libdrhip.so loads, exports exactly the
entry points include/drhip.h declares, and refuses work cleanly (error
codes, no crash) when no device is initialised.  No compute calls."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "drhip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(drhip_\w+)\s*\(", src, re.M)))


def test_header_declares_python_exports():
    import drhip
    assert declared_symbols() == sorted(drhip.EXPORTS)


def test_library_exports_every_declared_symbol():
    import drhip
    drhip.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", drhip.LIB_PATH], text=True)
    exported = set(re.findall(r" T (drhip_\w+)$", out, re.M))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    import drhip
    out = subprocess.check_output(["/opt/rocm/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                                   "--input=" + os.path.join(os.path.dirname(drhip.LIB_PATH), "build", "scan.o")],
                                  text=True, stderr=subprocess.STDOUT) if os.path.exists(
        os.path.join(os.path.dirname(drhip.LIB_PATH), "build", "scan.o")) else ""
    if out:
        assert "gfx950" in out


def test_calls_before_init_fail_cleanly():
    import drhip
    L = drhip.load()
    if drhip.device_count() > 0:
        pytest.skip("a device is visible; covered by the gpu tests")
    n = C.c_int(-1)
    assert L.drhip_nprocs(C.byref(n)) == 0 and n.value == 0
    out = C.c_double(0)
    rc = L.drhip_reduce(0, drhip.F32, drhip.PLUS, None, 0, C.byref(out))
    assert rc == 2  # DRHIP_ERR_NOT_INIT
    assert b"drhip_init" in L.drhip_last_error()
    devs = (C.c_int * 1)(0)
    assert L.drhip_init(devs, 1) != 0  # no device in this container
    assert L.drhip_init(None, 0) == 4  # DRHIP_ERR_BAD_ARG


def test_bad_arguments_rejected():
    import drhip
    L = drhip.load()
    assert L.drhip_csr_nnz(7, 0, 10, 10, 3, None) != 0
    nnz = C.c_size_t(0)
    assert L.drhip_csr_nnz(0, 0, 50, 50, 0, C.byref(nnz)) == 0
    import oracle
    rp, ci, v = oracle.csr_gen("banded", 0, 50, 50, 1)
    assert nnz.value == ci.size
    for row0, nrows, ncols in ((0, 1, 1), (3, 7, 9), (0, 1000, 1000), (990, 10, 1000), (5, 20, 8)):
        assert L.drhip_csr_nnz(0, row0, nrows, ncols, 0, C.byref(nnz)) == 0
        _, ci, _ = oracle.csr_gen("banded", row0, nrows, ncols, 1)
        assert nnz.value == ci.size, (row0, nrows, ncols)
