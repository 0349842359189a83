"""CPU sanitizer build ("a CPU build with -fsanitize=address,
undefined"; the reference's own instrumentation is libFuzzer,
test/fuzz/cpu/CMakeLists.txt:13-14).  Everything here is host code:

  * the oracle restatement (oracle/oracle.c) built under AddressSanitizer +
    UndefinedBehaviorSanitizer (oracle/Makefile `asan`) and driven by its own
    tests (tests/test_oracle.py: the reference's known answers) through
    ORACLE_LIB, with libasan preloaded into the Python child;
  * the distributed sort's exact splitting (dr/details/split_plan.hpp, the
    body of drhip_split_windows / drhip_split_exact) on random runs;
  * the mhp message lists (dr/details/halo_plan.hpp: span_halo and
    dr_plan::exchange_plan) on 1-4 MPICH ranks.
UB aborts (-fno-sanitize-recover=all), so a finding fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
MPIEXEC = "/opt/conda/bin/mpiexec"


def _make(directory, *targets):
    r = subprocess.run(["make", "-s", "-C", directory, *targets], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def _libasan():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(p) or not os.path.exists(p):
        pytest.skip("gcc's libasan.so not found")
    return p


@pytest.fixture(scope="module")
def oracle_asan():
    _make(os.path.join(ROOT, "oracle"), "asan")
    lib = os.path.join(ROOT, "oracle", "_asan", "liboracle.so")
    env = dict(os.environ, ORACLE_LIB=lib, LD_PRELOAD=_libasan(),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return env


def test_sanitizer_is_live(oracle_asan):
    """The instrumented oracle does catch a heap overflow: a reduce told to
    read 4096 floats past a 4096-float buffer aborts with an ASan report
    (so the clean run below means something)."""
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, ctypes as C, oracle as O; L = O.lib(); "
            "x = np.ones(4096, np.float32); "
            "L.orc_reduce_exact_f32(x.ctypes.data_as(C.c_void_p), C.c_size_t(8192), C.c_double(0), 0)"
            % os.path.join(ROOT, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], env=oracle_asan, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "AddressSanitizer" in r.stderr, r.stderr[-2000:]


def test_oracle_known_answers_under_asan_ubsan(oracle_asan):
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle.py")],
                       env=oracle_asan, capture_output=True, text=True, timeout=600, cwd=ROOT)
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0 and "passed" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_split_plan_under_asan_ubsan():
    _make(CPP, "bin/asan/split_plan_test")
    r = subprocess.run([os.path.join(CPP, "bin", "asan", "split_plan_test"), "400"], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_halo_and_exchange_plans_under_asan_ubsan(nranks):
    if not os.path.exists(MPIEXEC):
        pytest.skip("MPICH (mpiexec) not present")
    _make(CPP, "bin/asan/halo_plan_mpi")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")  # MPICH's own allocations
    r = subprocess.run([MPIEXEC, "-n", str(nranks), os.path.join(CPP, "bin", "asan", "halo_plan_mpi")], env=env,
                       capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:], r.stderr[-2000:])
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "runtime error" not in r.stderr
