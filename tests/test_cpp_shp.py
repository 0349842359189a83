"""The C++ shp drop-in layer (distributed-ranges_amd/include/dr/shp.hpp):
the reference's shp gtests restated in tests/cpp/shp_tests.cpp, run on the
default device list and with --devicesCount 3 (three segments duplicated on
one GPU), exactly as the reference registers `shp` and `shp-3`
(test/gtest/shp/CMakeLists.txt:28-30)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "bin", "shp_tests")


def test_cpp_tests_built():
    """build() compiles the C++ layer + tests with hipcc for gfx950."""
    assert os.path.exists(BIN), "run __graft_entry__.build() (make -C tests/cpp)"


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [0, 1, 2, 3, 4, 8])
def test_cpp_shp_suite(devices):
    args = [BIN] + (["--devicesCount", str(devices)] if devices else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    print(r.stdout[-6000:])
    print(r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [0, 3])
def test_cpp_shp_suite_epoch_wrap(devices):
    """The suite built with the template scan's status epoch wrapping every 3
    calls (DR_SHP_LB_EPOCH_MAX=3): the status buffer's clear on wrap and the
    epoch restart run between most scans."""
    exe = os.path.join(ROOT, "tests", "cpp", "bin", "shp_tests_epoch3")
    r = subprocess.run([exe] + (["--devicesCount", str(devices)] if devices else []), capture_output=True, text=True,
                       timeout=300)
    print(r.stdout[-6000:])
    print(r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


def _visible_gpus():
    import drhip
    drhip.load()
    return drhip.device_count()


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", ["distinct", "alternating"])
def test_cpp_shp_suite_distinct_devices(pattern):
    """The same suite with segments on DIFFERENT GPUs (--devices 0,1,...):
    peer copies of sort pieces, misaligned zipped scan pieces written across
    devices, pool access granted to peers, gemv's x replication.  Needs >= 2
    visible GPUs (skipped on a one-GPU box; the driver's 8-GPU node runs it).
    "alternating" puts two segments on each of two GPUs (0,1,0,1)."""
    n = _visible_gpus()
    if n < 2:
        pytest.skip(f"{n} GPU visible: distinct-device segments need >= 2")
    ids = list(range(n)) if pattern == "distinct" else [0, 1, 0, 1]
    r = subprocess.run([BIN, "--devices", ",".join(map(str, ids))], capture_output=True, text=True, timeout=300)
    print(r.stdout[-6000:])
    print(r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


MHP_BIN = os.path.join(ROOT, "tests", "cpp", "bin", "mhp_tests")


def test_cpp_mhp_tests_built():
    assert os.path.exists(MHP_BIN), "run __graft_entry__.build() (make -C tests/cpp)"


@pytest.mark.gpu
def test_cpp_mhp_suite():
    """dr/mhp.hpp (one process per GPU over the RCCL C-ABI): the reference's
    MhpTests.Reduce / MhpTests.Stencil known answers and the stencil-1d
    example, one rank."""
    r = subprocess.run([MHP_BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout[-6000:])
    print(r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


MPIEXEC = "/opt/conda/bin/mpiexec"
MHP_MPI_BIN = os.path.join(ROOT, "tests", "cpp", "bin", "mhp_tests_mpi")
PLAN_BIN = os.path.join(ROOT, "tests", "cpp", "bin", "halo_plan_mpi")


def _mpirun(binary, nranks, *args, timeout=240):
    if not os.path.exists(MPIEXEC):
        pytest.skip("MPICH (mpiexec) not present")
    if not os.path.exists(binary):
        pytest.fail(f"{binary} not built (make -C tests/cpp)")
    return subprocess.run([MPIEXEC, "-n", str(nranks), binary, *args], capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_halo_plan_over_mpi_cpu(nranks):
    """The mhp message sequence (dr/details/halo_plan.hpp -- what the RCCL
    halo exchange and the MPI transport both issue) on 1-4 MPICH ranks with
    host buffers: MhpTests.Reduce -> 1045, MhpTests.Stencil, the stencil-1d
    example and larger stencils against a serial loop, periodic halos, and
    the in-order send/receive pairing RCCL relies on.  The reference runs
    its mhp suite on the same rank counts (test/gtest/mhp/CMakeLists.txt:27-33)."""
    r = _mpirun(PLAN_BIN, nranks)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_cpp_mhp_suite_mpi_ranks(nranks):
    """dr/mhp.hpp itself on 1-4 ranks (mpiexec), every rank a process with
    its own segment: halo exchange, mhp::reduce's gather, the
    distributed_vector(n, halo_bounds) layout across ranks, and the
    reference's MhpTests Fill / ForEach / Copy / Transform / Subrange / Zip /
    Take / Drop / TransformView / DistributedVector* / IteratorConformance
    (misaligned copies through the alltoallv exchange), with the
    reference's MPI transport (dr/mhp_mpi.hpp) so the ranks may share the
    box's one GPU; the known answers are the reference tests' own."""
    r = _mpirun(MHP_MPI_BIN, nranks, "--transport", "mpi")
    print(r.stdout[-6000:], r.stderr[-2000:])
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.count("[  OK  ]") == 17 * nranks  # the 17 restated tests, every rank


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_cpp_mhp_suite_rccl_ranks(nranks):
    """The same suite with one rank per GPU over RCCL (the production
    transport; the communicator id travels by MPI_Bcast).  Needs nranks
    visible GPUs (skipped on a one-GPU box)."""
    n = _visible_gpus()
    if n < nranks:
        pytest.skip(f"{n} GPU(s) visible: {nranks} RCCL ranks need {nranks}")
    r = _mpirun(MHP_MPI_BIN, nranks, "--transport", "rccl")
    print(r.stdout[-6000:], r.stderr[-2000:])
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_c5_mhp_stencil1d_2pow32_eight_ranks():
    """C5 at its configured size through dr/mhp.hpp: examples/mhp/
    stencil-1d.cpp:16-66 on mhp::distributed_vector<float>(2^32,
    halo_bounds(1)) over 8 MPI ranks sharing the box's GPU (the reference's
    MPI transport, dr/mhp_mpi.hpp), 3 steps of span_halo exchange
    (details/halo.hpp:336-387) + mhp::transform.  Every rank checks the
    cells within 4096 of its segment edges and of 64 global random windows,
    bit-exact against a serial fp32 simulation of the same slab."""
    import json
    r = _mpirun(MHP_MPI_BIN, 8, "--transport", "mpi", "--c5", "32", "3", timeout=900)
    print(r.stdout[-4000:], r.stderr[-2000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(line[-1])
    assert res["cells"] == 1 << 32 and res["ranks"] == 8 and res["steps"] == 3
    assert res["cells_checked"] >= 8 * 2 * 4096 and res["cell_mismatches"] == 0
    assert res["ok"] and r.returncode == 0
