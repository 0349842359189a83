"""Measurement builds of libdrhip compile (CPU-side, no GPU).

tools/build_variant.sh and the A/B scripts under tools/ rebuild single
kernels with -D knobs (tile sizes, look-back width, ...).  A round-3
measurement build with DRHIP_SCAN_UBIG=16 made the scan launcher recurse
into its own instantiation (undefined behaviour that faulted the GPU).  The
launcher now picks the tile size once, in scan_dispatch (csrc/scan.hip), so
no instantiation calls itself; this test compiles the host side of every
knob value the tools use, and the device side of the scan knob that faulted,
so a variant that does not build (or reintroduces a launcher that names its
own instantiation) is caught here before it reaches the GPU box."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-ranges_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-parameter",
         "-munsafe-fp-atomics", "-ffp-contract=off"]

KNOBS = [
    ("scan.hip", ["-DDRHIP_SCAN_UBIG=16"]),
    ("scan.hip", ["-DDRHIP_SCAN_UBIG=32"]),
    ("scan.hip", ["-DDRHIP_WAVE_GIVEN_CLAIM=0", "-DDRHIP_TILES_UBIG=8"]),
    ("scan.hip", ["-DDRHIP_WAVE_GIVEN_CLAIM=1", "-DDRHIP_TILES_U=4"]),
    ("sort.hip", ["-DDRHIP_SORT_OS_LOOK=2"]),
    ("sort.hip", ["-DDRHIP_SORT_OS_LOOK=8"]),
    ("sort.hip", ["-DDRHIP_SORT_H0_CNT1=0"]),
    ("sort.hip", ["-DDRHIP_SORT_CNT_WO=0"]),
    ("sort.hip", ["-DDRHIP_SORT_STAMPS"]),
    ("sort.hip", ["-DDRHIP_SORT_P0_ONESHOT=1"]),
    ("spmv.hip", ["-DDRHIP_SPMV_XW=0"]),
    ("stencil.hip", ["-DDRHIP_ST2D_LDSE=0"]),
]

need_hipcc = pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="no hipcc")


def _compile(src, defs, tmp_path, side):
    out = tmp_path / (src + side + ".o")
    cmd = [HIPCC, *FLAGS, *defs, side, "-c", os.path.join(CSRC, src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


@need_hipcc
@pytest.mark.parametrize("src,defs", KNOBS, ids=[f"{s}:{' '.join(d)}" for s, d in KNOBS])
def test_knob_variant_host_builds(src, defs, tmp_path):
    _compile(src, defs, tmp_path, "--offload-host-only")


@need_hipcc
def test_scan_knob_device_builds(tmp_path):
    _compile("scan.hip", ["-DDRHIP_SCAN_UBIG=16"], tmp_path, "--offload-device-only")


def test_scan_launcher_never_names_itself():
    """No launch_scan body calls launch_scan: the size-based tile choice
    lives in scan_dispatch only."""
    src = open(os.path.join(CSRC, "scan.hip")).read()
    m = re.search(r"static int launch_scan\(.*?\n}\n", src, re.S)
    assert m, "launch_scan not found"
    body = m.group(0).split("{", 1)[1]
    assert "launch_scan" not in body
