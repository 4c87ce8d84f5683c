"""CPU: sanitizer builds (SURVEY §5 "race detection / memory checking" row).  tests/sanitize/Makefile builds the
oracle (oracle/rtcore_capi.cpp) with ASan + UBSan and with TSan, and the host-only C-ABI entry points (rt_load_obj,
rt_mesh_free, rt_image_write, rt_rgb_to_sigmoid, rt_rgb_fit_sigmoid; csrc/rt_io.cpp, csrc/rt_color.cpp) with
ASan + UBSan, as standalone executables (no preloading into Python).  The oracle driver renders with the reference,
path and MIS integrators on 4 threads over a multi-level octree and runs the canonical-rule check on 4 threads; the
host driver feeds valid and malformed OBJ files, writes PNG/PPM images, looks up the RGB table and trips the
exception firewall.  Any sanitizer report aborts the driver (non-zero exit) and fails the test."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SAN = ROOT / "tests" / "sanitize"
TABLE = ROOT / "computational_ray_tracer_amd" / "data" / "srgb64.rgbspec"
REPORTS = ("AddressSanitizer", "runtime error:", "ThreadSanitizer", "LeakSanitizer")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-j3"], cwd=SAN, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return SAN / "_build"


def _run(exe, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("ASAN_OPTIONS", "detect_leaks=1:abort_on_error=0")
    e.setdefault("TSAN_OPTIONS", "halt_on_error=1")
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, env=e)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and not any(s in out for s in REPORTS), out[-6000:]
    return out


@pytest.mark.parametrize("flavour", ["asan", "tsan"])
def test_oracle_under_sanitizer(built, flavour):
    out = _run(built / f"oracle_{flavour}")
    assert out.count("integrator") == 3


def test_host_abi_under_asan(built, tmp_path):
    assert TABLE.exists(), "RGB table missing: run __graft_entry__.build() (or make -C computational_ray_tracer_amd/csrc)"
    _run(built / "host_abi_asan", str(tmp_path), env={"RTMI_RGBSPEC_TABLE": str(TABLE)})
