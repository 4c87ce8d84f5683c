"""CPU: the C-ABI library loads without a GPU and exports every symbol include/rtmi355x.h declares;
without a gfx950 device rt_create fails loudly (RT_E_NODEVICE) — there is no CPU fallback."""
import ctypes as C
import re
from pathlib import Path

import pytest

from computational_ray_tracer_amd import capi

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    text = (ROOT / "include" / "rtmi355x.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(rt_\w+)\s*\(", text, re.M)))


def test_header_and_python_mirror_agree():
    assert header_symbols() == sorted(capi.EXPORTS)


def test_library_exports_every_symbol():
    lib = capi.load_library()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.rt_abi_version() == 1


def test_struct_sizes_match_header_layout():
    assert C.sizeof(capi.rt_pixel) == 16
    assert C.sizeof(capi.rt_sample_record) == 39 * 4
    assert C.sizeof(capi.rt_camera_desc) == 4 + 64 + 64 + 8


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = capi.load_library()
    h = C.c_void_p()
    rc = lib.rt_create(None, C.byref(h))
    assert rc == capi.RT_E_NODEVICE
    from computational_ray_tracer_amd.renderer import Renderer
    with pytest.raises(capi.RTError):
        Renderer()


def test_missing_library_is_loud(tmp_path):
    with pytest.raises(RuntimeError, match="missing"):
        capi.load_library(tmp_path / "nope.so")
