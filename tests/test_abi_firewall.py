"""The C-ABI's exception firewall (SURVEY §8b Errors: no C++ exception crosses the boundary; rt_guard.h).

RTMI_FAULT_INJECT makes every guarded entry point throw inside its firewall; the call must come back with a
negative status (std::bad_alloc -> RT_E_OOM, anything else -> RT_E_STATE) instead of terminating the process.
The CPU tests use the host-only entry points and rt_create (which throws before it looks for a device); the GPU
test injects into a live context and checks it stays usable.
"""
import ctypes as C

import numpy as np
import pytest

from computational_ray_tracer_amd import capi

CASES = [("bad_alloc", capi.RT_E_OOM), ("system_error", capi.RT_E_STATE), ("runtime", capi.RT_E_STATE),
         ("other", capi.RT_E_STATE)]


@pytest.fixture
def lib():
    return capi.load_library()


@pytest.mark.parametrize("kind,code", CASES)
def test_host_entry_points_return_status(lib, monkeypatch, tmp_path, kind, code):
    rgb = (C.c_float * 3)(0.2, 0.5, 0.7)
    coeffs = (C.c_float * 3)()
    obj = tmp_path / "tri.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    img = np.zeros((2, 2, 3), np.uint8)
    monkeypatch.setenv("RTMI_FAULT_INJECT", kind)
    assert lib.rt_rgb_to_sigmoid(rgb, coeffs) == code
    mesh = C.POINTER(capi.rt_mesh)()
    assert lib.rt_load_obj(str(obj).encode(), C.byref(mesh)) == code
    assert not mesh  # nothing allocated, nothing leaked to the caller
    assert lib.rt_image_write(str(tmp_path / "x.png").encode(), 2, 2,
                              img.ctypes.data_as(C.POINTER(C.c_uint8)), 0) == code
    ctx = C.c_void_p()
    opt = capi.rt_options()
    assert lib.rt_create(C.byref(opt), C.byref(ctx)) == code
    assert not ctx
    lib.rt_destroy(None)       # the release entry points are exempt from the injection (NULL: no-op)
    lib.rt_mesh_free(None)
    monkeypatch.delenv("RTMI_FAULT_INJECT")
    assert lib.rt_rgb_to_sigmoid(rgb, coeffs) == capi.RT_OK
    assert lib.rt_load_obj(str(obj).encode(), C.byref(mesh)) == capi.RT_OK
    assert mesh.contents.n_triangles == 1
    lib.rt_mesh_free(mesh)


@pytest.mark.gpu
def test_context_survives_injected_fault(monkeypatch):
    from computational_ray_tracer_amd import scene
    from computational_ray_tracer_amd.renderer import Renderer
    from oracle.oracle import OracleScene

    cfg = scene.cfg_cornell(res=(16, 16), spp_side=2)
    r = Renderer(cfg, device=0)
    lib = capi.load_library()
    sd = cfg.model.desc()
    monkeypatch.setenv("RTMI_FAULT_INJECT", "bad_alloc")
    assert lib.rt_scene_upload(r.h, C.byref(sd)) == capi.RT_E_OOM
    assert b"bad_alloc" in lib.rt_last_error(r.h)
    monkeypatch.setenv("RTMI_FAULT_INJECT", "system_error")
    st = capi.rt_stats()
    assert lib.rt_get_stats(r.h, C.byref(st)) == capi.RT_E_STATE
    assert b"system error" in lib.rt_last_error(r.h)
    monkeypatch.delenv("RTMI_FAULT_INJECT")
    film = r.render_pass(0, 4)
    ref = OracleScene(cfg).render(0, 4)
    assert np.array_equal(film.view(np.uint32), ref.view(np.uint32))
