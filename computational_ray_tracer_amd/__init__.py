"""computational_ray_tracer_amd — MI355X-native (gfx950, HIP/CDNA4) implementation of the Monte Carlo
ray-tracing inner loop of GiboDidact/Computational_ray_tracer, behind a drop-in C-ABI (include/rtmi355x.h).

Layout:
  csrc/        HIP kernels (rt_kernels.hip, rt_device.h) + host C-ABI layer (rt_host.cpp) -> lib/librtmi355x.so
  capi.py      ctypes mirror of include/rtmi355x.h (loads the in-tree library; fails loudly if missing)
  scene.py     host-side scene descriptors (camera matrices, samplers, film, meshes, Cornell box, configs)
  renderer.py  Renderer: the RayTracerTestApp render-loop mirror over the C-ABI
"""
from . import capi, scene  # noqa: F401

__all__ = ["capi", "scene", "Renderer"]


def __getattr__(name):
    if name == "Renderer":
        from .renderer import Renderer
        return Renderer
    raise AttributeError(name)
