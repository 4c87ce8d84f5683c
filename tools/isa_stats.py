#!/usr/bin/env python3
"""Per-kernel instruction mix of a hipcc -S gfx950 assembly file (static counts), including the scratch (spill)
loads / stores.

  hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
        computational_ray_tracer_amd/csrc/rt_kernels.hip -o /tmp/rtk.s && python3 tools/isa_stats.py /tmp/rtk.s
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    ins = []
    for l in body.split("\n"):
        t = l.strip()
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        ins.append(t.split()[0])
    c = collections.Counter(ins)
    f64 = sum(v for k, v in c.items() if "f64" in k)
    vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_", "scratch_")))
    smem = sum(v for k, v in c.items() if k.startswith("s_load") or k.startswith("s_buffer_load"))
    sst = sum(v for k, v in c.items() if k.startswith("scratch_store") or k.startswith("buffer_store") and "off" in k)
    sld = sum(v for k, v in c.items() if k.startswith("scratch_load"))
    print(f"{name[:70]:70s} n={len(ins):5d} scratch_st={sst:4d} scratch_ld={sld:4d} f64={f64:4d} vmem={vmem:4d} smem={smem:3d} "
          f"div_scale={c.get('v_div_scale_f32', 0):3d} sqrt={c.get('v_sqrt_f32', 0):3d} cndmask={c.get('v_cndmask_b32_e64', 0) + c.get('v_cndmask_b32_e32', 0):4d}")
