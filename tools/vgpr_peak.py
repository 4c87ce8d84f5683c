#!/usr/bin/env python3
"""Where a kernel's VGPR allocation peaks: the instructions of a hipcc -S gfx950 listing that touch the highest
VGPRs (SGPR-spill lanes — v_writelane / v_readlane — excluded), with a few lines of context each.

  hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 -std=c++17 -ffp-contract=off -fno-fast-math \\
        -munsafe-fp-atomics computational_ray_tracer_amd/csrc/rt_kernels.hip -o /tmp/rtk.s
  python3 tools/vgpr_peak.py /tmp/rtk.s k_path_shadeILi1 [top=3] [context=12]
"""
import re
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ctx = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    lines, on = [], False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*" + re.escape(kern) + r"\S*:", ln):
            on = True
        elif on and ln.startswith(".Lfunc_end"):
            break
        if on:
            lines.append(ln.rstrip("\n"))

    def vmax(s):
        m = -1
        for a in re.findall(r"\bv(\d+)\b", s):
            m = max(m, int(a))
        for _, b in re.findall(r"v\[(\d+):(\d+)\]", s):
            m = max(m, int(b))
        return m

    use = [(vmax(s), i) for i, s in enumerate(lines) if not s.strip().startswith(("v_writelane", "v_readlane", ";"))]
    hi = sorted({v for v, _ in use}, reverse=True)[:top]
    print(f"{kern}: {len(lines)} lines, highest VGPRs {hi}")
    shown = set()
    for v in hi:
        for vv, i in use:
            if vv == v and not any(abs(i - j) < ctx for j in shown):
                shown.add(i)
                print(f"--- v{v} at line {i}")
                print("\n".join(lines[max(0, i - ctx): i + 3]))


if __name__ == "__main__":
    main()
