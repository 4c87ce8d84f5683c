#!/bin/bash
# r03: per-sort radix digit widths (ray key 2 passes of 9 bits, NEE key 3 passes of 8) against 8-bit digits for both;
# the single-leaf pair append with double-buffered LDS counters (2 barriers per pair instead of 3)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec
for v in rsx db1; do
RTMI_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab7_t_$v.log 2>&1
rc=$?; echo "$v tests rc=$rc"; tail -n 2 gpurun_out/ab7_t_$v.log; [ $rc -ne 0 ] && exit $rc
done
SETS="cornell:b0,db1 cfg3:b0,rsx cfg4:b0,rsx" ROUNDS=3 bash scripts/gpu_ab_sets.sh
