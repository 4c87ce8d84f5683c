#!/bin/bash
# Parallel A/B variant builds: only rt_kernels.hip is recompiled per variant, the other objects come from the main
# build (make first).   [KRES=<part of a mangled kernel name>] bash scripts/build_variants.sh "nokz:-DRT_TRACE_KZ=0" ...
cd "$(dirname "$0")/../computational_ray_tracer_amd/csrc" || exit 1
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -Wno-unused-variable -Wno-unused-value -munsafe-fp-atomics"
mkdir -p ../lib/variants
OTHERS=$(ls ../lib/obj/*.o | grep -v rt_kernels)
for v in "$@"; do
  n=${v%%:*}; d=$(echo ${v#*:} | tr ',' ' ')
  ( /opt/rocm/bin/hipcc $FLAGS $d -c rt_kernels.hip -o /tmp/rtk_$n.o -Rpass-analysis=kernel-resource-usage 2> /tmp/rtk_$n.log &&
    /opt/rocm/bin/hipcc $FLAGS -shared -o ../lib/variants/$n.so /tmp/rtk_$n.o $OTHERS &&
    echo "$n: $(grep -A10 "Function Name: .*${KRES:-k_trace_closestILi0ELb1}" /tmp/rtk_$n.log | head -11 | grep -oE '(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): [0-9]+' | tr '\n' ' ')" ) &
done
wait
