#!/bin/bash
# A/B the kernel variants in computational_ray_tracer_amd/lib/variants/*.so (interleaved rounds, one process each).
cd "$GRAFT_REPO_ROOT"
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec  # variants live one level deeper
mkdir -p gpurun_out
for round in 1 2; do
  for so in computational_ray_tracer_amd/lib/variants/*.so; do
    n=$(basename $so .so)
    RTMI_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$n.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; exit $rc; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ab_$n.log') if x.startswith('{')][-1])
print('round $round', '$n', d['value'], d['stage_ms'])"
  done
done
