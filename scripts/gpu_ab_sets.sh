#!/bin/bash
# Interleaved A/B of kernel variants (lib/variants/<name>.so) with optional runtime options, per config, on one box:
#   SETS="cornell:base,pa1 cfg4:base,rs9,rs9+RTMI_SORT_NEE=1/6" ROUNDS=2 bash scripts/gpu_ab_sets.sh
# An item is <variant>[+ENV=value...]; each (round, config, item) is one bench process and one line.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec  # variants live one level deeper
for r in $(seq 1 ${ROUNDS:-2}); do
  for set in $SETS; do
    c=${set%%:*}
    s=${AB_STEPS:-2}; [ $c = cornell ] && s=${AB_STEPS_CORNELL:-6}
    for item in $(echo ${set#*:} | tr ',' ' '); do
      v=${item%%+*}; envs=""; [ "$item" != "$v" ] && envs=$(echo ${item#*+} | tr '+' ' ')
      tag=$(echo "${c}_${item}" | tr '/+=' '___')
      env RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/variants/$v.so $envs timeout -k 10 300 \
        python bench.py --config $c --steps $s --warmup 1 --no-cpu-baseline --project-shards 0 > gpurun_out/abs_${tag}_$r.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "$c $item rc=$rc"; tail -3 gpurun_out/abs_${tag}_$r.log; exit $rc; }
      python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/abs_${tag}_$r.log') if x.startswith('{')][-1])
print('round $r', '$c', '$item', d['value'], d['stage_ms'])"
    done
  done
done
exit 0
