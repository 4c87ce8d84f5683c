#!/bin/bash
# Interleaved A/B of kernel variants (lib/variants/<name>.so) with optional runtime options, per config, on one box:
#   SETS="cornell:base,pa1 cfg4:base,rs9,rs9+RTMI_SORT_NEE=1/6" ROUNDS=2 bash scripts/gpu_ab_sets.sh
#   AB=r04_ab13 bash scripts/gpu_ab_sets.sh            (a recorded experiment: scripts/ab_history.tsv)
# An item is <variant>[+ENV=value...]; each (round, config, item) is one bench process and one line.
# TESTS="<pytest -k expression>" or "all" runs the -m gpu suite first, once per variant in TEST_VARIANTS (default: the
# default library), and stops there on a failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec  # variants live one level deeper
V=$PWD/computational_ray_tracer_amd/lib/variants
if [ -n "$AB" ]; then
  row=$(awk -F'\t' -v id="$AB" '$1 == id' scripts/ab_history.tsv)
  [ -z "$row" ] && { echo "no A/B '$AB' in scripts/ab_history.tsv"; exit 2; }
  IFS=$'\t' read -r _ ROUNDS TESTS ABENV SETS _ <<< "$row"
  [ "$TESTS" = "-" ] && TESTS=""
  [ "$ABENV" != "-" ] && export $ABENV
fi
if [ -n "$TESTS" ]; then
  K=(); [ "$TESTS" != "all" ] && K=(-k "$TESTS")
  for tv in ${TEST_VARIANTS:-default}; do
    L=(); [ "$tv" != "default" ] && L=(env RTMI_LIB=$V/$tv.so)
    "${L[@]}" timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" \
      > gpurun_out/abt_$tv.log 2>&1
    rc=$?; echo "$tv tests rc=$rc"; tail -n 2 gpurun_out/abt_$tv.log; [ $rc -ne 0 ] && exit $rc
  done
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for set in $SETS; do
    c=${set%%:*}
    s=${AB_STEPS:-2}; [ $c = cornell ] && s=${AB_STEPS_CORNELL:-6}
    for item in $(echo ${set#*:} | tr ',' ' '); do
      v=${item%%+*}; envs=""; [ "$item" != "$v" ] && envs=$(echo ${item#*+} | tr '+' ' ')
      tag=$(echo "${c}_${item}" | tr '/+=' '___')
      env RTMI_LIB=$V/$v.so $envs timeout -k 10 300 \
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
