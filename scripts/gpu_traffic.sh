#!/bin/bash
# PMC traffic of one config under given runtime options / library, single lane, each counter pass its own run:
#   CFG=cfg3 TAG=nosort ENVS="RTMI_SORT=0" [LIB=variants/x.so] [LANES=2] [KT_ONLY=1] bash scripts/gpu_traffic.sh
# -> gpurun_out/traffic_<cfg>_<tag>.txt: per kernel, FETCH_SIZE KiB (raw), WRITE_SIZE KiB and the kernel time.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFG=${CFG:-cfg3}; TAG=${TAG:-t}; D=gpurun_out/traffic_${CFG}_$TAG
L=(); [ -n "$LIB" ] && L=(RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/$LIB RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec)
B="python3 bench.py --config $CFG --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --project-shards 0 $BENCH_ARGS"
for c in $([ -z "$KT_ONLY" ] && echo FETCH_SIZE WRITE_SIZE); do
  env RTMI_LANES=${LANES:-1} "${L[@]}" $ENVS timeout -s KILL 240 rocprofv3 --pmc $c -d $D/$c -o pmc --output-format csv -- $B > $D.$c.log 2>&1
  rc=$?; echo "$CFG $TAG $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D.$c.log; exit $rc; }
done
env RTMI_LANES=${LANES:-1} "${L[@]}" $ENVS timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- $B > $D.kt.log 2>&1
rc=$?; echo "$CFG $TAG kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
[ -z "$KT_ONLY" ] && python3 tools/pmc_summary.py $D/FETCH_SIZE/*counter_collection.csv $D/WRITE_SIZE/*counter_collection.csv > $D.txt
python3 -c "
import csv,glob
for f in glob.glob('$D/kt/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)): print('time', r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
" >> $D.txt
grep -E "trace|shade|nee|time" $D.txt | cut -c1-200
exit 0
