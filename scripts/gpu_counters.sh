#!/bin/bash
# Single-lane (RTMI_LANES=1) rocprofv3 passes of bench.py per config: kernel trace + stats, FETCH_SIZE, WRITE_SIZE,
# and the SQ instruction / stall mix — each in a run of its own (never combined with other tracing) — then
# tools/counters.py -> profiles/counters_<config>.json and the bench line itself.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
for c in ${CONFIGS:-cornell cfg3 cfg4}; do
  D=gpurun_out/cnt_${c}_$TAG
  B="python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --project-shards 0"
  RTMI_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- $B > $D.kt.log 2>&1
  rc=$?; echo "$c kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
  RTMI_LANES=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o pmc --output-format csv -- $B > $D.fetch.log 2>&1
  rc=$?; echo "$c fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
  RTMI_LANES=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $D/write -o pmc --output-format csv -- $B > $D.write.log 2>&1
  rc=$?; echo "$c write rc=$rc"; [ $rc -ne 0 ] && exit $rc
  RTMI_LANES=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $D/sq -o pmc --output-format csv -- $B > $D.sq.log 2>&1
  rc=$?; echo "$c sq rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/counters.py --config $c --tag $TAG --dir $D --out $D.counters.json > /dev/null || exit 1
done
exit 0
