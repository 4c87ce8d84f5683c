#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access shape (tools/fetch_calib.hip, built in tools/_build by
# __graft_entry__.build): one PMC pass per counter, then tools/fetch_calib_summary.py -> gpurun_out/calib_<TAG>.json
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-calib}; D=gpurun_out/calib_$TAG
timeout -k 10 60 tools/_build/fetch_calib > $D.bytes.txt 2>&1; rc=$?; echo "calib run rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $c -d $D/$n -o pmc --output-format csv -- tools/_build/fetch_calib > $D.$n.log 2>&1
  rc=$?; echo "calib $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D.$n.log; exit $rc; }
done
python3 tools/fetch_calib_summary.py $D > $D.json && cat $D.json
