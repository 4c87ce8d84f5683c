#!/bin/bash
# A/B kernel variants with a parity gate: each variant .so runs the Cornell / golden GPU parity tests, then the bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for so in computational_ray_tracer_amd/lib/variants/*.so; do
  n=$(basename $so .so)
  RTMI_LIB=$PWD/$so timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "${PARITY_K:-cornell or golden or sobol or shards}" > gpurun_out/abp_$n.log 2>&1
  rc=$?; echo "$n parity rc=$rc $(tail -1 gpurun_out/abp_$n.log)"; [ $rc -ne 0 ] && exit $rc
done
bash scripts/gpu_ab.sh
