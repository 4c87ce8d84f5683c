#!/bin/bash
# r04 ab3: BVH build quality (tools/bvh_quality.py on the CPU: 64 SAH bins and a lower node cost cut the CFG3 bounce
# rays' node visits 5.45 -> 4.70 and triangle tests 7.2 -> 5.9-6.1) on the GPU:
#   def   16 bins, SAH node cost 3 (round 3's build)        b64   64 bins (the default build), +RTMI_BVH_CI=2.5 / 2
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sort.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab3_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab3_t.log; [ $rc -ne 0 ] && exit $rc
SETS="cfg3:def,b64,b64+RTMI_BVH_CI=2.5,b64+RTMI_BVH_CI=2 cfg4:def,b64,b64+RTMI_BVH_CI=2.5,b64+RTMI_BVH_CI=2" ROUNDS=2 bash scripts/gpu_ab_sets.sh
