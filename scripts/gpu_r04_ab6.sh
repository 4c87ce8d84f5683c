#!/bin/bash
# r04 ab6: k_path_pixel (the Cornell box's whole path per pixel thread, state in registers) against the wavefront
# kernels (RTMI_PIXEL_PATH=0), at 4 / 3 / 2 waves per SIMD (pw4 = the default build).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cornell or camera or sobol or independent or multi_device or full_size or concurrent or shards" > gpurun_out/r04ab6_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 gpurun_out/r04ab6_t.log; [ $rc -ne 0 ] && exit $rc
RTMI_AB_COMPAT=1 SETS="cornell:pw4+RTMI_PIXEL_PATH=0,pw4,pw3,pw2" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
