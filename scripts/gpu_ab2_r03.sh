cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec
RTMI_LIB=$V/cpasp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2_t_cpasp.log 2>&1
rc=$?; echo "cpasp full tests rc=$rc"; tail -n 2 gpurun_out/ab2_t_cpasp.log; [ $rc -ne 0 ] && exit $rc
RTMI_LIB=$V/cur.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg3 or cfg4 or nee" > gpurun_out/ab2_t_cur.log 2>&1
rc=$?; echo "cur tests rc=$rc"; tail -n 2 gpurun_out/ab2_t_cur.log; [ $rc -ne 0 ] && exit $rc
SETS="cornell:base,cur,cpa,csp,cpasp cfg3:base,cur cfg4:base,cur" ROUNDS=2 bash scripts/gpu_ab_sets.sh
