cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/variants/b_pre.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_pre.log 2>&1
rc=$?; echo "pytest(pre) rc=$rc"; tail -3 gpurun_out/pt_pre.log; [ $rc -ne 0 ] && exit $rc
CFGS="cfg4" bash scripts/gpu_tmp.sh
