cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec
for v in rs9 mw; do
RTMI_LIB=$V/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg3 or cfg4 or nee or concurrent" > gpurun_out/ab1_t_$v.log 2>&1
rc=$?; echo "$v tests rc=$rc"; tail -n 2 gpurun_out/ab1_t_$v.log; [ $rc -ne 0 ] && exit $rc
done
for v in pa1 sp1 mw; do
RTMI_LIB=$V/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cornell or concurrent or shards or cfg0 or sensor" > gpurun_out/ab1_t_$v.log 2>&1
rc=$?; echo "$v tests rc=$rc"; tail -n 2 gpurun_out/ab1_t_$v.log; [ $rc -ne 0 ] && exit $rc
done
SETS="cornell:base,pa1,sp1,mw cfg4:base,rs9,mat1,mw cfg3:base,rs9,mw" ROUNDS=2 bash scripts/gpu_ab_sets.sh
