cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for c in cfg3 cfg4; do
 echo "== $c"
 CASES="g1:RTMI_GRID_DIV=1 g2:RTMI_GRID_DIV=2 l3:RTMI_LANES=3" BENCH_ARGS="--config $c" BENCH_STEPS=1 bash scripts/gpu_ab_env.sh || exit 1
done
