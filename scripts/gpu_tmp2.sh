cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for c in cfg3 cfg4; do
 echo "== $c"
 CASES="l2:RTMI_LANES=2 l1:RTMI_LANES=1 b4:RTMI_BATCH_SAMPLES=4194304 b16:RTMI_BATCH_SAMPLES=16777216" BENCH_ARGS="--config $c" BENCH_STEPS=1 bash scripts/gpu_ab_env.sh || exit 1
done
