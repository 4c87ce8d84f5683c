cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for c in cfg3; do
 echo "== $c"
 CASES="inl:RTMI_LIB=/root/repo/computational_ray_tracer_amd/lib/variants/w0.so,RTMI_SHADOW_QUEUE=0 qbfs:RTMI_LIB=/root/repo/computational_ray_tracer_amd/lib/variants/w0.so,RTMI_SHADOW_QUEUE=1,RTMI_SHADOW_DFS=0 qdfs:RTMI_LIB=/root/repo/computational_ray_tracer_amd/lib/variants/w0.so,RTMI_SHADOW_QUEUE=1,RTMI_SHADOW_DFS=1 qbfs4:RTMI_LIB=/root/repo/computational_ray_tracer_amd/lib/variants/w4.so,RTMI_SHADOW_QUEUE=1,RTMI_SHADOW_DFS=0 qdfs4:RTMI_LIB=/root/repo/computational_ray_tracer_amd/lib/variants/w4.so,RTMI_SHADOW_QUEUE=1,RTMI_SHADOW_DFS=1" BENCH_ARGS="--config $c" BENCH_STEPS=1 bash scripts/gpu_ab_env.sh || exit 1
done
