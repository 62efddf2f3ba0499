# A/B of sparse waves (CPT_MAX_LANES builds under build/ab/): per-block alone latency + N=8 rank 0
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in cpppathtracer_amd/libcpt.so build/ab/*.so; do
  echo "### $lib"
  CPT_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/chain_latency.py --spp 128 --ns 1,8 > gpurun_out/lat_$(basename $lib).log 2>&1 || exit $?
  tail -n 1 gpurun_out/lat_$(basename $lib).log | python -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['block_alone_ms']; print({k:v for k,v in b.items() if k!='all'}, d['rank0_full_gpu_ms'])"
done
