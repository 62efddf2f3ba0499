cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/chain_latency.py --spp 128 > gpurun_out/chain_latency.log 2>&1 || exit $?
tail -n 1 gpurun_out/chain_latency.log | cut -c1-600
for lib in cpppathtracer_amd/libcpt.so build/ab/*.so; do
  echo "### $lib"
  CPT_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/scaling_rehearsal.py --ns 1,8 > gpurun_out/reh_$(basename $lib).log 2>&1 || exit $?
  tail -n 1 gpurun_out/reh_$(basename $lib).log
done
