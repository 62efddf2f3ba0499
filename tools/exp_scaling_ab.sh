# Scaling rehearsal (tools/scaling_rehearsal.py) for every A/B library under build/ab/.
#   NS=4,8 bash tools/exp_scaling_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in cpppathtracer_amd/libcpt.so build/ab/*.so; do
  [ -e "$lib" ] || continue
  echo "### $lib"
  CPT_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/scaling_rehearsal.py --ns ${NS:-1,8} --reps ${REPS:-1} > gpurun_out/reh_$(basename $lib).log 2>&1 || exit $?
  tail -n 1 gpurun_out/reh_$(basename $lib).log
done
