#!/bin/bash
# A/B the kernel variants built under build/ab/ (CPT_LIB_PATH picks the library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args="${AB_ARGS:---spp 32 --steps 2 --warmup 1 --no-cpu-baseline}"
for lib in cpppathtracer_amd/libcpt.so build/ab/*.so; do
    echo "### $lib"
    CPT_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py $args | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], 'Mpaths/s', d['roofline']['kernel_avg_ms'], 'ms', d['roofline']['frac'])" || exit 1
done
