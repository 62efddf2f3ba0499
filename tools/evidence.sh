#!/bin/bash
# HEAD evidence in one GPU call (run on the gpurun box): GPU tests, the C1-C4 bench lines, the
# wavefront line, the rocprofv3 profile of the bench workload and the strong-scaling rehearsals.
#   bash tools/evidence.sh <tag>
# Writes gpurun_out/<step>.log and gpurun_out/prof_c4full_<tag>/; stops at the first crash or
# timeout (tools/gpu_check.sh).
tag="${1:?tag}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
exec_steps=(
    "tests:600:python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread"
    "bench_c4:300:python bench.py"
    "bench_c3:200:python bench.py --config c3"
    "bench_c2:200:python bench.py --config c2"
    "bench_c1:200:python bench.py --config c1"
    "bench_c4_wavefront:400:python bench.py --path wavefront"
    "profile:900:bash tools/profile.sh c4full_$tag --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-probe --no-count --no-strong-check"
    "reh_c4:300:python tools/scaling_rehearsal.py --config c4"
    "reh_c5:300:python tools/scaling_rehearsal.py --config c5 --spp 4096 --ns 1,8"
    "dispatch_c4:200:python bench.py --dispatch 30"
    "profile_dn:400:bash tools/profile.sh dn_$tag --dispatch 10 --dispatch-contexts 1"
)
bash tools/gpu_check.sh "${exec_steps[@]}"
