#!/bin/bash
# The DispatchRay regime (1 spp per pass, C4 1920x1080): ms per frame of the render variants,
# to pick the per-pass kernel configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
    timeout -k 10 120 python bench.py --spp 1 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-probe --no-count "$@" \
        2>/dev/null | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], 'ms/frame')"
    rc=${PIPESTATUS[0]}
    [ "$rc" -eq 0 ] || { echo "rc=$rc ($*)"; exit "$rc"; }
}
run --schedule tiles
run --schedule cost
run --schedule tiles --walk reference
run --path wavefront
run --schedule tiles --spp 2
