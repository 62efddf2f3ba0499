#!/bin/bash
# ms per C4 frame at small spp (the DispatchRay regime: 1 spp per pass), to separate the
# per-launch cost and the frame's tail from the per-pass throughput: t(spp) = a + b * spp.
#   usage: tools/spp_sweep.sh [schedule]   (tiles | cost)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
sched="${1:-tiles}"
for s in 1 2 4 8 16 64; do
    timeout -k 10 120 python bench.py --spp $s --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-probe --no-count \
        --schedule "$sched" 2>/dev/null | tail -n 1 |
        python -c "import json,sys; d=json.loads(sys.stdin.read()); print('spp', $s, '$sched', d['ms_per_step'], 'ms/frame')"
    rc=${PIPESTATUS[0]}
    [ "$rc" -eq 0 ] || { echo "rc=$rc"; exit "$rc"; }
done
