#!/bin/bash
# A/B of the strong-scaling rehearsal across libraries (interleaved, R rounds): slowest-rank ms
# per N for C4 (N = 1, 2, 4, 8) and C5 (N = 8).   usage: R=1 tools/ab_rehearsal.sh lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${R:-1}"); do
    for lib in cpppathtracer_amd/libcpt.so "$@"; do
        for spec in "c4:1024:1,2,4,8" "c5:4096:8"; do
            IFS=: read -r cfg spp ns <<< "$spec"
            CPT_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/scaling_rehearsal.py --config "$cfg" --spp "$spp" --ns "$ns" 2>/dev/null | tail -n 1 |
                python -c "import json,sys; d=json.loads(sys.stdin.read())['results']; print('$r', '$lib', '$cfg', ' '.join(f'N{n}={v[\"max_rank_ms\"]:.0f}' for n, v in d.items()))"
            rc=${PIPESTATUS[0]}
            [ "$rc" -eq 0 ] || { echo "rc=$rc ($lib $cfg)"; exit "$rc"; }
        done
    done
done
