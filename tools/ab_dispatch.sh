#!/bin/bash
# A/B of the per-pass DispatchRay loop across libraries (interleaved, R rounds): render_ms,
# display_ms and pass_ms medians of `bench.py --dispatch 20`.   usage: R=2 tools/ab_dispatch.sh lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${R:-2}"); do
    for lib in cpppathtracer_amd/libcpt.so "$@"; do
        CPT_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --dispatch 20 --dispatch-contexts 1 2>/dev/null | tail -n 1 |
            python -c "import json,sys; d=json.loads(sys.stdin.read())['single']; print('$r', '$lib', 'render', d['render_ms']['median'], 'display', d['display_ms']['median'], 'dev_only', d['display_device_only_ms']['median'], 'pass', d['pass_ms']['median'])"
        rc=${PIPESTATUS[0]}
        [ "$rc" -eq 0 ] || { echo "rc=$rc ($lib)"; exit "$rc"; }
    done
done
