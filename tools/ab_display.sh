#!/bin/bash
# A/B of the display kernel (k_denoise_rows) across libraries: the display parity tests, then
# the per-pass DispatchRay timing (display_ms) of each.   usage: tools/ab_display.sh lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in cpppathtracer_amd/libcpt.so "$@"; do
    echo "### $lib"
    CPT_LIB_PATH=$PWD/$lib timeout -k 10 200 python -m pytest tests -q -m gpu -x \
        -k "display or golden or dispatch" 2>&1 | tail -n 1
    rc=${PIPESTATUS[0]}
    case $rc in 0|1|5) ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
    CPT_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --dispatch 20 --dispatch-contexts 1 2>/dev/null | tail -n 1 |
        python -c "import json,sys; d=json.loads(sys.stdin.read())['single']; print('display_ms', d['display_ms'], 'render_ms', d['render_ms']['median'], 'pass_ms', d['pass_ms']['median'])"
done
