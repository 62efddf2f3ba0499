#!/bin/bash
# A/B the kernel variants built under build/ab/ (CPT_LIB_PATH picks the library): each
# variant first passes the bit-exact render parity subset, then runs the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args="${AB_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-count}"
for lib in cpppathtracer_amd/libcpt.so build/ab/*.so; do
    [ -e "$lib" ] || continue
    echo "### $lib"
    if [ -z "${AB_NOTEST:-}" ]; then
        CPT_LIB_PATH=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x \
            -k "render_bitexact or single_object or tiny_depths or empty_scene" 2>&1 | tail -n 1
        rc=${PIPESTATUS[0]}
        case $rc in 0) ;; 1) echo "parity failed: no bench for $lib"; continue ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
    fi
    CPT_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py $args > /tmp/ab_out.txt 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -n 5 /tmp/ab_out.txt; exit $rc; }
    tail -n 1 /tmp/ab_out.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'Mpaths/s', d['ms_per_step'], 'ms/step', d['config']['workload'], d['config']['schedule'])"
done
