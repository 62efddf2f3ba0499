#!/bin/bash
# Interleaved A/B of the libraries named on the command line (ABAB... R rounds) at the bench
# workload: run-to-run drift on one box is about 2%, so single runs cannot rank variants that
# close.  usage: R=3 tools/ab_interleave.sh lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args="${AB_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-count}"
for r in $(seq 1 "${R:-3}"); do
    for lib in "$@"; do
        CPT_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py $args > /tmp/ab_out.txt 2>&1
        rc=$?
        [ $rc -eq 0 ] || { echo "bench rc=$rc ($lib)"; tail -n 5 /tmp/ab_out.txt; exit $rc; }
        tail -n 1 /tmp/ab_out.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$lib', d['value'], 'Mpaths/s', d['ms_per_step'], 'ms/step')"
    done
done
