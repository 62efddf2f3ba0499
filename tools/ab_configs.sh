#!/bin/bash
# Interleaved A/B of the build/ab/ variants across configs (no parity pass: the caller has run
# it or the variant changes scheduling only).  AB_CONFIGS="c2 c4 ..."  AB_ROUNDS=2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${AB_ROUNDS:-2}"); do
  for c in ${AB_CONFIGS:-c2 c3 c4}; do
    case $c in c4|c3) st="${AB_C4_STEPS:---steps 2 --warmup 1}" ;; *) st="--steps 20 --warmup 5" ;; esac
    AB_NOTEST=1 AB_ARGS="--config $c $st --no-cpu-baseline --no-hbm-probe --no-count" bash tools/ab_bench.sh || exit $?
  done
done
