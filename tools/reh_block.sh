#!/bin/bash
# Strong-scaling rehearsal over row-interleave block sizes (interleaved, R rounds): slowest / mean
# rank ms.   usage: R=2 BLOCKS="8 4 2 1" bash tools/reh_block.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 "${R:-2}"); do
  for b in ${BLOCKS:-8 4 2 1}; do
    for spec in ${SPECS:-c4:1024:2,4,8 c5:4096:8}; do
      IFS=: read -r cfg spp ns <<< "$spec"
      timeout -k 10 200 python tools/scaling_rehearsal.py --config "$cfg" --spp "$spp" --ns "$ns" --block "$b" 2>/dev/null | tail -n 1 |
        python -c "import json,sys; d=json.loads(sys.stdin.read())['results']; print('$r block=$b $cfg', ' '.join(f'N{n}={v[\"max_rank_ms\"]:.0f}/{v[\"mean_rank_ms\"]:.0f}' for n, v in d.items()))"
      rc=${PIPESTATUS[0]}
      [ "$rc" -eq 0 ] || { echo "rc=$rc ($cfg block $b)"; exit "$rc"; }
    done
  done
done
