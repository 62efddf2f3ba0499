#!/bin/bash
# i-cache behaviour of the timed megakernel (46 KB of code): the SQC instruction-cache counters on
# a short C4 render (64 spp).  Writes gpurun_out/icache/.  Run on the gpurun box.
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/icache"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
rocprofv3 --list-avail > "$out/avail.txt" 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*" "$out/avail.txt" | sort -u > "$out/icache_counters.txt" || true
cat "$out/icache_counters.txt"
ctrs=$(grep -E "^SQC_ICACHE_(HITS|MISSES|REQ)$" "$out/icache_counters.txt" | head -3 | tr '\n' ' ')
[ -n "$ctrs" ] || { echo "no SQC_ICACHE counters"; exit 0; }
timeout -s KILL 120 rocprofv3 --pmc $ctrs SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$out/pmc" -o pmc -- \
    python3 "$root/bench.py" --spp 64 --steps 1 --warmup 0 --no-cpu-baseline --no-hbm-probe --no-count > "$out/pmc.log" 2>&1
echo "rc=$?"
