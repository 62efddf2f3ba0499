#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: kernel-trace + stats, and one PMC pass per counter group
# (counters in their own runs, never combined with tracing domains).
set -u
tag="$1"; shift
args="${*:---spp 16 --steps 1 --warmup 0 --no-cpu-baseline}"
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/prof_$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
run() {
    name="$1"; shift
    echo "=== rocprofv3 $name"
    timeout -k 10 400 rocprofv3 "$@" --output-format csv -d "$out/$name" -o "$name" -- \
        python3 "$root/bench.py" $args > "$out/$name.log" 2>&1
    rc=$?
    echo "rc=$rc"; tail -n 2 "$out/$name.log"
    case $rc in 0|1|2) ;; *) exit $rc ;; esac
}
run trace --kernel-trace --stats
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run pmc_sq2 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FP64
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_l2 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum
if [ -n "${PROFILE_LDS:-}" ]; then
    run pmc_lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
fi
exit 0
