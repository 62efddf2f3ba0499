#!/bin/bash
# VALU instruction mix of the megakernel per library (the f64 share before/after a change):
#   tools/valu_mix.sh <tag> lib1.so lib2.so ...   (on the GPU box, via gpurun)
# One PMC pass per library at C4 64 spp; writes gpurun_out/valu_<tag>/<lib>/.
set -u
tag="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
    name=$(basename "$lib" .so)
    out="$root/gpurun_out/valu_$tag/$name"
    mkdir -p "$out"
    CPT_LIB_PATH="$root/$lib" timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
        SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU \
        --output-format csv -d "$out" -o pmc -- python3 "$root/bench.py" --spp 64 --steps 1 --warmup 0 \
        --no-cpu-baseline --no-hbm-probe --no-count > "$out.log" 2>&1
    rc=$?
    echo "$lib rc=$rc"; tail -n 1 "$out.log"
    [ $rc -eq 0 ] || exit $rc
done
