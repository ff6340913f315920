#!/bin/bash
# Kernel-trace stats + PMC passes over a short bench run (GPU box, repo root).
# Usage: bash scripts/lk_probe.sh <tag> [bench args...]
# Each pass is its own rocprofv3 run; stops at the first crash-like exit (>1).
tag=$1; shift
args="$@"
[ -z "$args" ] && args="--steps 3 --warmup 1 --no-cpu --no-roofline"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/probe_$tag; mkdir -p $out
run() {  # name, extra rocprof args...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --kernel-trace -d $out/$name -o run --output-format csv \
        -- python3 bench.py $args > $out/$name.json 2> $out/$name.err
    local rc=$?; echo "$name rc=$rc"
    [ $rc -le 1 ] || exit $rc
}
run stats --stats
run sq --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU
run cache --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
[ -n "$PROBE_MEM" ] && run mem --pmc FETCH_SIZE WRITE_SIZE
exit 0
