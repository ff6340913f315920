#!/bin/bash
# LK iteration-kernel pipe counters (GPU box, repo root): VALU / LDS / memory busy per kernel.
tag=${1:-lds}
args="--steps 2 --warmup 1 --no-cpu --no-roofline"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/probe_$tag; mkdir -p $out
run() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --kernel-trace -d $out/$name -o run --output-format csv \
        -- python3 bench.py $args > $out/$name.json 2> $out/$name.err
    local rc=$?; echo "$name rc=$rc"
    [ $rc -le 1 ] || exit $rc
}
run sq --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM
run ta --pmc TA_BUSY_avr TA_TA_BUSY_sum
run ta2 --pmc TD_BUSY_avr GRBM_GUI_ACTIVE
exit 0
