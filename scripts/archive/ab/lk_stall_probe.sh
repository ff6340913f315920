#!/bin/bash
# LK stall breakdown (GPU box, repo root): where wave time goes in k_lk_iter.
tag=${1:-stall}
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
run w1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VSKIPPED
run w2 --pmc SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_THREAD_CYCLES_VALU
run w3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM
exit 0
