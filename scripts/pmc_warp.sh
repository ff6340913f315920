#!/bin/bash
# GPU box: counter passes over the warp+diff roofline leg (4K x 32, true H): issue, LDS, waits.
# Output: <out>/p<i>/run_counter_collection.csv (summarise with pmc_warp_summary.py)
# Usage: bash scripts/pmc_warp.sh [out dir, default gpurun_out/pmc_warpc]
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=${1:-gpurun_out/pmc_warpc}; mkdir -p $out
ARGS="--only-roofline --roofline-h affine --steps 3 --warmup 1 --roofline-warmup 2 --no-cpu"
S1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
S2="SQ_INSTS_SALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
i=0
for set in "$S1" "$S2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv \
        -- python3 bench.py $ARGS > $out/p$i.json 2> $out/p$i.err
    rc=$?; echo "pass $i rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
