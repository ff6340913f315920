#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only) of the default bench step for variant
# libraries; per-dispatch means per kernel via scripts/pmc_summary.py.
# Usage (GPU box): bash scripts/pmc_var.sh <kernel-substring> head old ...
ks=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM"
S2="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"
for v in "$@"; do
    if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
    i=0
    for set in "$S1" "$S2"; do
        i=$((i+1)); out=gpurun_out/pmcv_$v/p$i; mkdir -p $out
        timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $out -o run --output-format csv \
            -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-roofline --no-live --no-4k --no-lk-roofline \
            > $out.json 2> $out.err
        rc=$?; [ $rc -le 1 ] || { echo "$v pass $i rc=$rc"; exit $rc; }
    done
    echo "== $v"; python3 scripts/pmc_summary.py gpurun_out/pmcv_$v $ks
done
