#!/bin/bash
# GPU box: PMC passes over the roofline leg (k_warp_*, 4K x32) per MDX_WARP implementation.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU"
S2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
S3="SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_IFETCH SQ_WAIT_INST_VMEM GRBM_COUNT"
for impl in ${IMPLS:-1 2}; do
    out=gpurun_out/wpmc_env_$impl; mkdir -p $out
    i=0
    for set in "$S1" "$S2" "$S3"; do
        i=$((i+1))
        MDX_WARP=$impl timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv \
            -- python3 bench.py --only-roofline --steps 3 --warmup 1 --no-cpu > $out/p$i.json 2> $out/p$i.err
        rc=$?; echo "$impl pass $i rc=$rc"
        [ $rc -le 1 ] || break
    done
done
exit 0
