#!/bin/bash
# GPU box: PMC passes over the roofline leg (k_warp_diff, 4K x32) for libmdx.so and each
# libmdx_<name>.so argument.  One rocprofv3 --pmc pass per counter set.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
S2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
S3="TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_RD GRBM_COUNT"
for v in default "$@"; do
    if [ $v = default ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so; fi
    out=gpurun_out/wpmc_$v; mkdir -p $out
    i=0
    for set in "$S1" "$S2" "$S3"; do
        i=$((i+1))
        timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv \
            -- python3 bench.py --only-roofline --steps 3 --warmup 1 --no-cpu > $out/p$i.json 2> $out/p$i.err
        rc=$?; echo "$v pass $i rc=$rc"
        [ $rc -le 1 ] || break
    done
done
exit 0
