#!/bin/bash
# GPU box: rocprofv3 kernel-trace and PMC passes (one counter set per run) over the live leg only
# (5 x 1080p rgb8 trajectory on the resident ring + fitSubspace).  Usage: bash scripts/live_pmc.sh <tag>
tag=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/livepmc_$tag; mkdir -p $out
CMD="import sys, json; sys.path.insert(0, '.'); import bench; print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False, reps=3)))"
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU"
S2="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 -c "$CMD" > $out/kt.json 2> $out/kt.err || exit $?
i=0
for set in "$S1" "$S2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv -- python3 -c "$CMD" > $out/p$i.json 2> $out/p$i.err
    rc=$?; echo "pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
