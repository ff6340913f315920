#!/bin/bash
# GPU box: PMC pass over the default bench step for the LK kernels (k_lk_class, k_lk_A, k_lk_iter):
# executed VALU / LDS wave-instructions and busy cycles; summarised per step into
# gpurun_out/pmc_lk/pmc_lk.json by scripts/pmc_lk_to_json.py (copy to profiles/pmc_lk_iter.json).
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
S2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
out=gpurun_out/pmc_lk; mkdir -p $out
ARGS="--steps 2 --warmup 1 --no-cpu --no-roofline --no-live --no-4k --no-ransac --no-lk-roofline"
i=0
for set in "$S1" "$S2"; do
    i=$((i+1))
    # the level dataflow stays on: counter collection serializes kernels, so its waits give up and
    # the abandoned levels are recomputed in sequence within each call (round 5; lk_fallbacks in
    # the bench line counts them) -- the same groups and iterations, plus the abandoned launches
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv \
        -- python3 bench.py $ARGS > $out/p$i.json 2> $out/p$i.err
    rc=$?; echo "pass $i rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
python3 scripts/pmc_lk_to_json.py $out auto > $out/pmc_lk.json && cat $out/pmc_lk.json
