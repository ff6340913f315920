#!/bin/bash
# PMC passes with caller-chosen counter sets over a short bench run (GPU box, repo root).
# Usage: bash scripts/pmc_sets.sh <tag> "<ctr ctr ...>" ["<ctr ...>" ...]
# Env BENCH_ARGS overrides the bench arguments; MDX_LIB_PATH selects a variant library.
tag=$1; shift
args=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu --no-roofline"}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag; mkdir -p $out
i=0
for set in "$@"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d $out/p$i -o run --output-format csv \
        -- python3 bench.py $args > $out/p$i.json 2> $out/p$i.err
    rc=$?; echo "pass $i rc=$rc ($set)"
    [ $rc -le 1 ] || exit $rc
done
exit 0
