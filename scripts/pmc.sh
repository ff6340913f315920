#!/bin/bash
# PMC pass (counters only, kernel-trace; no sys/runtime trace) over a short bench run.
# Usage: bash scripts/pmc.sh <tag> "<counters>" [bench args...]
set -o pipefail
tag=$1; shift; ctrs=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/pmc_$tag
timeout -k 10 600 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc_$tag -o run --output-format csv \
    -- python3 bench.py "$@" > gpurun_out/pmc_$tag/bench.json 2> gpurun_out/pmc_$tag/stderr.log
rc=$?; echo "pmc rc=$rc"; exit $rc
