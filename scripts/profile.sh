#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (run on the GPU box from the repo root).
# Usage: bash scripts/profile.sh <tag> [bench args...]
set -o pipefail
tag=${1:-r01}; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof_$tag
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv \
    -- python3 bench.py "$@" > gpurun_out/prof_$tag/bench_stdout.json 2> gpurun_out/prof_$tag/bench_stderr.log
rc=$?; echo "rocprof rc=$rc"; exit $rc
