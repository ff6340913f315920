#!/bin/bash
# Kernel traces of the default bench and C4 (in-tree library) for the wave-parallel fit.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/fitkt; mkdir -p $out/main $out/c4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/main -o run --output-format csv -- python3 bench.py \
    --steps 10 --warmup 3 --no-cpu --no-live --no-4k --no-roofline --no-lk-roofline --no-ransac > $out/main.json 2> $out/main.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/c4 -o run --output-format csv -- python3 bench.py \
    --workload c4 --config 8k --bands 8 --inflight 2 --steps 3 --warmup 2 > $out/c4.json 2> $out/c4.err || exit 1
echo done
