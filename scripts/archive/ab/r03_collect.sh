#!/bin/bash
# Round-3 evidence on the GPU box (repo root), HEAD's library: kernel-trace summary of the default
# bench, the LK PMC passes, FETCH/WRITE passes over the step and over the roofline leg, C4 runs.
# Outputs under gpurun_out/r03/; the *_to_json scripts turn them into profiles/ (CPU side).
set -o pipefail
out=gpurun_out/r03; mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1"; }
step profile
bash scripts/profile.sh r03 --no-cpu > $out/profile.log 2>&1 || exit 1
step pmc_lk
bash scripts/pmc_lk.sh > $out/pmc_lk.log 2>&1 || exit 1
step pmc_step
BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-roofline --no-live --no-4k --no-lk-roofline" \
    bash scripts/pmc_sets.sh step "FETCH_SIZE" "WRITE_SIZE" > $out/pmc_step.log 2>&1 || exit 1
step pmc_warp
BENCH_ARGS="--only-roofline --steps 3 --warmup 1 --no-cpu" \
    bash scripts/pmc_sets.sh warp "FETCH_SIZE" "WRITE_SIZE" > $out/pmc_warp.log 2>&1 || exit 1
step c4
timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 8 --inflight 2 --steps 10 --warmup 3 \
    > $out/c4_n1_k8_f2.json 2> $out/c4_f2.err || exit 1
timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 1 --inflight 2 --steps 10 --warmup 3 \
    > $out/c4_n1_k1_f2.json 2> $out/c4_k1.err || exit 1
timeout -k 10 300 python3 bench.py --workload c4 --config 8k --gpus 2 --rehearse --bands 8 --inflight 2 --steps 10 \
    --warmup 3 > $out/c4_n2_k8_f2.json 2> $out/c4_reh.err || exit 1
echo done
