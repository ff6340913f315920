#!/bin/bash
# Round-6 evidence on the GPU box (repo root), HEAD's library.  Two parts so each fits one gpurun call:
#   bash scripts/r06_collect.sh a   -> GPU tests, default bench, kernel-trace summary of the bench
#   bash scripts/r06_collect.sh b   -> LK / step / warp PMC passes, warp kernel trace, LK tail stamps, live-leg kernel
#                                      trace, C4 runs
# Outputs under gpurun_out/r06/; the *_to_json scripts turn them into profiles/ (CPU side).
set -o pipefail
part=${1:-a}
out=gpurun_out/r06; mkdir -p $out
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "$part" = w ]; then   # the warp evidence alone (also in part b)
    BENCH_ARGS="--only-roofline --roofline-h affine --steps 3 --warmup 1 --roofline-warmup 2 --no-cpu" \
        bash scripts/pmc_sets.sh warp "FETCH_SIZE" "WRITE_SIZE" > $out/pmc_warp.log 2>&1 || exit 1
    mkdir -p $out/warp_kt $out/warp_kt_proj
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/warp_kt -o run --output-format csv -- python3 bench.py \
        --only-roofline --roofline-h affine --steps 20 --warmup 3 --no-cpu > $out/warp_kt/p1.json 2> $out/warp_kt/p1.err || exit 1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/warp_kt_proj -o run --output-format csv -- python3 bench.py \
        --only-roofline --roofline-h projective --steps 20 --warmup 3 --no-cpu > $out/warp_kt_proj/p1.json \
        2> $out/warp_kt_proj/p1.err || exit 1
elif [ "$part" = a ]; then
    step pytest_gpu
    timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > $out/pytest_gpu.log 2>&1 || exit 1
    step bench
    timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 1
    step smoke
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit 1
    step profile
    bash scripts/profile.sh r06 --no-cpu > $out/profile.log 2>&1 || exit 1
else
    step pmc_lk
    bash scripts/pmc_lk.sh > $out/pmc_lk.log 2>&1 || exit 1
    step pmc_step
    # dataflow ON (round 5): under counter collection kernels serialize, the waits give up and
    # the levels are recomputed in sequence within each call (lk_fallbacks in the bench line)
    BENCH_ARGS="--steps 2 --warmup 1 --no-cpu --no-roofline --no-live --no-4k --no-ransac --no-lk-roofline" \
        bash scripts/pmc_sets.sh step "FETCH_SIZE" "WRITE_SIZE" > $out/pmc_step.log 2>&1 || exit 1
    step pmc_warp
    BENCH_ARGS="--only-roofline --roofline-h affine --steps 3 --warmup 1 --roofline-warmup 2 --no-cpu" \
        bash scripts/pmc_sets.sh warp "FETCH_SIZE" "WRITE_SIZE" > $out/pmc_warp.log 2>&1 || exit 1
    step pmc_warp_counters
    bash scripts/pmc_warp.sh gpurun_out/pmc_warpc > $out/pmc_warpc.log 2>&1 || exit 1
    step warp_kt
    mkdir -p $out/warp_kt
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/warp_kt -o run --output-format csv -- python3 bench.py \
        --only-roofline --roofline-h affine --steps 20 --warmup 3 --no-cpu > $out/warp_kt/p1.json 2> $out/warp_kt/p1.err || exit 1
    mkdir -p $out/warp_kt_proj
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/warp_kt_proj -o run --output-format csv -- python3 bench.py \
        --only-roofline --roofline-h projective --steps 20 --warmup 3 --no-cpu > $out/warp_kt_proj/p1.json \
        2> $out/warp_kt_proj/p1.err || exit 1
    step lk_levels
    mkdir -p $out/seq
    MDX_LK_FLOW=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $out/seq -o run --output-format csv -- python3 bench.py \
        --steps 5 --warmup 2 --no-cpu --no-roofline --no-live --no-4k --no-ransac --no-lk-roofline --no-pipelining \
        > $out/seq.json 2> $out/seq.err || exit 1
    MDX_LK_DEBUG=1 timeout -k 10 300 python3 scripts/lk_level_diag.py --times "$(find $out/seq -name run_kernel_trace.csv | head -n 1)" \
        > $out/lk_levels.txt 2> $out/lk_levels.err || exit 1
    step lk_tail
    MDX_LK_DEBUG=1 timeout -k 10 200 python3 scripts/lk_tail.py > $out/lk_tail.txt 2> $out/lk_tail.err || exit 1
    step live_kt
    mkdir -p $out/live
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/live/kt -o run --output-format csv -- python3 -c \
        "import sys, json; sys.path.insert(0, '.'); import bench; print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False, reps=3)))" \
        > $out/live/kt.json 2> $out/live/kt.err || exit 1
    step c4
    timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 8 --inflight 2 --steps 10 --warmup 3 \
        > $out/c4_n1_k8_f2.json 2> $out/c4_f2.err || exit 1
    timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 1 --inflight 2 --steps 10 --warmup 3 \
        > $out/c4_n1_k1_f2.json 2> $out/c4_k1.err || exit 1
    timeout -k 10 300 python3 bench.py --workload c4 --config 8k --gpus 2 --rehearse --bands 8 --inflight 2 \
        --steps 10 --warmup 3 > $out/c4_n2_k8_f2.json 2> $out/c4_reh.err || exit 1
    step c4_band
    timeout -k 10 120 scripts/micro/bin/c4_band_timer $PWD/motion_detection_amd/lib/libmdx.so 20 2 0 8 > $out/c4_band_timer.txt || exit 1
    step c4_kt
    mkdir -p $out/c4kt
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/c4kt -o run --output-format csv -- python3 bench.py \
        --workload c4 --config 8k --bands 8 --inflight 2 --steps 3 --warmup 2 > $out/c4kt/p1.json 2> $out/c4kt/p1.err || exit 1
fi
echo done
