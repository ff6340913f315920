#!/bin/bash
# Round-6 LK diagnosis on the GPU box: default bench, per-level k_lk_iter times with the levels in
# sequence (MDX_LK_FLOW=0, kernel trace), per-level iterations / lockstep (debug trace).
set -o pipefail
out=gpurun_out/r06diag; mkdir -p $out
export TMPDIR=/tmp
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu > $out/bench.json 2> $out/bench.err || exit 1
echo "== seq kt $(date +%T)"
MDX_LK_FLOW=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/seq -o run --output-format csv -- python3 bench.py \
    --steps 5 --warmup 2 --no-cpu --no-roofline --no-live --no-4k --no-ransac --no-lk-roofline > $out/seq.json 2> $out/seq.err || exit 1
csv=$(find $out/seq -name 'run_kernel_trace.csv' | head -n 1)
echo "== diag $(date +%T) $csv"
MDX_LK_DEBUG=1 timeout -k 10 300 python3 scripts/lk_level_diag.py --times "$csv" > $out/diag.txt 2> $out/diag.err || exit 1
cat $out/diag.txt
echo done
