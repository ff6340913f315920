#!/bin/bash
# GPU box: the warp+diff roofline leg under each MDX_WARP implementation (1: FP64 coordinates,
# 2: fixed point), alternating, after the warp parity tests.
out=gpurun_out/warp_ab; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_warp_gpu.py > $out/tests.log 2>&1
rc=$?; echo "warp tests rc=$rc"; tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for impl in ${IMPLS:-1 2}; do
    MDX_WARP=$impl timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --no-live --no-4k --only-roofline \
        > $out/r${rep}_$impl.json 2> $out/r${rep}_$impl.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/r${rep}_$impl.json')); r=d['roofline']; print('impl $impl', r['avg_launch_us'], r['frac'])" || { echo "impl $impl rc=$rc"; exit 1; }
  done
done
