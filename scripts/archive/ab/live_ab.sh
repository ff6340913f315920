#!/bin/bash
# Live-chain leg only (5 x 1080p rgb8 trajectory + fitSubspace), alternating env settings.
# Usage (GPU box): ROUNDS=2 bash scripts/live_ab.sh "MDX_LK_AUX=1" "MDX_LK_AUX=0"
mkdir -p gpurun_out/live
for r in $(seq 1 ${ROUNDS:-2}); do
    for e in "$@"; do
        env $e timeout -k 10 120 python3 -c "
import sys, json; sys.path.insert(0, '.')
import bench
print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False, reps=${REPS:-10})))" > gpurun_out/live/out.json 2> gpurun_out/live/err.log
        rc=$?; [ $rc -eq 0 ] || { echo "$e rc=$rc"; tail -5 gpurun_out/live/err.log; exit $rc; }
        python3 -c "import json; d=json.load(open('gpurun_out/live/out.json')); print('$e round $r: ring callback', d['trajectory_ms'], 'ms, list', d['trajectory_list_ms'], 'ms, fit_subspace', d['fit_subspace_ms'], 'ms, ring==list', d['ring_equals_list'])"
    done
done
