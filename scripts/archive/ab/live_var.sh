#!/bin/bash
# Live-leg timing of variant libraries (motion_detection_amd/lib_var/<name>), env applied to each.
# Usage (GPU box): ROUNDS=1 bash scripts/live_var.sh head v1 v2 ...
mkdir -p gpurun_out/live
for r in $(seq 1 ${ROUNDS:-1}); do
    for v in "$@"; do
        if [ "$v" = head ]; then lib=""; else lib="MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so"; fi
        env $lib ${ENV} timeout -k 10 120 python3 -c "
import sys, json; sys.path.insert(0, '.')
import bench
print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False, reps=${REPS:-6})))" > gpurun_out/live/out.json 2> gpurun_out/live/err.log
        rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/live/err.log; exit $rc; }
        python3 -c "import json; d=json.load(open('gpurun_out/live/out.json')); print('$v round $r: ring callback', d['trajectory_ms'], 'ms, list', d['trajectory_list_ms'], 'ms, ring==list', d['ring_equals_list'])"
    done
done
