#!/bin/bash
# GPU box: live-leg (trajectory + fitSubspace) timing of library variants.
# Usage: bash scripts/live_ab.sh default w5 ...  (see scripts/lib_ab.sh for the naming)
out=gpurun_out/live_ab; mkdir -p $out
i=0
for v in "$@"; do
    i=$((i+1))
    lib=$PWD/motion_detection_amd/lib/libmdx_$v.so
    [ "$v" = default ] && lib=$PWD/motion_detection_amd/lib/libmdx.so
    MDX_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-roofline --no-4k \
        > $out/${i}_$v.json 2> $out/${i}_$v.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/${i}_$v.json')); print('$v', d['live_path']['trajectory_ms'])" \
        || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
