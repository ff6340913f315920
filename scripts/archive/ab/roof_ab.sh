#!/bin/bash
# GPU box: warp+diff roofline leg of library variants (bench.py --only-roofline).
# Usage: bash scripts/roof_ab.sh default old ...  (naming as scripts/lib_ab.sh)
out=gpurun_out/roof_ab; mkdir -p $out
i=0
for v in "$@"; do
    i=$((i+1))
    lib=$PWD/motion_detection_amd/lib/libmdx_$v.so
    [ "$v" = default ] && lib=$PWD/motion_detection_amd/lib/libmdx.so
    MDX_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-live --no-4k --only-roofline \
        > $out/${i}_$v.json 2> $out/${i}_$v.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/${i}_$v.json')); r=d['roofline']; print('$v', r['avg_launch_us'], r['frac'])" \
        || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
