#!/bin/bash
# GPU box: roofline leg of bench.py per variant library.
out=gpurun_out/wvariants; mkdir -p $out
for v in "$@"; do
    MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so timeout -k 10 200 python bench.py --only-roofline \
        --steps 10 --warmup 2 --no-cpu > $out/$v.json 2> $out/$v.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/$v.json')); print('$v', d['roofline']['avg_launch_us'], d['roofline']['frac'])" || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
