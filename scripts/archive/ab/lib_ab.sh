#!/bin/bash
# GPU box: time library variants with the default bench step (no CPU / roofline / live / 4K legs).
# Usage: bash scripts/lib_ab.sh default old nodma ...   ("default" = motion_detection_amd/lib/libmdx.so,
# any other name = motion_detection_amd/lib/libmdx_<name>.so, e.g. from scripts/lk_variants.sh).
out=gpurun_out/lib_ab; mkdir -p $out
i=0
for v in "$@"; do
    i=$((i+1))
    lib=$PWD/motion_detection_amd/lib/libmdx_$v.so
    [ "$v" = default ] && lib=$PWD/motion_detection_amd/lib/libmdx.so
    MDX_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --no-live --no-4k \
        > $out/${i}_$v.json 2> $out/${i}_$v.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/${i}_$v.json')); s=d['stage_ms_per_step']; print('$v', d['value'], 'lk', s['lk'], 'total', s['total'])" \
        || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
