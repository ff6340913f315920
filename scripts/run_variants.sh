#!/bin/bash
# GPU box: time each variant library with the default bench (LK stage ms from stage timing).
out=gpurun_out/variants; mkdir -p $out
for v in "$@"; do
    MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 \
        --no-cpu --no-roofline > $out/$v.json 2> $out/$v.err
    rc=$?
    python3 -c "import json,sys; d=json.load(open('$out/$v.json')); print('$v', d['ms_per_step'], d['stage_ms_per_step'])" || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
    case $v in f[0-9]*) ;; *)
        MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so timeout -k 10 300 python -m pytest tests -m gpu -q -x \
            > $out/$v.tests 2>&1; rc=$?; echo "$v tests rc=$rc: $(tail -1 $out/$v.tests)"
        [ $rc -le 1 ] || exit $rc ;;
    esac
done
