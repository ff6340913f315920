#!/bin/bash
# GPU box: LK group-size A/B.  Parity of the full path under each MDX_LK_G setting, then the
# default bench step (no CPU / roofline legs).  Usage: bash scripts/lk_ab.sh "" 2 4 ...
mkdir -p gpurun_out
for g in "$@"; do
    tag=${g:-auto}
    MDX_LK_G=$g timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -k "full_path or batch_dev or small" \
        --timeout 120 --timeout-method thread > gpurun_out/lk_tests_$tag.log 2>&1
    rt=$?; echo "G=$tag tests rc=$rt $(tail -1 gpurun_out/lk_tests_$tag.log)"
    [ $rt -le 1 ] || exit $rt
    MDX_LK_G=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --no-live \
        > gpurun_out/lk_bench_$tag.json 2> gpurun_out/lk_bench_$tag.err
    rb=$?
    python3 -c "import json; d=json.load(open('gpurun_out/lk_bench_$tag.json')); print('G=$tag', d['value'], d['stage_ms_per_step']['lk'])" || echo "G=$tag bench rc=$rb"
    [ $rb -le 1 ] || exit $rb
done
