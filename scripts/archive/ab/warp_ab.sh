#!/bin/bash
# GPU box: for the current libmdx.so and each libmdx_<name>.so given as an argument (A/B of
# k_warp_diff builds): the warp parity tests, then the roofline leg of bench.py.
mkdir -p gpurun_out
rc=0
for v in default "$@"; do
    if [ $v = default ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so; fi
    timeout -k 10 300 python -u -m pytest tests/test_warp_gpu.py -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/warp_tests_$v.log 2>&1
    rt=$?; echo "$v: warp tests rc=$rt $(tail -1 gpurun_out/warp_tests_$v.log)"
    [ $rt -le 1 ] || exit $rt
    [ $rt -eq 0 ] || rc=1
    timeout -k 10 200 python bench.py --only-roofline --steps 20 --warmup 3 --no-cpu > gpurun_out/roof_$v.json 2> gpurun_out/roof_$v.err
    rc2=$?
    python3 -c "import json; d=json.load(open('gpurun_out/roof_$v.json')); print('$v', d['roofline']['avg_launch_us'], d['roofline']['frac'])" || echo "$v rc=$rc2"
    [ $rc2 -le 1 ] || exit $rc2
done
exit $rc
