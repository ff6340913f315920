#!/bin/bash
# Round 6: warp tests on the in-tree library, then the same-box roofline A/B of head against the
# given variants (r06_warp_ab.sh), then one SQ_INSTS_VALU pass per library.
set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_warp_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wab_tests.log 2>&1 || { tail -20 gpurun_out/wab_tests.log; exit 1; }
tail -1 gpurun_out/wab_tests.log
ROUNDS=${ROUNDS:-3} ROOF_H=${ROOF_H:-affine} bash scripts/r06_warp_ab.sh head "$@" || exit 1
[ -n "$NOPMC" ] && { echo done; exit 0; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/wpmc
for v in head "$@"; do
    if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/wpmc/$v -o run \
        --output-format csv -- python3 bench.py --only-roofline --roofline-h affine --steps 3 --warmup 1 --roofline-warmup 2 \
        --no-cpu > gpurun_out/wpmc/$v.json 2> gpurun_out/wpmc/$v.err || exit 1
done
echo done
