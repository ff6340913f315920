#!/bin/bash
# Round 6, batch 4: LK at 5 waves per SIMD with the chain reads in two halves (w5s), the split alone
# (ds4), and the iteration launches' share of the resident waves (MDX_LK_CAP 75 / 95), against head.
set -o pipefail
MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/w5s/libmdx.so timeout -k 10 600 python3 -u -m pytest \
    tests/test_parity_gpu.py tests/test_bench_path_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_w5s.log 2>&1 || { tail -30 gpurun_out/pytest_w5s.log; exit 1; }
tail -1 gpurun_out/pytest_w5s.log
ROUNDS=3 bash scripts/r06_ab.sh head w5s ds4 head:MDX_LK_CAP=75 head:MDX_LK_CAP=95
