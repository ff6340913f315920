#!/bin/bash
# Round 6, first measurement batch: FD parity + LK A/B, C4 revision A/B, warp weight-table A/B.
set -o pipefail
bash scripts/r06_fd.sh head head:MDX_LK_FD=1 pcvt plds head:MDX_LK_G=4 || exit 1
echo "== c4 $(date +%T)"
bash scripts/r06_c4bisect.sh head r04 b508 b0b5 b1f1 bbdd || exit 1
echo "== warp tests wtab $(date +%T)"
MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/wtab/libmdx.so timeout -k 10 300 python3 -u -m pytest tests/test_warp_gpu.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06fd/pytest_wtab.log 2>&1 || { tail -20 gpurun_out/r06fd/pytest_wtab.log; exit 1; }
tail -1 gpurun_out/r06fd/pytest_wtab.log
echo "== warp ab $(date +%T)"
ROUNDS=3 bash scripts/r06_warp_ab.sh head wtab
