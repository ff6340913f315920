#!/bin/bash
# Round 6: LK parity tests on the in-tree library, then same-box A/B of the default step (r06_ab.sh)
# against the given variants.
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_parity_gpu.py tests/test_bench_path_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/lkab_tests.log 2>&1 || { tail -20 gpurun_out/lkab_tests.log; exit 1; }
tail -1 gpurun_out/lkab_tests.log
ROUNDS=${ROUNDS:-3} bash scripts/r06_ab.sh "$@" || exit 1
echo done
