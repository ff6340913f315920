#!/bin/bash
# Round 6, batch 3: the GPU suite on the plain / dataflow k_lk_iter split, C4 one band A/B (head, round 5,
# round 4) with every band's real record, and the default bench A/B head vs round 5.
set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_b3.log 2>&1 || { tail -30 gpurun_out/pytest_b3.log; exit 1; }
tail -1 gpurun_out/pytest_b3.log
bash scripts/r06_c4bisect.sh head r05 r04 || exit 1
ROUNDS=2 bash scripts/r06_ab.sh head r05
