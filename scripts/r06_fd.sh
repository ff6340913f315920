#!/bin/bash
# Round 6: the float-derivative LK planes (MDX_LK_FD=1) -- the whole GPU suite with them on, then
# the alternating A/B against the int planes and the probes.
set -o pipefail
out=gpurun_out/r06fd; mkdir -p $out
echo "== pytest FD $(date +%T)"
MDX_LK_FD=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest_fd.log 2>&1 || { tail -30 $out/pytest_fd.log; exit 1; }
tail -2 $out/pytest_fd.log
echo "== ab $(date +%T)"
ROUNDS=${ROUNDS:-3} bash scripts/r06_ab.sh "$@"
