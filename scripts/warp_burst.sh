#!/bin/bash
# Round 6: the warp's burst transient, per launch (GPU box).  300 k_warp_diff launches (4K x 32,
# affine) after 2 s idle: (1) kernel records; (2) kernel records + GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES
# per dispatch; (3) the stamped diagnostic library (in-kernel clock per launch, no profiler);
# (4) the copy probe's records for comparison.
set -o pipefail
out=gpurun_out/burst; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $out/kt -o run --output-format csv -- python3 scripts/warp_burst.py 300 2 \
    > $out/kt.json 2> $out/kt.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $out/pmc -o run --output-format csv \
    -- python3 scripts/warp_burst.py 300 2 > $out/pmc.json 2> $out/pmc.err || exit 1
MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/wstamp/libmdx.so timeout -k 10 120 python3 scripts/warp_burst.py 300 2 \
    > $out/stamp.json 2> $out/stamp.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $out/probe -o run --output-format csv -- python3 scripts/warp_burst.py 300 2 --probe \
    > $out/probe.json 2> $out/probe.err || exit 1
echo done
