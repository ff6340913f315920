#!/bin/bash
# Round 6: C4 one-band time (8K RGB, band 0 of 8, F = 2) across library revisions, alternating.
# Usage (GPU box): bash scripts/r06_c4bisect.sh head r04 b508 ...   (lib_var/<name>/libmdx.so)
for r in 1 2; do
    for v in "$@"; do
        if [ "$v" = head ]; then lib=$PWD/motion_detection_amd/lib/libmdx.so; else lib=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
        timeout -k 10 120 scripts/micro/bin/c4_band_timer "$lib" 20 2 0 8 | sed "s|$PWD/||" || exit 1
    done
done
