#!/bin/bash
# Round 6, batch 2: C4 one-band A/B (head, per-level carry off for levels in sequence, round 4) and the
# kernel records of one band on head and on round 4's library.
set -o pipefail
bash scripts/r06_c4bisect.sh head nocarry r04 || exit 1
export TMPDIR=/tmp
for v in head r04; do
    if [ "$v" = head ]; then lib=$PWD/motion_detection_amd/lib/libmdx.so; else lib=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
    mkdir -p gpurun_out/c4kt_$v
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c4kt_$v -o run --output-format csv -- \
        scripts/micro/bin/c4_band_timer "$lib" 10 2 0 8 || exit 1
done
