#!/bin/bash
# GPU box: run the -m gpu suite against variant libraries (names as arguments).
for v in "$@"; do
    MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so timeout -k 10 300 python -m pytest tests -m gpu -q -x \
        > gpurun_out/vtest_$v.log 2>&1
    echo "$v tests: $(tail -1 gpurun_out/vtest_$v.log)"
done
