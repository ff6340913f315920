#!/bin/bash
# Alternating same-box A/B of the warp+diff roofline leg (4K x 32, true H) between libraries:
# "head" = the in-tree build, other names = motion_detection_amd/lib_var/<name>/libmdx.so.
# usage (GPU box): scripts/ab_roof.sh <rounds> head wold ...
N=$1; shift
for i in $(seq 1 "$N"); do
  for v in "$@"; do
    if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
    out=$(timeout -k 10 120 python bench.py --only-roofline --steps 20 --warmup 5 --no-cpu 2>/dev/null) || { echo "run failed: $v"; exit 1; }
    echo "$v :: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read())["roofline"]; print(d["avg_launch_us"], d["frac"])')"
  done
done
