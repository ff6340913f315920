#!/bin/bash
# rocprofv3 kernel trace (and optionally one PMC pass) of the live leg only (GPU box).
# Usage: bash scripts/live_prof.sh <tag> [counters...]
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/liveprof_$tag; mkdir -p $out
CMD="import sys, json; sys.path.insert(0, '.'); import bench; print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False, reps=3)))"
if [ $# -gt 0 ]; then
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $out -o run --output-format csv -- python3 -c "$CMD" > $out/out.json 2> $out/err.log
else
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 -c "$CMD" > $out/out.json 2> $out/err.log
fi
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || tail -3 $out/err.log
exit $rc
