#!/bin/bash
# GPU box: A/B of environment settings on the default bench step (no CPU / roofline / live / 4K legs).
# Usage: bash scripts/env_ab.sh "MDX_STREAM_PRIO=0" "MDX_STREAM_PRIO=1" ...   (each argument: one run's env)
out=gpurun_out/env_ab; mkdir -p $out
i=0
for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --no-live --no-4k \
        > $out/$i.json 2> $out/$i.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out/$i.json')); s=d['stage_ms_per_step']; print('$v', d['value'], 'lk', s['lk'], 'total', s['total'])" \
        || echo "$v rc=$rc"
    [ $rc -le 1 ] || exit $rc
done
