#!/bin/bash
# GPU box: LK dataflow on/off against pairs per XCD (batch / 8) at 1080p and 4K.
for args in "$@"; do
  for v in "MDX_LK_FLOW=0" "MDX_LK_FLOW=1"; do
    env MDX_PIPE=0 $v timeout -k 10 200 python bench.py $args --steps 5 --warmup 2 --no-cpu --no-roofline --no-live --no-4k \
        --no-lk-roofline > gpurun_out/abfb.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/abfb.json')); print('$args $v', d['value'], d['stage_ms_per_step']['lk'])"
  done
done
