#!/bin/bash
# GPU box: LK dataflow / call pipelining settings at 4K x 8 (one pair per XCD) and 1080p x 32,
# and the C4 8-band rehearsal with and without pipelining.
for cfg in 4k 1080p; do
  for v in "MDX_PIPE=0 MDX_LK_FLOW=0" "MDX_PIPE=0" "MDX_PIPE=1"; do
    env $v timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu --no-roofline --no-live --no-4k \
        --no-lk-roofline > gpurun_out/ab4k.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab4k.json')); print('$cfg $v', d['value'], d['stage_ms_per_step']['lk'])"
  done
done
for v in "MDX_PIPE=0" "MDX_PIPE=1"; do
  env $v timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 8 --inflight 2 --steps 10 --warmup 3 \
      > gpurun_out/abc4.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abc4.json')); print('c4 $v', d['value'], d['ms_per_frame'], d['one_band_ms'])"
done
