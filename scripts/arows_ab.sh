#!/bin/bash
# GPU box: coarsest-level A sums by k_lk_A_rows (default) vs the LDS-DMA k_lk_A on every level
# (MDX_LK_A_DMA_ALL=1), alternating default bench runs without the CPU / roofline / live / 4K legs.
set -e
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  for v in rows dma; do
    if [ $v = dma ]; then export MDX_LK_A_DMA_ALL=1; else unset MDX_LK_A_DMA_ALL; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --no-live --no-4k > gpurun_out/arows_${v}_$i.json 2> gpurun_out/arows_${v}_$i.err
    python3 -c "import json; d=json.load(open('gpurun_out/arows_${v}_$i.json')); s=d['stage_ms_per_step']; print('$v', d['value'], 'lk', s['lk'], 'total', s['total'])"
  done
done
