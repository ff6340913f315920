#!/bin/bash
# GPU box: the C4 row-tiled workload (8K RGB) -- 1 rank whole frame, 1 rank rehearsing 8 bands,
# at 1/2/3 frames in flight, and 2 ranks sharing the one GPU (real record exchange over gloo,
# --rehearse).  Each run under its own limit.
out=gpurun_out/c4; mkdir -p $out
runs=""
for F in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c4 --inflight $F --steps 5 --warmup 2 > $out/n1_k1_f$F.json 2> $out/n1_k1_f$F.err || exit $?
  timeout -k 10 300 python bench.py --workload c4 --bands 8 --inflight $F --steps 5 --warmup 2 > $out/n1_k8_f$F.json 2> $out/n1_k8_f$F.err || exit $?
  runs="$runs n1_k1_f$F n1_k8_f$F"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --workload c4 --gpus 2 --rehearse --steps 5 --warmup 2 > $out/n2_k2.json 2> $out/n2_k2.err || exit $?
for f in $runs n2_k2; do python3 -c "
import json; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], 'Mpx/s', d['ms_per_frame'], 'ms/frame', d['phase_ms_per_step_rank0'], 'one_band', d['one_band_ms'], 'nv', d['num_vectors'], 'n_gpus', d['n_gpus'])"; done
