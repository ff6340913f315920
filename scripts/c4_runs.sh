#!/bin/bash
# GPU box: the C4 row-tiled workload (8K RGB) -- 1 rank whole frame, 1 rank rehearsing 8 bands,
# and 2 ranks sharing the one GPU (real record exchange over gloo).  Each run under its own limit.
out=gpurun_out/c4; mkdir -p $out
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > $out/n1_k1.json 2> $out/n1_k1.err || exit $?
timeout -k 10 300 python bench.py --workload c4 --bands 8 --steps 5 --warmup 2 > $out/n1_k8.json 2> $out/n1_k8.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --workload c4 --gpus 2 --steps 5 --warmup 2 > $out/n2_k2.json 2> $out/n2_k2.err || exit $?
for f in n1_k1 n1_k8 n2_k2; do python3 -c "
import json; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], 'Mpx/s', d['ms_per_step'], 'ms', d['phase_ms_per_step_rank0'], 'one_band', d['one_band_ms'], 'nv', d['num_vectors'])"; done
