#!/bin/bash
# Round 6, final: the default bench (stamped summaries attach) and a 2-rank C3 rehearsal (two ranks
# sharing the box's one GPU; the driver's N-GPU runs use one GPU per rank).
set -o pipefail
out=gpurun_out/r06f; mkdir -p $out
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --rehearse --steps 10 --warmup 3 --no-cpu --no-roofline --no-live \
    --no-4k --no-ransac --no-lk-roofline > $out/c3_n2_rehearse.json 2> $out/c3_n2_rehearse.err || exit 1
echo done
