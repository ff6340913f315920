#!/bin/bash
# Alternating same-box A/B of the default bench step under two environment settings.
# usage: scripts/ab_env.sh "<envA>" "<envB>" [rounds]   (run on the GPU box; prints value per run)
A="$1"; B="$2"; N="${3:-3}"
args="--steps 20 --warmup 5 --no-cpu --no-live --no-4k --no-roofline --no-lk-roofline --no-parity"
for i in $(seq 1 "$N"); do
  for v in "$A" "$B"; do
    out=$(env $v timeout -k 10 120 python bench.py $args 2>/dev/null) || { echo "run failed: $v"; exit 1; }
    echo "$v :: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step"]["lk"], d.get("value_unpipelined"))')"
  done
done
