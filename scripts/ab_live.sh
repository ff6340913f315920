#!/bin/bash
# Alternating same-box A/B of the live leg (bench.live_leg: ring callback, list entry, fitSubspace)
# under two environment settings.  usage: scripts/ab_live.sh "<envA>" "<envB>" [rounds]
A="$1"; B="$2"; N="${3:-3}"
for i in $(seq 1 "$N"); do
  for v in "$A" "$B"; do
    out=$(env $v timeout -k 10 120 python -c '
import json, bench
print(json.dumps(bench.live_leg(0, 1920, 1080, 16, with_cpu=False)))' 2>/dev/null) || { echo "run failed: $v"; exit 1; }
    echo "$v :: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["trajectory_ms"], d["trajectory_list_ms"], d["fit_subspace_ms"], d["ring_equals_list"])')"
  done
done
