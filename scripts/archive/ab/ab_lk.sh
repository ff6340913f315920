#!/bin/bash
# GPU box: parity suite on the current library, then per-stage timing of env configurations
# (LK_ENVS="name:VAR=v,VAR2=v name2:..."; default: the plain build) and of extra libraries named
# on the command line (motion_detection_amd/lib/libmdx_<v>.so).
out=gpurun_out/ab; mkdir -p $out
bash scripts/gpu_check.sh || exit $?
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $out/$name.json 2> $out/$name.err
    local rc=$?
    python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', d['ms_per_step'], d['stage_ms_per_step'])" || echo "$name rc=$rc"
    [ $rc -le 1 ] || exit $rc
}
for cfg in ${LK_ENVS:-default:MDX_NONE=0}; do
    name=${cfg%%:*}; envs=${cfg#*:}
    run $name ${envs//,/ }
done
for v in "$@"; do run $v MDX_LIB_PATH=$PWD/motion_detection_amd/lib/libmdx_$v.so; done
