#!/bin/bash
# Round 6: same-box A/B of the warp roofline leg (4K x 32, affine true H, 200 untimed + 20 timed
# launches) across library variants: name[:ENV=VAL] as in r06_ab.sh.
mkdir -p gpurun_out/wab
for r in $(seq 1 ${ROUNDS:-3}); do
    for spec in "$@"; do
        v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
        tag=$(echo "$spec" | tr ':=,' '___')
        if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
        env ${envs//,/ } timeout -k 10 120 python3 bench.py --only-roofline --roofline-h ${ROOF_H:-affine} --steps 20 \
            --warmup 3 --no-cpu > gpurun_out/wab/$tag.$r.json 2> gpurun_out/wab/$tag.$r.err
        rc=$?
        [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -3 gpurun_out/wab/$tag.$r.err; exit $rc; }
        python3 -c "
import json; d=json.load(open('gpurun_out/wab/$tag.$r.json')); r=d['roofline']
p=r.get('projective') or {}
print(f'{\"$spec\":20s} round $r: launch {r[\"avg_launch_us\"]:.1f} us frac {r[\"frac\"]:.4f} copy {r.get(\"copy_ceiling_frac\")} proj {p.get(\"avg_launch_us\")}')"
    done
done
