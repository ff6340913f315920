#!/bin/bash
# Round-6 same-box A/B: alternating variants of the default bench step.  Each argument is
# name[:ENV=VAL[,ENV=VAL]] -- name "head" = the in-tree library, else lib_var/<name>/libmdx.so.
# Usage (GPU box): ROUNDS=3 bash scripts/r06_ab.sh head pcvt head:MDX_LK_G=4
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-3}); do
    for spec in "$@"; do
        v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
        tag=$(echo "$spec" | tr ':=,' '___')
        if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
        env ${envs//,/ } timeout -k 10 120 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu --no-live --no-4k \
            --no-roofline --no-lk-roofline --no-ransac ${BENCH_EXTRA} > gpurun_out/ab/$tag.$r.json 2> gpurun_out/ab/$tag.$r.err
        rc=$?
        [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -3 gpurun_out/ab/$tag.$r.err; exit $rc; }
        python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$tag.$r.json')); s=d['stage_ms_per_step']; print(f'{\"$spec\":28s} round $r: {d[\"value\"]:8.1f} Mpx/s  lk {s[\"lk\"]:.3f} ms  parity {d.get(\"parity\")}')"
    done
done
