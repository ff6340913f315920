#!/bin/bash
# Same-box A/B of variant libraries (motion_detection_amd/lib_var/<name>/libmdx.so, "head" = the
# in-tree build): default 1080p x 32 bench step only, alternating ROUNDS times.
# Usage (GPU box): ROUNDS=2 bash scripts/var_ab.sh head old w5 ...
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
    for v in "$@"; do
        if [ "$v" = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
        timeout -k 10 120 python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu --no-live --no-4k --no-roofline \
            --no-lk-roofline ${BENCH_EXTRA} > gpurun_out/ab/$v.$r.json 2> gpurun_out/ab/$v.$r.err
        rc=$?
        [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/ab/$v.$r.err; exit $rc; }
        python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$r.json')); s=d['stage_ms_per_step']; print(f'$v round $r: {d[\"value\"]:8.1f} Mpx/s  lk {s[\"lk\"]:.3f} ms  total {s[\"total\"]:.3f} ms')"
    done
done
