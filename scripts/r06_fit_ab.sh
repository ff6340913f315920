set -o pipefail
mkdir -p gpurun_out/fit
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fit/pytest.log 2>&1 || { tail -30 gpurun_out/fit/pytest.log; exit 1; }
tail -2 gpurun_out/fit/pytest.log
ROUNDS=3 bash scripts/r06_ab.sh hd head head:MDX_LK_XCALL=1 || exit 1
for v in hd head hd head; do
  if [ $v = head ]; then unset MDX_LIB_PATH; else export MDX_LIB_PATH=$PWD/motion_detection_amd/lib_var/$v/libmdx.so; fi
  timeout -k 10 200 python3 bench.py --workload c4 --config 8k --bands 8 --inflight 2 --steps 10 --warmup 3 > gpurun_out/fit/c4_$v.json 2> gpurun_out/fit/c4_$v.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/fit/c4_$v.json')); print('$v c4', d.get('ms_per_step'), d.get('value'), d.get('parity'))"
done
