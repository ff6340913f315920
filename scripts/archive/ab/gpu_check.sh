#!/bin/bash
# GPU-box check: smoke, then the -m gpu suite.  Stops after any crash-like exit
# (signal / timeout), continues past an ordinary assertion failure (exit 1).
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
exit $rc
