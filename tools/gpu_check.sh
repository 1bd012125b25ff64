#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
R=$(pwd)
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 ${PYTEST_T:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log; fatal $rc pytest
if [ -n "$ONLY_TESTS" ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -n 5 gpurun_out/smoke.log; fatal $rc smoke
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.log; fatal $rc bench
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu ${BENCH_ARGS} > "$R/gpurun_out/prof.log" 2>&1; rc=$?
  echo "prof rc=$rc"; tail -n 5 "$R/gpurun_out/prof.log"; fatal $rc prof
fi
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -d "$R/gpurun_out/pmc_$ctr" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu ${BENCH_ARGS} > "$R/gpurun_out/pmc_$ctr.log" 2>&1; rc=$?
    echo "pmc $ctr rc=$rc"; tail -n 3 "$R/gpurun_out/pmc_$ctr.log"; fatal $rc pmc
  done
fi
exit 0
