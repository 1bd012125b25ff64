#!/bin/bash
# One GPU session (run under gpurun from the repo root): optional parity
# tests, then bench lines, each GPU step under its own time limit; a fault,
# abort or timeout ends the script.  Outputs in gpurun_out/$TAG/.
#   TAG=r02a TESTS=1 PYTEST_ARGS="-k c5" BENCH1="" BENCH2="--config imix --shards 8 --no-cpu"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/${TAG:-session}
mkdir -p "$O"
fatal() { case $1 in 0) ;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PYTEST_T:-900} python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_ARGS} > "$O/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 4 "$O/pytest_gpu.log"; fatal $rc pytest
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -n 2 "$O/smoke.log"; fatal $rc smoke
fi
for k in 1 2 3 4 5 6; do
  v=BENCH$k
  [ -z "${!v+x}" ] && continue
  timeout -k 10 ${BENCH_T:-600} python -u bench.py ${!v} > "$O/bench$k.log" 2> "$O/bench$k.err"; rc=$?
  echo "bench$k (${!v}) rc=$rc"; tail -c 3000 "$O/bench$k.log"; echo; fatal $rc bench$k
done
exit 0
