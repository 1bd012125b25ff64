#!/bin/bash
# One GPU session for the round's record: parity tests, smoke, the default
# bench line (C2 headline with in-run PMC traffic, C3/C4 legs, both record
# forms, CPU baseline, e2e, replay, BPF), C5 on one GPU, and the rocprofv3
# kernel statistics of the default bench command (its PMC passes are the
# bench's own child runs).  Every GPU step has its own time limit; a fault,
# abort or timeout ends the script.  Outputs go to gpurun_out/round/;
# tools/collect_profiles.py <tag> turns them into profiles/<tag>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/round
mkdir -p "$O"
fatal() { case $1 in 0) ;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 3 "$O/pytest_gpu.log"; fatal $rc pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -n 2 "$O/smoke.log"; fatal $rc smoke
fi
timeout -k 10 900 python -u bench.py > "$O/bench_default.log" 2> "$O/bench_default.err"; rc=$?
echo "bench default rc=$rc"; tail -c 600 "$O/bench_default.log"; echo; fatal $rc bench
timeout -k 10 900 python -u bench.py --config imix --shards 8 --no-cpu --no-e2e --no-replay --no-bpf --no-legs --steps 5 --warmup 1 > "$O/bench_c5.log" 2> "$O/bench_c5.err"; rc=$?
echo "bench c5 rc=$rc"; tail -c 300 "$O/bench_c5.log"; echo; fatal $rc bench_c5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-e2e --no-replay --no-pmc --steps 10 --warmup 2 > "$O/stats.log" 2>&1; rc=$?
echo "stats rc=$rc"; fatal $rc stats
exit 0
