#!/bin/bash
# One GPU session for the round's record: parity tests, smoke, the three
# bench lines, rocprofv3 kernel stats per config and the HBM byte counters
# (FETCH_SIZE / WRITE_SIZE in separate --pmc passes, MI355X_MICROARCH.md
# "HBM").  Every GPU step has its own time limit; a fault, abort or timeout
# ends the script.  Outputs go to gpurun_out/round/; tools/collect_profiles.py
# turns them into profiles/<tag>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/round
mkdir -p "$O"
fatal() { case $1 in 0) ;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 3 "$O/pytest_gpu.log"; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -n 2 "$O/smoke.log"; fatal $rc smoke
timeout -k 10 600 python bench.py > "$O/bench_udp64.log" 2>&1; rc=$?
echo "bench udp64 rc=$rc"; fatal $rc bench
for cfg in imix ipv6x; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu > "$O/bench_$cfg.log" 2>&1; rc=$?
  echo "bench $cfg rc=$rc"; fatal $rc bench
done
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-e2e --no-replay --steps 10 --warmup 2"
for cfg in udp64 imix ipv6x; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg $ARGS > "$O/stats_$cfg.log" 2>&1; rc=$?
  echo "stats $cfg rc=$rc"; fatal $rc stats
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -d "$O/pmc_${cfg}_$ctr" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg $ARGS > "$O/pmc_${cfg}_$ctr.log" 2>&1; rc=$?
    echo "pmc $cfg $ctr rc=$rc"; fatal $rc pmc
  done
done
exit 0
