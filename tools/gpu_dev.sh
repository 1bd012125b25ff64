#!/bin/bash
# Development GPU session: optional parity tests, bench lines per config and
# rocprofv3 kernel stats.  Every GPU step has its own time limit; a fault,
# abort or timeout ends the script.
#   TESTS=1            run pytest -m gpu first
#   CFGS="udp64 imix"  bench configs (default: all three)
#   PROF="ipv6x"       configs to run under rocprofv3 --kernel-trace --stats
#   BENCH_ARGS=...     extra bench args
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/dev
mkdir -p "$O"
fatal() { case $1 in 0) ;; *) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > "$O/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 15 "$O/pytest_gpu.log"; fatal $rc pytest
fi
for cfg in ${CFGS-udp64 imix ipv6x}; do
  timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu --no-e2e ${BENCH_ARGS} > "$O/bench_$cfg.log" 2>&1; rc=$?
  echo "bench $cfg rc=$rc"
  python3 - "$O/bench_$cfg.log" <<'EOF' || tail -5 "$O/bench_$cfg.log"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(d["config"]["workload"][:3], d["value"], "Mpkt/s", r["achieved"], "GB/s frac", r["frac"], "read_frac", r.get("read_frac"), "kernel_ms", r.get("kernel_ms"), "copy", r.get("copy_gbs"))
EOF
  fatal $rc bench
done
cd /tmp && export TMPDIR=/tmp
for cfg in $PROF; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 5 --warmup 1 --no-cpu --no-e2e > "$O/prof_$cfg.log" 2>&1; rc=$?
  echo "prof $cfg rc=$rc"; fatal $rc prof
  f=$(find "$O/prof_$cfg" -name '*kernel_stats.csv' | head -n 1)
  python3 - "$f" <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:48]:50s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f}")
EOF
done
exit 0
