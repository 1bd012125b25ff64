#!/bin/bash
# Per-kernel times of library variants (variants/<name>/libnsdissect.so;
# "base" = the in-tree build) on one bench config, via rocprofv3 stats.
#   VARS="base u8" CFG=imix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/var
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  if [ "$v" = base ]; then unset NSD_LIB; else export NSD_LIB=$R/variants/$v/libnsdissect.so; fi
  for cfg in ${CFG:-udp64}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${v}_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 5 --warmup 1 --no-cpu --no-e2e --no-replay ${BENCH_ARGS} > "$O/${v}_$cfg.log" 2>&1; rc=$?
    echo "== $v $cfg rc=$rc"; [ $rc = 0 ] || { tail -5 "$O/${v}_$cfg.log"; exit $rc; }
    f=$(find "$O/${v}_$cfg" -name '*kernel_stats.csv' | head -n 1)
    python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "nsd::" in r["Name"]:
        print(f"  {r['Name'].split('(')[0][5:]:28s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
  done
done
exit 0
