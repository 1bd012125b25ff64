#!/bin/bash
# Per-kernel times of library variants on one bench config, via rocprofv3
# stats.  Runs on the GPU box's scratch copy of the tree: each variant's
# variants/<name>/libnsdissect.so is copied over the in-tree library for its
# run ("base" = the in-tree build), and the in-tree build is restored after.
#   VARS="base u8" CFG=imix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/var
mkdir -p "$O"
LIB=$R/netsniff-ng_amd/libnsdissect.so
cp "$LIB" "$O/base.so"
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  if [ "$v" = base ]; then cp "$O/base.so" "$LIB"; else cp "$R/variants/$v/libnsdissect.so" "$LIB"; fi
  for cfg in ${CFG:-udp64}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${v}_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 5 --warmup 1 --no-cpu --no-e2e --no-replay --no-legs --no-pmc ${BENCH_ARGS} > "$O/${v}_$cfg.log" 2>&1; rc=$?
    echo "== $v $cfg rc=$rc"; [ $rc = 0 ] || { tail -5 "$O/${v}_$cfg.log"; cp "$O/base.so" "$LIB"; exit $rc; }
    f=$(find "$O/${v}_$cfg" -name '*kernel_stats.csv' | head -n 1)
    python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "nsd::" in r["Name"]:
        print(f"  {r['Name'].split('(')[0][5:]:28s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
  done
done
cp "$O/base.so" "$LIB"
exit 0
