#!/bin/bash
# Kernel time of library variants (tools/build_variant.sh -> variants/<name>/)
# over bench configs, via tools/kbench.py --lib (HIP events, no result
# checks).  Each variant's library is loaded from its own path; the in-tree
# product library is never replaced ("base" = the in-tree build).
#   VARS="base u8" CFGS=imix,ipv6x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/var
mkdir -p "$O"
for v in $VARS; do
  if [ "$v" = base ]; then L=$R/netsniff-ng_amd/libnsdissect.so; else L=$R/variants/$v/libnsdissect.so; fi
  timeout -k 10 300 python -u tools/kbench.py --lib "$L" --configs ${CFGS:-udp64,imix,ipv6x} --steps ${STEPS:-10} ${KB_ARGS} > "$O/$v.log" 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -E "kernel_ms|phases" "$O/$v.log"
  [ $rc = 0 ] || { tail -5 "$O/$v.log"; exit $rc; }
done
exit 0
