#!/bin/bash
# Kernel time of library variants (tools/build_variant.sh -> variants/<name>/)
# over bench configs, via tools/kbench.py (HIP events, no result checks).
# Runs on the GPU box's scratch copy of the tree: each variant's library is
# copied over the in-tree one for its run ("base" = the in-tree build); the
# in-tree build is restored after.
#   VARS="base u8" CFGS=imix,ipv6x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/var
mkdir -p "$O"
LIB=$R/netsniff-ng_amd/libnsdissect.so
cp "$LIB" "$O/base.so"
for v in $VARS; do
  if [ "$v" = base ]; then cp "$O/base.so" "$LIB"; else cp "$R/variants/$v/libnsdissect.so" "$LIB"; fi
  timeout -k 10 300 python -u tools/kbench.py --configs ${CFGS:-udp64,imix,ipv6x} --steps ${STEPS:-10} ${KB_ARGS} > "$O/$v.log" 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -E "kernel_ms|phases" "$O/$v.log"
  [ $rc = 0 ] || { tail -5 "$O/$v.log"; cp "$O/base.so" "$LIB"; exit $rc; }
done
cp "$O/base.so" "$LIB"
exit 0
