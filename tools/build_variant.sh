#!/bin/bash
# Build an experiment variant of libnsdissect.so into variants/<name>/
# (git-ignored; travels to the GPU box with gpurun).  Tuning knobs come in as
# -D flags; experiments that change code (e.g. skip a phase to time the
# rest) are patches (paths csrc/...) applied to a scratch copy of the
# sources, never switches in the product sources.
#   tools/build_variant.sh u8 -DNSD_CSUM_U=8
#   PATCH=/tmp/nop2.patch tools/build_variant.sh nop2
#   REV=HEAD~1 tools/build_variant.sh prev        (a committed revision's kernels)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
d=variants/$name
rm -rf $d && mkdir -p $d/x/a $d/x/include
if [ -n "$REV" ]; then   # the sources of a git revision instead of the working tree
  mkdir -p $d/x/a/csrc && git archive "$REV" netsniff-ng_amd/csrc | tar -x -C $d/x/a --strip-components=1
  git show "$REV":include/netsniff_dissect.h > $d/x/include/netsniff_dissect.h
else
  cp -r netsniff-ng_amd/csrc $d/x/a/csrc
fi
[ -n "$REV" ] || cp include/netsniff_dissect.h $d/x/include/
if [ -n "$PATCH" ]; then patch -s -d $d/x/a -p0 < "$PATCH"; fi
make -s -C netsniff-ng_amd
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $*"
$H -c $d/x/a/csrc/nsd_kernels.hip -o $d/k.o
objs="$d/k.o"
for f in nsd_bpf nsd_cpu nsd_host nsd_pipe nsd_format nsd_lookup nsd_pcap nsd_proto; do
  objs="$objs netsniff-ng_amd/build/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libnsdissect.so $objs
rm -rf $d/k.o $d/x
