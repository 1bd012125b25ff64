#!/bin/bash
# Build a variant of libnsdissect.so with extra compile flags into
# variants/<name>/ (git-ignored; travels to the GPU box with gpurun).
#   tools/build_variant.sh u8 -DNSD_CSUM_U=8
set -e
cd "$(dirname "$0")/.."
name=$1; shift
d=variants/$name
mkdir -p $d
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $*"
$H -c netsniff-ng_amd/csrc/nsd_kernels.hip -o $d/k.o
objs="$d/k.o"
for f in nsd_bpf nsd_host nsd_pipe nsd_format nsd_lookup nsd_pcap; do
  [ netsniff-ng_amd/build/$f.o -nt netsniff-ng_amd/csrc/$f.cpp ] || [ netsniff-ng_amd/build/$f.o -nt netsniff-ng_amd/csrc/$f.hip ] || make -s -C netsniff-ng_amd
  objs="$objs netsniff-ng_amd/build/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libnsdissect.so $objs
rm -f $d/k.o
