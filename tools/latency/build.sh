#!/bin/bash
# Builds tools/latency/_build/latency_probe against the in-tree libalpenglow_rs.so (rpath);
# with an argument, latency_probe_<name> against alpenglow_amd/_lib/<name>.so (A/B builds).
set -eu
cd "$(dirname "$0")"
mkdir -p _build
lib=${1:-libalpenglow_rs}
out=_build/latency_probe${1:+_$1}
g++ -O2 -std=c++17 -I../../include latency_probe.cpp -L../../alpenglow_amd/_lib -l:$lib.so \
  -Wl,-rpath,'$ORIGIN/../../../alpenglow_amd/_lib' -o $out
[ $# -gt 0 ] || /opt/rocm/bin/hipcc -O2 -std=c++17 -I../../include latency_paths.cpp -L../../alpenglow_amd/_lib \
  -lalpenglow_rs -Wl,-rpath,'$ORIGIN/../../../alpenglow_amd/_lib' -o _build/latency_paths
