#!/bin/bash
# Diagnostic build (not the product): tools/xh8_repro/_build/libxh8_repro.so and its ISA.
set -eu
cd "$(dirname "$0")"
mkdir -p _build
CS=../../alpenglow_amd/csrc
FL="-O3 -std=c++20 -fno-slp-vectorize --offload-arch=gfx950 -I../../include -I$CS -mllvm -amdgpu-promote-alloca-to-vector-limit=2048"
/opt/rocm/bin/hipcc $FL -fPIC -shared xh8_repro.hip -o _build/libxh8_repro.so
/opt/rocm/bin/hipcc $FL --cuda-device-only -S -x hip xh8_repro.hip -o _build/xh8_repro.s
