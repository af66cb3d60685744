#!/bin/bash
# build the k-NN lab library (development tool)
set -e
cd "$(dirname "$0")"
R=../..
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -I$R/include -I$R/fast-livo-noted_amd/csrc \
  -o ${OUT:-libknn_lab.so} knn_lab.hip $R/fast-livo-noted_amd/csrc/map_build.cpp -pthread -Wno-unused-value -Wno-unused-result ${EXTRA:-}
