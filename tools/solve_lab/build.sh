#!/bin/bash
# build the k_solve lab (development tool): the product kernels with phase marks
set -e
cd "$(dirname "$0")"
R=../..
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt \
  -DLIVO_SOLVE_PROF -fgpu-rdc -I$R/include -I$R/fast-livo-noted_amd/csrc \
  -o ${OUT:-solve_lab} solve_lab.cpp -x hip $R/fast-livo-noted_amd/csrc/livo_kernels.hip ${EXTRA:-}
