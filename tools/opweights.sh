#!/bin/bash
# Static VALU instruction count of each ocml FP64 function on gfx950 (see opweights.json).
set -e
d=$(mktemp -d)
for f in exp log sqrt asin sin cos atan div none; do
  if [ $f = div ]; then expr="a / b[i]"; elif [ $f = none ]; then expr="a + b[i]"; else expr="$f(a)"; fi
  printf '#include <hip/hip_runtime.h>\nextern "C" __global__ void k(const double* __restrict__ a_, const double* __restrict__ b, double* __restrict__ o) {\n  int i = blockIdx.x*256+threadIdx.x; double a = a_[i];\n  o[i] = %s;\n}\n' "$expr" > $d/k_$f.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -S --cuda-device-only -o $d/k_$f.s $d/k_$f.hip
  echo "$f $(awk '/^k:/,/s_endpgm/' $d/k_$f.s | grep -cE '^\s+v_')"
done
rm -rf $d
