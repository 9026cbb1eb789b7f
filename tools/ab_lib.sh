#!/bin/bash
# A/B of two builds of the library on one box, alternating: bash tools/ab_lib.sh OUT ROWS [rounds]
#   kompressor_amd/libkompressor_hip.so (the working tree) vs kompressor_amd/libkompressor_hip_prev.so
#   (a build of an earlier commit, KOMPRESSOR_HIP_LIB), tools/bench_rows.py --rows ROWS each time.
set -o pipefail
OUT=$1; ROWS=$2; N=${3:-2}
for i in $(seq $N); do
  for lib in libkompressor_hip.so libkompressor_hip_prev.so; do
    echo "## $lib" >> $OUT
    KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 200 python -u tools/bench_rows.py --rows $ROWS --no-cpu --reps 10 2>&1 | grep -v amdgpu.ids >> $OUT || exit 1
  done
done
