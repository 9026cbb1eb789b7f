#!/bin/bash
# rocprofv3 kernel times of tools/ktime.py (encode / decode alternating) for two libraries in
# alternation: the working tree's libkompressor_hip.so (A) and kompressor_amd/libkompressor_hip_<B>.so.
#   bash tools/ab_kprof.sh OUTDIR B "ktime args" [rounds] [kernel-name filter]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$1; B=$2; ARGS=$3; N=${4:-2}; F=${5:-kmp}
mkdir -p $O
for i in $(seq $N); do
  for lib in libkompressor_hip.so libkompressor_hip_$B.so; do
    d=$O/r${i}_${lib%.so}
    KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/$lib timeout -k 10 180 rocprofv3 --kernel-trace -d $d -o run -- python3 tools/ktime.py $ARGS > $d.log 2>&1 || { cat $d.log | tail -5; exit 1; }
    db=$(find $d -name "run_results.db" | head -1)
    echo "== round $i $lib"
    python3 tools/kstats.py $db $F
  done
done
