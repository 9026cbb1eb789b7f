#!/bin/bash
# SQ (shader sequencer) counters of the fused codec kernels, two rocprofv3 --pmc passes of at most
# 8 SQ counters each (MI355X_MICROARCH.md § rocprofv3 PMC slots), summarised per kernel and per
# wave by tools/sq_summary.py:
#   bash tools/sq_counters.sh OUTDIR "ktime args" ["ENV=.. ENV=.."] [script, default tools/ktime.py]
# e.g. bash tools/sq_counters.sh gpurun_out/sq_l3p "volume 1 3 linear" "KMP_W3_XCD=1"
#      bash tools/sq_counters.sh gpurun_out/sq_gen "lin1_odd 3" "" tools/ktime_generic.py
set -o pipefail
export TMPDIR=/tmp
O=$1; ARGS=$2; ENVS=$3; PROG=${4:-tools/ktime.py}
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  ( for kv in $ENVS; do export "$kv"; done
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $O/p$i -o run -- python3 $PROG $ARGS > $O/p$i.log 2>&1 ) || exit 1
done
python3 tools/sq_summary.py $O/p1 $O/p2
