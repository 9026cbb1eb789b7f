set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/probe1; mkdir -p $O
timeout -k 10 120 ./tools/probe_bw > $O/probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pmc2 -o run --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc2.log 2>&1
rc=$?; cat $O/probe.log; exit $rc
