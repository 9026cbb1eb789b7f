set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3fin1; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; return $rc; }
step debug_parity 600 env KMP_DEBUG=1 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_linear.py tests/test_packing.py tests/test_gpu_fuzz_rice.py -m gpu -x -q --timeout 120 --timeout-method thread && \
step bench_n2_gloo 300 env KMP_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-e2e
rc=$?
tail -2 $O/debug_parity.log; tail -1 $O/bench_n2_gloo.log | cut -c1-300
exit $rc
