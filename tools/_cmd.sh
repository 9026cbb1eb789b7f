set -o pipefail
mkdir -p gpurun_out/w2p
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -x -v --timeout 120 --timeout-method thread -k "wave2d_p12 or img" > gpurun_out/w2p/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/w2p/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/w2p/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_rows.py --rows image_mean_p1 --no-cpu > gpurun_out/w2p/rows.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/w2p/rows.log; exit $rc
