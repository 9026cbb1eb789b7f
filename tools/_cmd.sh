timeout -k 10 300 python -m pytest tests/test_gpu_codec.py tests/test_gpu_linear.py tests/test_gpu_stream.py -q -x > gpurun_out/w2_pytest.log 2>&1 && \
bash tools/kprof.sh gpurun_out/kw2 image "KMP_W2_XCD=1" "KMP_W2_XCD=0" "KMP_DISABLE_WAVE=1" > gpurun_out/kw2.log 2>&1
rc=$?; tail -3 gpurun_out/w2_pytest.log; cat gpurun_out/kw2.log; exit $rc
