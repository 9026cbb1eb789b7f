timeout -k 10 300 python -m pytest tests/test_gpu_codec.py -q -x > gpurun_out/kp4_pytest.log 2>&1 && \
bash tools/kprof.sh gpurun_out/kp4 volume "KMP_W3_PL=2 KMP_W3_WPE=4" "KMP_W3_PL=2 KMP_W3_WPE=3" "KMP_W3_PL=1" "KMP_DISABLE_WAVE=1" > gpurun_out/kp4.log 2>&1
rc=$?; tail -1 gpurun_out/kp4_pytest.log; cat gpurun_out/kp4.log; exit $rc
