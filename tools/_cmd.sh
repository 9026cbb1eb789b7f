bash tools/kprof.sh gpurun_out/kp1 volume "KMP_DISABLE_WAVE=1" "KMP_W3_ROLL=1" "KMP_W3_XCD=1" "KMP_W3_XCD=0" "KMP_W3_PL=2" "KMP_W3_PL=2 KMP_W3_XCD=0" > gpurun_out/kp1.log 2>&1
rc=$?; cat gpurun_out/kp1.log; exit $rc
