set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/r4c6; mkdir -p $O
KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/libkompressor_hip_sub4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -k categorical -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "" _sub4 "" _sub4; do
  echo "== $v" >> $O/ab.log
  KOMPRESSOR_HIP_LIB=$PWD/kompressor_amd/libkompressor_hip$v.so timeout -k 10 200 python -u tools/bench_rows.py --rows categorical --no-cpu --reps 10 2>&1 | grep '"categorical' >> $O/ab.log || exit 1
done
python3 - <<'PY'
import json
cur=None; res={}
for l in open('gpurun_out/r4c6/ab.log'):
    if l.startswith('=='): cur=l.strip(); continue
    d=json.loads(l); res.setdefault(d['row'],[]).append((cur,d['us']))
for k,v in res.items(): print(k, v)
PY
