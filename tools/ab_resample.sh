set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_augment.py tests/test_e2e_gpu.py -m gpu > gpurun_out/rsm_tests.log 2>&1 || { tail -30 gpurun_out/rsm_tests.log; exit 1; }
tail -1 gpurun_out/rsm_tests.log
for V in mfma valu mfma valu; do
  if [ $V = valu ]; then export HBK_PS_RESAMPLE_VALU=1; else unset HBK_PS_RESAMPLE_VALU; fi
  echo "== $V"; timeout -k 10 120 python tools/probe_pitch.py 25600 5 2>&1 | grep us/clip || exit 1
done
