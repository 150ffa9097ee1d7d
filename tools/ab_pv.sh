#!/bin/bash
# A/B of the pitch vocoder: the headline stagewise test and tools/probe_pitch.py
# on the current library and on lib/libhbk_oldpv.so (built from the previous
# hbk_augment.hip). A test failure (exit 1) is reported and the next step runs;
# any other non-zero exit (time limit, fault) ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in libhbk_oldpv.so libhbk.so; do
  HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abpv_$L.log 2>&1
  rc=$?
  echo "== $L e2e rc=$rc"; grep -E "passed|failed|Error:" gpurun_out/abpv_$L.log | tail -3
  [ $rc -gt 1 ] && exit $rc
  HBK_LIB=hey-buddy_amd/lib/$L timeout -k 10 120 python tools/probe_pitch.py 25600 5 || exit 1
done
echo "=== done"
