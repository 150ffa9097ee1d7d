#!/bin/bash
# Round-3 GPU session: FIRST_TESTS (if set) first, then optionally the whole
# GPU suite + smoke (FULL=1), then the headline profile (PROFILE=1,
# tools/profile_headline.sh). Each GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r03x}
if [ -n "$FIRST_TESTS" ]; then
  echo "=== first tests: $FIRST_TESTS"
  timeout -k 10 600 python -u -m pytest $FIRST_TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_first.log 2>&1 || { tail -60 $OUT/${TAG}_first.log; exit 1; }
  tail -3 $OUT/${TAG}_first.log
fi
if [ -n "$FULL" ]; then
  echo "=== tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_gpu.log 2>&1 || { tail -60 $OUT/${TAG}_tests_gpu.log; exit 1; }
  tail -2 $OUT/${TAG}_tests_gpu.log
  echo "=== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { tail -20 $OUT/${TAG}_smoke.log; exit 1; }
  tail -1 $OUT/${TAG}_smoke.log
fi
if [ -n "$PROFILE" ]; then
  TAG=$TAG bash tools/profile_headline.sh || exit 1
fi
if [ -n "$CMD" ]; then
  echo "=== $CMD"
  timeout -k 10 ${CMD_TIMEOUT:-300} bash -c "$CMD" > $OUT/${TAG}_cmd.log 2>&1 || { tail -40 $OUT/${TAG}_cmd.log; exit 1; }
  tail -${CMD_TAIL:-20} $OUT/${TAG}_cmd.log
fi
echo "=== all done"
