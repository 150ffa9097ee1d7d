#!/bin/bash
# A GPU session: GPU tests + smoke, the driver's bench command (with configs_other), probes, profiles.
# STEPS selects parts (default "tests bench cus"); every GPU step has its own time limit and
# the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r05a}
for S in ${STEPS:-tests bench cus}; do
  case $S in
    tests)
      echo "=== tests"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_tests_gpu.log 2>&1 || { tail -40 $OUT/${TAG}_tests_gpu.log; exit 1; }
      tail -2 $OUT/${TAG}_tests_gpu.log
      echo "=== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { tail -20 $OUT/${TAG}_smoke.log; exit 1; }
      tail -1 $OUT/${TAG}_smoke.log ;;
    bench)
      echo "=== bench (driver settings) ${BENCH_ARGS:-}"
      timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/${TAG}_bench_c5.json 2> $OUT/${TAG}_bench_c5.err || { tail -30 $OUT/${TAG}_bench_c5.err; exit 1; }
      cut -c1-400 $OUT/${TAG}_bench_c5.json ;;
    configs)
      for C in 1 2 3 4; do
        echo "=== bench config $C"
        timeout -k 10 600 python bench.py --config $C > $OUT/${TAG}_bench_c$C.json 2> $OUT/${TAG}_bench_c$C.err || { tail -30 $OUT/${TAG}_bench_c$C.err; exit 1; }
        cut -c1-300 $OUT/${TAG}_bench_c$C.json
      done ;;
    prof234)
      for C in 2 3 4; do
        echo "=== profile config $C"
        TAG=$TAG CONFIG=$C SKIP_BENCH=1 timeout -k 10 900 bash tools/profile_headline.sh > $OUT/${TAG}_prof_c$C.log 2>&1 || { tail -30 $OUT/${TAG}_prof_c$C.log; exit 1; }
        tail -3 $OUT/${TAG}_prof_c$C.log
      done ;;
    prof5)
      echo "=== profile config 5"
      TAG=$TAG CONFIG=5 SKIP_BENCH=1 timeout -k 10 1100 bash tools/profile_headline.sh > $OUT/${TAG}_prof_c5.log 2>&1 || { tail -30 $OUT/${TAG}_prof_c5.log; exit 1; }
      tail -3 $OUT/${TAG}_prof_c5.log ;;
    dp)
      echo "=== DP step latency"
      timeout -k 10 900 bash tools/dp_probe.sh > $OUT/${TAG}_dp_probe.log 2>&1 || { tail -20 $OUT/${TAG}_dp_probe.log; exit 1; }
      cat $OUT/${TAG}_dp_probe.log ;;
    eval)
      echo "=== evaluation passes"
      timeout -k 10 500 bash tools/eval_probe.sh > $OUT/${TAG}_eval_probe.log 2>&1 || { tail -20 $OUT/${TAG}_eval_probe.log; exit 1; }
      cat $OUT/${TAG}_eval_probe.log ;;
    trace64)
      echo "=== train-step stage trace on a 64-CU stream (libhbk_trace.so)"
      timeout -k 10 300 python tools/probe_mlp.py --trace --cus=64 > $OUT/${TAG}_trace64.log 2>&1 || { tail -20 $OUT/${TAG}_trace64.log; exit 1; }
      tail -5 $OUT/${TAG}_trace64.log ;;
    cus)
      echo "=== train step per CU count"
      timeout -k 10 500 bash tools/mlp_cus.sh > $OUT/${TAG}_mlp_cus.log 2>&1 || { tail -20 $OUT/${TAG}_mlp_cus.log; exit 1; }
      cat $OUT/${TAG}_mlp_cus.log ;;
  esac
done
echo "=== done"
