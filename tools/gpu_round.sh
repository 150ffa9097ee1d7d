#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel stats (+ optional PMC passes).
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
step() { echo "=== $1"; }
step tests
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests_$TAG.log 2>&1 || { tail -40 $OUT/tests_$TAG.log; exit 1; }
tail -3 $OUT/tests_$TAG.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -20 $OUT/smoke_$TAG.log; exit 1; }
cat $OUT/smoke_$TAG.log | tail -2
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
if [ -n "$PROF" ]; then
  step rocprof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { tail -20 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
if [ -n "$PMC" ]; then
  step pmc
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc_fetch_$TAG -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/pmc_fetch_$TAG.log 2>&1 || { tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_write_$TAG -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/pmc_write_$TAG.log 2>&1 || { tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
  find $OUT/pmc_*_$TAG -name "*.csv" | head
fi
echo "=== done"
