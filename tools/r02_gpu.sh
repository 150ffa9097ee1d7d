#!/bin/bash
# Round-2 GPU session: new-kernel tests first, then the whole GPU suite, the
# headline bench (config 5) and its rocprof kernel summary. Every GPU step has
# its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r02a}
if [ -n "$FIRST_TESTS" ]; then
  echo "=== first tests: $FIRST_TESTS"
  timeout -k 10 600 python -u -m pytest $FIRST_TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/first_$TAG.log 2>&1 || { tail -60 $OUT/first_$TAG.log; exit 1; }
  tail -3 $OUT/first_$TAG.log
fi
if [ -z "$SKIP_TESTS" ]; then
  echo "=== tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || { tail -60 $OUT/tests_$TAG.log; exit 1; }
  tail -2 $OUT/tests_$TAG.log
  echo "=== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -20 $OUT/smoke_$TAG.log; exit 1; }
  tail -1 $OUT/smoke_$TAG.log
fi
for C in ${CONFIGS:-5}; do
  echo "=== bench config $C"
  timeout -k 10 600 python bench.py --config $C ${BENCH_ARGS:-} > $OUT/bench_${TAG}_c$C.json 2> $OUT/bench_${TAG}_c$C.err || { tail -30 $OUT/bench_${TAG}_c$C.err; exit 1; }
  cat $OUT/bench_${TAG}_c$C.json
done
if [ -n "$PROF" ]; then
  for C in ${PROF_CONFIGS:-5}; do
    echo "=== rocprof config $C"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_${TAG}_c$C -o run -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu > $OUT/prof_${TAG}_c$C.log 2>&1 || { tail -20 $OUT/prof_${TAG}_c$C.log; exit 1; }
    find $OUT/prof_${TAG}_c$C -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_${TAG}_c$C.csv
  done
fi
if [ -n "$PMC" ]; then
  for C in ${PROF_CONFIGS:-5}; do
    echo "=== pmc config $C"
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmcf_${TAG}_c$C -o run -- python3 bench.py --config $C --steps 1 --warmup 0 --no-cpu --no-check --overlap off > $OUT/pmcf_${TAG}_c$C.log 2>&1 || { tail -20 $OUT/pmcf_${TAG}_c$C.log; exit 1; }
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmcw_${TAG}_c$C -o run -- python3 bench.py --config $C --steps 1 --warmup 0 --no-cpu --no-check --overlap off > $OUT/pmcw_${TAG}_c$C.log 2>&1 || { tail -20 $OUT/pmcw_${TAG}_c$C.log; exit 1; }
    python tools/pmc_summary.py $OUT/pmcf_${TAG}_c$C $OUT/pmcw_${TAG}_c$C $OUT/pmc_${TAG}_c$C.json $C
  done
fi
echo "=== done"
