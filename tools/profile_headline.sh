#!/bin/bash
# The headline's evidence, reproducible from one command on the GPU box:
#   1. the driver's bench command (N = 1)                  -> $OUT/${TAG}_bench_c5.json
#   2. rocprofv3 --kernel-trace --stats of the same bench   -> kernel_stats + per-step trace summary
#   3. FETCH_SIZE, WRITE_SIZE and SQ busy counter passes (one rocprofv3 --pmc run each)
#   4. tools/prof_summary.py: dispatches between bench.py's markers only
#      (timed region 1 -> 2, sequential stage steps 3 -> 4), per step
# Every GPU step has its own time limit; the first failure ends the script.
# usage: TAG=r03a bash tools/profile_headline.sh   (CONFIG=5 default; BENCH_ARGS extra)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r03a}
C=${CONFIG:-5}
BA="--config $C --other-configs= ${BENCH_ARGS:-}"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"

if [ -z "$SKIP_BENCH" ]; then
  echo "=== bench ($BA --steps 20 --warmup 5)"
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 $BA > $OUT/${TAG}_bench_c$C.json 2> $OUT/${TAG}_bench_c$C.err \
    || { tail -30 $OUT/${TAG}_bench_c$C.err; exit 1; }
  cut -c1-600 $OUT/${TAG}_bench_c$C.json
fi
echo "=== kernel trace"
rm -rf $OUT/${TAG}_trace_c$C
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/${TAG}_trace_c$C -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu $BA > $OUT/${TAG}_trace_c$C.log 2>&1 \
  || { tail -20 $OUT/${TAG}_trace_c$C.log; exit 1; }
find $OUT/${TAG}_trace_c$C -name "*kernel_stats.csv" -exec cp {} $OUT/${TAG}_kernel_stats_c$C.csv \;
for P in fetch write sq; do
  case $P in fetch) CTR=FETCH_SIZE ;; write) CTR=WRITE_SIZE ;; sq) CTR=$SQ ;; esac
  echo "=== pmc $P"
  rm -rf $OUT/${TAG}_pmc${P}_c$C
  timeout -k 10 600 rocprofv3 --pmc $CTR -f csv -d $OUT/${TAG}_pmc${P}_c$C -o run -- \
    python3 bench.py --steps 1 --warmup 1 --stage-steps 1 --no-cpu --no-check $BA > $OUT/${TAG}_pmc${P}_c$C.log 2>&1 \
    || { tail -20 $OUT/${TAG}_pmc${P}_c$C.log; exit 1; }
done
echo "=== summaries"
python3 tools/prof_summary.py --trace $OUT/${TAG}_trace_c$C --steps 5 --stage-steps 2 --config $C \
  --label "$TAG kernel trace: bench.py --steps 5 --warmup 2 --no-cpu $BA" --out $OUT/${TAG}_trace_c$C.json
python3 tools/prof_summary.py --fetch $OUT/${TAG}_pmcfetch_c$C --write $OUT/${TAG}_pmcwrite_c$C --sq $OUT/${TAG}_pmcsq_c$C \
  --steps 1 --stage-steps 1 --config $C \
  --label "$TAG counter passes: bench.py --steps 1 --warmup 1 --stage-steps 1 --no-cpu --no-check $BA" \
  --out $OUT/${TAG}_pmc_c$C.json
# the raw per-dispatch CSVs exceed gpurun's 64 MiB copy-back: keep the summaries and kernel_stats
rm -rf $OUT/${TAG}_trace_c$C $OUT/${TAG}_pmcfetch_c$C $OUT/${TAG}_pmcwrite_c$C $OUT/${TAG}_pmcsq_c$C
echo "=== done"
