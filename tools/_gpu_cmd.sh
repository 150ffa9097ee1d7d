set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_classifier_gpu.py tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/cls_tests.log 2>&1 || { tail -30 gpurun_out/cls_tests.log; exit 1; }
tail -2 gpurun_out/cls_tests.log
timeout -k 10 200 python bench.py --config 4 --no-cpu > gpurun_out/c4.json 2>gpurun_out/c4.err || { tail -5 gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --config 4 --steps 20 --warmup 2 --no-cpu > gpurun_out/prof_c4.log 2>&1
