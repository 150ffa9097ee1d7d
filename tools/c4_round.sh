export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_classifier_gpu.py tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c4_tests.log 2>&1 || { tail -40 gpurun_out/c4_tests.log; exit 1; }
tail -2 gpurun_out/c4_tests.log
timeout -k 10 200 python bench.py --config 4 --steps 50 --warmup 5 > gpurun_out/c4h.json 2>gpurun_out/c4h.err || { tail -5 gpurun_out/c4h.err; exit 1; }
cut -c1-300 gpurun_out/c4h.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c4h -o run -- python3 bench.py --config 4 --steps 20 --warmup 2 --no-cpu > gpurun_out/prof_c4h.log 2>&1 || exit 1
