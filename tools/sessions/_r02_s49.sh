O=gpurun_out/r02_s49; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test_bench.log 2>&1 || exit 1
tail -8 $O/test_bench.log
