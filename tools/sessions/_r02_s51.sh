O=gpurun_out/r02_s51; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_bench.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test_bench.log 2>&1 || exit 1
tail -3 $O/test_bench.log
