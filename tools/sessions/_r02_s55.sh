O=gpurun_out/r02_s55; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deferred or flat or max_single" > $O/t.log 2>&1 || exit 1
tail -3 $O/t.log
