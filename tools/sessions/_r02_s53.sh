O=gpurun_out/r02_s53; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "test_flat_round_vs_round or test_deferred_writes_bitwise" > $O/t.log 2>&1 || exit 1
tail -5 $O/t.log
