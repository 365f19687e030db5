O=gpurun_out/r02_s8; mkdir -p $O
timeout -k 10 60 ./tests/cpp/test_reduce > $O/test_reduce.log 2>&1 || { cat $O/test_reduce.log; exit 1; }
cat $O/test_reduce.log
export FMS_QUICK=1
timeout -k 10 200 ./tools/flat_map_sweep f64 32768 8192 8192x65536 > $O/fms_f64.log 2>&1 && \
timeout -k 10 200 ./tools/flat_map_sweep f32 32768 > $O/fms_f32.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "rc=$?"
