O=gpurun_out/r02_s6; mkdir -p $O
export FMS_QUICK=1
timeout -k 10 300 ./tools/flat_map_sweep f64 32768 8192x65536 8192 2880x23040 > $O/fms_f64.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 > $O/fms_f32.log 2>&1 && \
unset FMS_QUICK && \
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo "rc=$?"
