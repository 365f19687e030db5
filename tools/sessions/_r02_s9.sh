O=gpurun_out/r02_s9; mkdir -p $O
timeout -k 10 300 ./tools/flat_map_sweep f64 32768 8192x65536 8192 2880x23040 4096x16384 > $O/fms_f64.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 8192x32768 > $O/fms_f32.log 2>&1
echo "rc=$?"
