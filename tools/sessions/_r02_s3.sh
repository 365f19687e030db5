mkdir -p gpurun_out/r02_s3
timeout -k 10 300 ./tools/flat_map_sweep f64 32768 8192x65536 8192 2880x23040 > gpurun_out/r02_s3/flat_map_f64.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 > gpurun_out/r02_s3/flat_map_f32.log 2>&1
