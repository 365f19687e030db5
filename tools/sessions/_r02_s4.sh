O=gpurun_out/r02_s4; mkdir -p $O
timeout -k 10 300 ./tools/flat_map_sweep f64 32768 8192x65536 8192 2880x23040 > $O/vload_f64.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep_sload f64 32768 8192x65536 8192 2880x23040 > $O/sload_f64.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 > $O/vload_f32.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep_sload f32 32768 8192 > $O/sload_f32.log 2>&1
