O=gpurun_out/r02_s10; mkdir -p $O
export FMS_PT=0,4,8,16,32
timeout -k 10 400 ./tools/flat_map_sweep f64 32768 32768x65536 16384x65536 8192x65536 > $O/fms_f64_nt.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f64 8192 2880x23040 12288 > $O/fms_f64_cached.log 2>&1 && \
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 > $O/fms_f32.log 2>&1
echo "rc=$?"
