O=gpurun_out/r02_s18; mkdir -p $O
export FMS_R8=1 FMS_PT=0,16,32 FMS_MAX_NP=5 FMS_STORE_NP=5
timeout -k 10 400 ./tools/flat_map_sweep f64 8192 12288 2880x23040 > $O/r8_f64_cached.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep f32 8192 16384 > $O/r8_f32_cached.log 2>&1 || exit 1
cat $O/r8_f64_cached.log $O/r8_f32_cached.log
