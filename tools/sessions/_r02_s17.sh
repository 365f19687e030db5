O=gpurun_out/r02_s17; mkdir -p $O
export FMS_R8=1 FMS_PT=0,32 FMS_MAX_NP=5 FMS_STORE_NP=5
timeout -k 10 400 ./tools/flat_map_sweep f64 32768 8192x65536 > $O/r8_f64.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 > $O/r8_f32.log 2>&1 || exit 1
cat $O/r8_f64.log $O/r8_f32.log
