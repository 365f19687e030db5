O=gpurun_out/r02_s30; mkdir -p $O
FMS_R1=1 FMS_PT=0,4,8,16 FMS_MAX_NP=5 FMS_STORE_NP=5 timeout -k 10 400 ./tools/flat_map_sweep f64 8192 2880x23040 12288 > $O/r1_f64_cached.log 2>&1 || exit 1
FMS_R8=1 FMS_PT=0,4,8,16 FMS_MAX_NP=5 FMS_STORE_NP=5 timeout -k 10 400 ./tools/flat_map_sweep f64 8192 2880x23040 > $O/r8_f64_cached.log 2>&1 || exit 1
FMS_R1=1 FMS_PT=0,4,8,16 FMS_MAX_NP=5 FMS_STORE_NP=5 timeout -k 10 400 ./tools/flat_map_sweep f32 8192 > $O/r1_f32_cached.log 2>&1 || exit 1
cat $O/*.log
