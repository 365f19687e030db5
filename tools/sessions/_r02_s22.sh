O=gpurun_out/r02_s22; mkdir -p $O
export FMS_EVERY=1 FMS_PT=0,2,3,4,5,6
timeout -k 10 400 ./tools/flat_map_sweep f64 32768 8192x65536 > $O/every2_f64_nt.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep f32 32768 > $O/every2_f32.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep f64 8192 > $O/every2_f64_cached.log 2>&1 || exit 1
cat $O/every2_*.log
