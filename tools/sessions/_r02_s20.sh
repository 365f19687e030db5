O=gpurun_out/r02_s20; mkdir -p $O
bash tools/gpu_session.sh r02_s20 tests defer || exit 1
export FMS_EVERY=1 FMS_PT=0,4,8,16
timeout -k 10 400 ./tools/flat_map_sweep_ptall f64 32768 8192x65536 16384x65536 > $O/every_f64_nt.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep_ptall f64 8192 2880x23040 4096x16384 > $O/every_f64_cached.log 2>&1 || exit 1
timeout -k 10 300 ./tools/flat_map_sweep_ptall f32 32768 > $O/every_f32.log 2>&1 || exit 1
cat $O/every_*.log
