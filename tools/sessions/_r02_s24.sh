O=gpurun_out/r02_s24; mkdir -p $O
FMS_EVERY=1 FMS_U2=1 FMS_PT=0,2,4,8 timeout -k 10 400 ./tools/flat_map_sweep f64 32768 8192x65536 > $O/every_u2_f64.log 2>&1 || exit 1
FMS_EVERY=1 FMS_U2=1 FMS_PT=0,2,4,8 timeout -k 10 300 ./tools/flat_map_sweep f32 32768 > $O/every_u2_f32.log 2>&1 || exit 1
cat $O/every_u2_*.log
bash tools/gpu_session.sh r02_s24 bench defer_pmc
