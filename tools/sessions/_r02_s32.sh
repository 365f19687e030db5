O=gpurun_out/r02_s32; mkdir -p $O
for rep in 1 2; do for V in flat_map_sweep flat_map_sweep_old; do
  FMS_R8=1 FMS_PT=0,16,32 FMS_MAX_NP=5 FMS_STORE_NP=5 timeout -k 10 300 ./tools/$V f64 32768 8192 > $O/${V}_$rep.log 2>&1 || exit 1
done; done
