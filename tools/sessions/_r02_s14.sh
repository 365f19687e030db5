O=gpurun_out/r02_s14; mkdir -p $O
export FMS_PT=0,16,32 FMS_MAX_NP=5
for S in 4 5; do
  FMS_STORE_NP=$S timeout -k 10 400 ./tools/flat_map_sweep f64 32768 8192x65536 8192 > $O/np_store${S}_f64.log 2>&1 || exit 1
  FMS_STORE_NP=$S timeout -k 10 300 ./tools/flat_map_sweep f32 32768 8192 > $O/np_store${S}_f32.log 2>&1 || exit 1
done
echo done
