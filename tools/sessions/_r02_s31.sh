O=gpurun_out/r02_s31; mkdir -p $O
for SK in 0 1 3 7 33 65; do
  FMS_EVERY=1 FMS_SK=$SK FMS_PT=4,8 timeout -k 10 300 ./tools/flat_map_sweep f64 8192x65536 32768 16384x65536 >> $O/skew_f64_nt.log 2>&1 || exit 1
done
grep -v "R=4" $O/skew_f64_nt.log
