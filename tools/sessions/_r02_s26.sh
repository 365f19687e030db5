O=gpurun_out/r02_s26; mkdir -p $O
for rep in 1 2; do
FMS_EVERY=1 FMS_PT=0,4,6,8,12,16 timeout -k 10 300 ./tools/flat_map_sweep f64 8192 5824x11648 4096x16384 2880x23040 12288 6144 > $O/every_cached_f64_$rep.log 2>&1 || exit 1
FMS_EVERY=1 FMS_PT=0,4,6,8,12,16 timeout -k 10 300 ./tools/flat_map_sweep f32 8192 12288 16384 4096x32768 > $O/every_cached_f32_$rep.log 2>&1 || exit 1
done
grep -h -v "R=4" $O/every_cached_*.log
