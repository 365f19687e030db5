O=gpurun_out/r02_s25; mkdir -p $O
timeout -k 10 300 ./tools/mall_split f64 8192 4096x16384 2880x23040 6144 > $O/mall_split_f64.log 2>&1 || exit 1
timeout -k 10 300 ./tools/mall_split f32 8192 12288 > $O/mall_split_f32.log 2>&1 || exit 1
cat $O/mall_split_*.log
