O=gpurun_out/r02_s44; mkdir -p $O
timeout -k 10 300 ./tools/mfree_probe f32 32768 16384 > $O/mfree_f32.log 2>&1 || exit 1
timeout -k 10 300 ./tools/mfree_probe f64 32768 > $O/mfree_f64.log 2>&1 || exit 1
cat $O/mfree_*.log
