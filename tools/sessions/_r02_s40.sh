O=gpurun_out/r02_s40; mkdir -p $O
for rep in 1 2; do
FMS_EVERY=1 FMS_U1=1 FMS_PT=0,4,8 timeout -k 10 300 ./tools/flat_map_sweep f64 5824x11648 8192 2880x23040 6144x11648 > $O/u1_$rep.log 2>&1 || exit 1
done
cat $O/u1_*.log
