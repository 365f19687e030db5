O=gpurun_out/r02_s7; mkdir -p $O
export FMS_QUICK=1
for rep in 1 2; do
for v in base flat_map_sweep masked dppinit; do
  b=./tools/flat_map_sweep_$v; [ $v = flat_map_sweep ] && b=./tools/flat_map_sweep
  timeout -k 10 120 $b f64 32768 8192 > $O/${v}_f64_$rep.log 2>&1 || exit 1
  timeout -k 10 120 $b f32 32768 > $O/${v}_f32_$rep.log 2>&1 || exit 1
done
done
echo done
