O=gpurun_out/r02_s42; mkdir -p $O
timeout -k 10 300 python3 tools/alloc_probe.py --reps 8 > $O/alloc_f64.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --reps 8 --keep 0 > $O/alloc_f64_nokeep.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --reps 8 --dtype f32 > $O/alloc_f32.log 2>&1 || exit 1
cat $O/*.log | grep -v amdgpu
