O=gpurun_out/r02_s47; mkdir -p $O
timeout -k 10 300 python3 tools/alloc_probe.py --n 65536 --reps 2 --keep 0 > $O/fresh.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --n 65536 --reps 2 --keep 0 --pre 8192,11648,16384,23040,32768,32768,32768 > $O/after_pre.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --n 32768 --reps 2 --keep 0 > $O/fresh32.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --n 32768 --reps 2 --keep 0 --pre 8192,65536 > $O/after_pre32.log 2>&1 || exit 1
for f in fresh after_pre fresh32 after_pre32; do echo "== $f"; grep '^{' $O/$f.log; done
