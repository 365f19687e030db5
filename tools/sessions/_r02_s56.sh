O=gpurun_out/r02_s56; mkdir -p $O
for rep in 1 2 3; do for V in base np0r1 np0r1t8; do
  if [ $V = base ]; then unset EIGEN_VALUE_LIB; else export EIGEN_VALUE_LIB=$PWD/eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; fi
  for W in "hilbert 8192 f64 40" "random 12288 f64 20" "random 10240 f64 30"; do
    set -- $W
    echo -n "$V rep$rep " >> $O/ab.log
    timeout -k 10 120 python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles $4 2>/dev/null | grep workload >> $O/ab.log || exit 1
  done
done; done
