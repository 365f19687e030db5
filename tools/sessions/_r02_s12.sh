O=gpurun_out/r02_s12; mkdir -p $O
for rep in 1 2; do
for v in base r0c4 pt0c16; do
  if [ $v = base ]; then unset EIGEN_VALUE_LIB; else export EIGEN_VALUE_LIB=$PWD/eigen_value_amd/lib/variants/$v/libsimilarity_transform.so; fi
  for W in "hilbert 8192 f64" "random 12288 f64" "random 8192 f32" "random 16384 f32"; do
    set -- $W
    echo "$v $rep $W $(timeout -k 10 120 python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 40)" >> $O/probe.log || exit 1
  done
done
done
echo done
