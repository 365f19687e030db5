O=gpurun_out/r02_s23; mkdir -p $O
export TMPDIR=/tmp
for V in base store_nt; do
  if [ $V = base ]; then unset EIGEN_VALUE_LIB; else export EIGEN_VALUE_LIB=$PWD/eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; fi
  for W in "hilbert 8192 f64" "random 12288 f64" "random 16384 f32" "random 8192 f32"; do
    set -- $W
    timeout -k 10 120 python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 40 >> $O/$V.log 2>&1 || exit 1
  done
done
cat $O/base.log $O/store_nt.log
