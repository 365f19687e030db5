O=gpurun_out/r02_s28; mkdir -p $O
for rep in 1 2; do for V in base every_old; do
  if [ $V = base ]; then unset EIGEN_VALUE_LIB; else export EIGEN_VALUE_LIB=$PWD/eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; fi
  echo "== $V rep $rep" >> $O/split_cost.log
  timeout -k 10 300 python3 tools/split_cost.py >> $O/split_cost.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/split_cost.log
