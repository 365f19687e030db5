O=gpurun_out/r02_s29; mkdir -p $O; export TMPDIR=/tmp
for V in base every_old; do
  if [ $V = base ]; then unset EIGEN_VALUE_LIB; else export EIGEN_VALUE_LIB=$PWD/eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; fi
  for W in "hilbert 8192" "random 32768"; do set -- $W
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${V}_$1$2 -o run -- python3 bench.py --kind $1 --n $2 --no-cpu --no-north-star --no-headline > $O/${V}_$1$2.log 2>&1 || exit 1
  done
done
for f in $O/*/run_kernel_stats.csv; do python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'k_parts' in r['Name'] or ('k_flat' in r['Name'] and ', -1,' in r['Name']): print('$f'.split('/')[2], r['Name'][:50], r['Calls'], r['AverageNs'])
"; done
grep -ho '"ms_per_step": [0-9.]*' $O/*.log
