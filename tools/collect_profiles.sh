#!/bin/bash
# Copy one gpu_session.sh run's evidence (tests smoke bench prof profile
# profile_f32 defer defer_pmc) into profiles/ under the round's prefix.
#   bash tools/collect_profiles.sh gpurun_out/r02_s35 r02
set -e
S=$1; P=${2:-r02}; D=profiles
cp $S/pytest_gpu.log $D/${P}_pytest_gpu.log
grep -h '^{' $S/bench.log > $D/${P}_bench_default.log
cp $S/prof/run_kernel_stats.csv $D/${P}_bench_default_kernel_stats.csv
for W in hilbert8192:hilbert8192_f64 random32768:random32768_f64 random32768_f32:random32768_f32; do
  src=${W%%:*}; dst=${W##*:}
  cp $S/$src/prof/run_kernel_stats.csv $D/${P}_${dst}_kernel_stats.csv
  cp $S/$src/pmc.json $D/${P}_${dst}_pmc.json
done
for w in hilbert8192_f64 random32768_f64 random32768_f32; do
  cp $S/defer_$w/prof/run_kernel_stats.csv $D/${P}_defer_profile_${w}_kernel_stats.csv
  cp $S/defer_$w/cycle.json $D/${P}_defer_cycle_${w}.json
done
for w in random32768_f64 random32768_f32; do
  cp $S/defer_pmc_$w/pmc.json $D/${P}_defer_pmc_${w}.json
done
echo "collected $S into $D/${P}_*"
