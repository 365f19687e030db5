O=gpurun_out/r02_s37; mkdir -p $O; export TMPDIR=/tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"
for W in "random 32768 f64" "hilbert 8192 f64"; do set -- $W
  timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/$1$2_p1 -o run -- python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 2 > $O/$1$2_p1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/$1$2_p2 -o run -- python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 2 > $O/$1$2_p2.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/$1$2_e1 -o run -- python3 bench.py --kind $1 --n $2 --steps 5 --warmup 1 --no-cpu --no-north-star --no-headline > $O/$1$2_e1.log 2>&1 || exit 1
  python3 tools/sq_counters.py $O/$1$2_p1/run_counter_collection.csv $O/$1$2_p2/run_counter_collection.csv --json=$O/sq_$1$2.json
  python3 tools/sq_counters.py $O/$1$2_e1/run_counter_collection.csv
done
