# round-6 GPU session steps (S=r06_sN STEPS="…" bash tools/session_r06.sh)
set -u
O=gpurun_out/${S:-r06_s1}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fail() { echo "== stopping: $1 exited $2"; exit $2; }
run() { # name secs cmd...  (rc 0/1 continue; anything else ends the session)
  local n=$1 t=$2; shift 2
  echo "== $n: $*"; local t0=$(date +%s)
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc ($(( $(date +%s) - t0 ))s)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then fail $n $rc; fi
}
for step in ${STEPS:-tests smoke bench}; do case $step in
new)
  # this round's new paths first (flat K0, traced solves): a failure ends the session
  timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rowsum or trace or fp32_random_at_reference_eps or fuzz or flat_round_vs_round or deferred_writes_bitwise or sharded_single_gpu or native_multi_gpu_flat" > $O/new.log 2>&1; rc=$?
  tail -25 $O/new.log; [ $rc -eq 0 ] || fail new $rc ;;
new2)
  # session 2's changes first: the fast round path, the tuning build, the
  # one-GPU rehearsals of the multi-device workers, the communicator probes
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_tuning.py tests/test_zz_multi_device.py tests/test_gpu_fullsize.py -k "fast_path or tuning or rehearsal or comm_init or grouped_init or trace or rowsum" > $O/new2.log 2>&1; rc=$?
  tail -30 $O/new2.log; [ $rc -eq 0 ] || fail new2 $rc ;;
collect) python3 -m pytest --collect-only -q -m gpu tests/ > $O/collect.log 2>&1; tail -25 $O/collect.log ;;
tests) run pytest_gpu 900 python3 -u -m pytest -x -q -rs --timeout 300 --timeout-method thread -m gpu tests/; tail -15 $O/pytest_gpu.log ;;
smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"; tail -3 $O/smoke.log ;;
fuzz) run fuzz 900 python3 -u tools/fuzz_parity.py --cases ${FUZZ_CASES:-300} --seed ${FUZZ_SEED:-20261201} --json $O/r06_fuzz_parity.json; tail -3 $O/fuzz.log; grep -c STRADDLE $O/fuzz.log || true ;;
fuzzwrap) run fuzzwrap 900 python3 -u tools/fuzz_parity.py --profile wrapper --cases ${FUZZ_CASES:-200} --seed ${FUZZ_SEED:-20270202} --json $O/r06_fuzz_wrapper.json; tail -3 $O/fuzzwrap.log; grep -c STRADDLE $O/fuzzwrap.log || true ;;
bench) run bench 900 python3 bench.py --steps 20 --warmup 5; tail -c 1500 $O/bench.log ;;
benchquick) run benchquick 600 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-north-star --no-headline; tail -c 2500 $O/benchquick.log ;;
profdefault)
  # the default bench line under a kernel trace (the driver's command)
  D=$O/profdefault; mkdir -p $D
  run prof_default 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 20 --warmup 5
  head -8 $D/run_kernel_stats.csv | cut -c1-200 ;;
prof)
  D=$O/prof; mkdir -p $D
  run prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-north-star --no-headline
  head -14 $D/run_kernel_stats.csv ;;
k0)
  # K0 (the initial row-sum pass) alone at configs[1] and the north star,
  # both forms, under a kernel trace
  D=$O/k0; mkdir -p $D
  run k0 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 tools/k0_probe.py
  cat $O/k0.log | tail -12; head -12 $D/run_kernel_stats.csv ;;
sync)
  # the host clock's fixed start / stop latency
  run sync_default 300 python3 tools/sync_probe.py --json $O/r06_sync_probe_default.json; tail -6 $O/sync_default.log
  HSA_ENABLE_INTERRUPT=0 run sync_polling 300 python3 tools/sync_probe.py --json $O/r06_sync_probe_polling.json; tail -6 $O/sync_polling.log ;;
tables)
  # the reference's own benchmark tables (README.md whole-solve Hilbert,
  # benchmarks/similarity_transform.md per kernel) through the C-ABI, and
  # the flat walk's own memory ceiling (no arithmetic)
  run tables_hilbert 300 bash -c './tools/bench_hilbert f32 && ./tools/bench_hilbert f64' && \
  run tables_kernels 300 ./tools/bench_kernels && \
  run tables_mall 300 ./tools/mall_stream 8192x8192 32768x32768; tail -40 $O/tables_*.log ;;
everyab)
  # the every-round flat launch of configs[1] under workgroup caps / tiles
  # (tuning build; interleaved passes of 20 rounds)
  EIGEN_VALUE_LIB=eigen_value_amd/lib/libsimilarity_transform_tuning.so run everyab 400 python3 -u tools/defer_profile.py --n 8192 --kind hilbert --every-ab "${EVERY_AB:-0;0:0:3;0:0:4;0:0:6;0:4;0:16}" --steps 20 --passes 9 --ab-json $O/r06_every_ab.json; tail -8 $O/everyab.log ;;
k0order)
  # K0 walked front to back vs from the end on cacheable blocks (tuning build)
  EIGEN_VALUE_LIB=eigen_value_amd/lib/libsimilarity_transform_tuning.so run k0order 400 python3 -u tools/k0_order_probe.py --json $O/r06_k0_order.json; tail -8 $O/k0order.log ;;
prefix)
  # the headline pass fresh and after each step bench.py runs before it
  run prefix 300 python3 -u tools/prefix_probe.py --json $O/r06_prefix_probe.json; cat $O/prefix.log | tail -12 ;;
pmc)
  # kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench's own legs
  # for the headline workload and the north star (fp64, fp32), one process
  # each (--strong: no weak-scaled rank blocks in the same trace)
  for W in "hilbert 8192 f64" "random 32768 f64" "random 32768 f32"; do
    set -- $W; K=$1; N=$2; T=$3; WL=$K${N}_$T; D=$O/pmc_$WL; mkdir -p $D
    A="bench.py --n $N --kind $K --dtype $T --strong --no-cpu --no-north-star --no-headline --no-configs3 --steps 20 --warmup 5"
    run prof_$WL 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 $A
    run fetch_$WL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 $A
    run write_$WL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 $A
    EL=8; [ $T = f32 ] && EL=4; DT=double; [ $T = f32 ] && DT=float
    python3 tools/pmc_traffic.py --workload $WL --n $N --elem $EL --dtype $DT --fetch $D/fetch/run_counter_collection.csv --write $D/write/run_counter_collection.csv --trace $D/prof/run_kernel_trace.csv --out $O/r06_${WL}_pmc.json | tee -a $O/pmc_summary.log
  done ;;
*) echo "unknown step $step"; exit 2 ;;
esac; done
