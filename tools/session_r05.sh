# round-5 GPU session steps (S=r05_sN STEPS="…" bash tools/session_r05.sh)
set -u
O=gpurun_out/${S:-r05_s1}; mkdir -p $O
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
comm) run comm_tests 400 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "comm_init or grouped_init or all_devices or config3"; tail -40 $O/comm_tests.log ;;
tests) run pytest_gpu 900 python3 -u -m pytest -x -q -rs --timeout 300 --timeout-method thread -m gpu tests/; tail -15 $O/pytest_gpu.log ;;
smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"; tail -3 $O/smoke.log ;;
bench) run bench 900 python3 bench.py; tail -c 1500 $O/bench.log ;;
benchquick) run benchquick 600 python3 bench.py --no-cpu --no-north-star --no-headline; tail -c 2500 $O/benchquick.log ;;
prof)
  D=$O/prof; mkdir -p $D
  run prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --no-cpu --no-north-star --no-headline
  head -12 $D/run_kernel_stats.csv ;;
rcclchar)
  # RCCL deadline behaviour on torch's bundled RCCL (a crash at exit is the finding)
  timeout -k 5 40 python3 tools/rccl_deadline_torch.py --abort 0 > $O/rcclchar_noabort.log 2>&1; echo "rcclchar_noabort rc=$?"; grep "^\[" $O/rcclchar_noabort.log
  timeout -k 5 40 python3 tools/rccl_deadline_torch.py --abort 1 > $O/rcclchar_abort.log 2>&1; echo "rcclchar_abort rc=$?"; grep "^\[" $O/rcclchar_abort.log ;;
deferleg)
  # the bench's own deferred legs under a kernel trace: the
  # rocprof source bench.py quotes beside its HIP-event figure
  EV='"every_ms":{"hilbert8192_f64":0.153,"random32768_f64":2.64,"random32768_f32":1.31}'
  for W in "0 hilbert8192_f64" "1 random32768_f64" "2 random32768_f32"; do
    set -- $W; I=$1; WL=$2; D=$O/deferleg_$WL; mkdir -p $D
    run deferleg_$WL 600 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --leg deferred --leg-args "{\"device\":0,\"steps\":200,\"warmup\":10,\"kind\":\"hilbert\",\"n\":8192,\"dtype\":\"f64\",\"representative\":true,\"which\":$I,$EV}"
    python3 tools/defer_profile.py --kind hilbert --trace $D/run_kernel_trace.csv --bench-leg $O/deferleg_$WL.log --json $O/r05_defer_bench_$WL.json
  done
  for W in "weak_rank_blocks hilbert" "rank_blocks random"; do
    set -- $W; L=$1; K=$2; D=$O/deferleg_$L; mkdir -p $D
    run deferleg_$L 900 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --leg $L --leg-args "{\"device\":0,\"steps\":200,\"warmup\":10,\"kind\":\"hilbert\",\"n\":8192,\"dtype\":\"f64\",\"representative\":true}"
    python3 tools/defer_profile.py --kind $K --trace $D/run_kernel_trace.csv --bench-leg $O/deferleg_$L.log --json $O/r05_defer_bench_$L.json
  done ;;
*) echo "unknown step $step"; exit 2 ;;
esac; done
