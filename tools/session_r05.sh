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
bitwise)
  # the flat launches' bitwise tests first: a failure ends the session
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tail or 2d_grid or flat_round_vs_round or deferred_writes_bitwise or mfree_flat or split_flat" > $O/bitwise.log 2>&1; rc=$?
  tail -3 $O/bitwise.log; [ $rc -eq 0 ] || fail bitwise $rc ;;
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
    A="{\"device\":0,\"steps\":200,\"warmup\":10,\"kind\":\"hilbert\",\"n\":8192,\"dtype\":\"f64\",\"representative\":true,\"which\":$I,$EV}"
    run deferleg_$WL 600 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --leg deferred --leg-args "$A"
    run deferplain_$WL 600 python3 bench.py --leg deferred --leg-args "$A"
    python3 tools/defer_profile.py --kind hilbert --trace $D/run_kernel_trace.csv --bench-leg $O/deferleg_$WL.log --bench-leg-plain $O/deferplain_$WL.log --json $O/r05_defer_bench_$WL.json
  done
  for W in "weak_rank_blocks hilbert" "rank_blocks random"; do
    set -- $W; L=$1; K=$2; D=$O/deferleg_$L; mkdir -p $D
    A="{\"device\":0,\"steps\":200,\"warmup\":10,\"kind\":\"hilbert\",\"n\":8192,\"dtype\":\"f64\",\"representative\":true}"
    run deferleg_$L 900 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --leg $L --leg-args "$A"
    run deferplain_$L 900 python3 bench.py --leg $L --leg-args "$A"
    python3 tools/defer_profile.py --kind $K --trace $D/run_kernel_trace.csv --bench-leg $O/deferleg_$L.log --bench-leg-plain $O/deferplain_$L.log --json $O/r05_defer_bench_$L.json
  done ;;
tailab)
  # ragged rows' tail workgroups: off / table / 2 / 4 / 8 row
  # groups per workgroup of the last piece, every-round and deferred
  for W in "11648 2" "23040 8" "4352 0"; do
    set -- $W; N=$1; P=$2
    run tailab_h${N}_p${P} 400 python3 tools/defer_profile.py --kind hilbert --n $N --rank-block $P --dtype f64 --tail-ab "1;0;2;4;8" --steps 100 --cycles 20 --passes 7 --ab-json $O/r05_tail_ab_h${N}_p${P}.json
    grep median $O/tailab_h${N}_p${P}.log
  done ;;
loopab)
  # the tail loop around k_flat's body against the round-4 build (ab_base)
  # on whole-piece blocks (the headline shapes), alternating builds
  for rep in 1 2; do for V in new base; do
    L=eigen_value_amd/lib/libsimilarity_transform.so; [ $V = base ] && L=eigen_value_amd/lib/ab_base/libsimilarity_transform.so
    for W in "8192 0" "16384 4" "32768 0"; do
      set -- $W; N=$1; P=$2; K=hilbert; [ $N = 32768 ] && K=random
      EIGEN_VALUE_LIB=$L run loopab_${V}${rep}_${N}_p${P} 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype f64 --tail-ab "1" --steps 100 --cycles 6 --passes 5 --ab-json $O/r05_loop_ab_${V}${rep}_${N}_p${P}.json
      grep median $O/loopab_${V}${rep}_${N}_p${P}.log | sed "s/^/$V$rep /"
    done
  done; done ;;
storenp)
  # VERDICT r04 #7, one bounded attempt: what the storing launch pays for
  # its pending scalings - single k_flat launches (tools/bin/flat_map_sweep,
  # built on the CPU) with the store at NP = 5 (shipped) against NP = 2,
  # same rows / tile, 32768^2 and the P = 8 block of configs[3]
  for SNP in 5 2; do
    FMS_R8=1 FMS_MAX_NP=5 FMS_PT=16 FMS_STORE_NP=$SNP run storenp_$SNP 300 ./tools/bin/flat_map_sweep f64 32768 8192x65536
    cat $O/storenp_$SNP.log
  done ;;
torchrun8)
  # the driver's N > 1 launch line, rehearsed: torch.distributed.run with 8
  # ranks, all on cuda:0 over gloo (--one-gpu: plumbing, not scaling data)
  run torchrun8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 8 --steps 5 --warmup 1 --backend gloo --one-gpu
  grep -v "^\[W\|socket.cpp\|amdgpu.ids" $O/torchrun8.log | tail -c 3000 ;;
fuzzbig) run fuzz_parity_big 1100 python3 -u tools/fuzz_parity.py --cases 1500 --seed 5052026 --json $O/r05_fuzz_parity_1500.json; tail -2 $O/fuzz_parity_big.log ;;
fuzz) run fuzz_parity 900 python3 -u tools/fuzz_parity.py --cases 300 --seed 20261105 --json $O/r05_fuzz_parity.json; tail -3 $O/fuzz_parity.log ;;
pmc)
  # HBM bytes of the headline launches (separate FETCH_SIZE / WRITE_SIZE
  # passes, tools/pmc_traffic.py applies the gfx950 x2 FETCH correction)
  for W in "hilbert 8192 f64 8" "random 32768 f64 8" "random 32768 f32 4"; do
    set -- $W; K=$1; N=$2; DT=$3; E=$4; D=$O/${K}${N}_${DT}; mkdir -p $D
    X="--kind $K --n $N --dtype $DT --no-cpu --no-north-star --no-headline"
    run prof_${K}${N}_${DT} 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py $X
    run pmcf_${K}${N}_${DT} 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 bench.py $X --steps 20 --warmup 2
    run pmcw_${K}${N}_${DT} 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 bench.py $X --steps 20 --warmup 2
    T=double; [ $DT = f32 ] && T=float
    python3 tools/pmc_traffic.py --workload ${K}${N}_${DT} --n $N --elem $E --dtype $T --fetch $D/pmc_fetch/run_counter_collection.csv --write $D/pmc_write/run_counter_collection.csv --trace $D/prof/run_kernel_trace.csv --out $O/r05_${K}${N}_${DT}_pmc.json
    cp $D/prof/run_kernel_stats.csv $O/r05_${K}${N}_${DT}_kernel_stats.csv
  done ;;
*) echo "unknown step $step"; exit 2 ;;
esac; done
