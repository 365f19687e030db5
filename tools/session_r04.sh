# round-4 GPU session steps (one file, rewritten per session; earlier
# sessions' steps are in tools/gpu_session.sh)
set -u
O=gpurun_out/${S:-r04_s3}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fail() { echo "== stopping: $1 exited $2"; exit $2; }
run() { # name secs cmd...  (rc 0/1 continue; anything else ends the session)
  local n=$1 t=$2; shift 2
  echo "== $n: $*"; local t0=$(date +%s)
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc ($(( $(date +%s) - t0 ))s)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then fail $n $rc; fi
}
for step in ${STEPS:-cdp stagger deferweak l2 tests}; do case $step in
cdp)
  # not run under run(): a hang here is the finding, and it ends only this probe
  CDP_THREAD=1 CDP_ABORT=0 timeout -k 5 30 ./tools/comm_deadline_probe > $O/cdp_thread_noabort.log 2>&1; echo "cdp_thread_noabort rc=$?"
  CDP_THREAD=1 CDP_ABORT=1 timeout -k 5 30 ./tools/comm_deadline_probe > $O/cdp_thread_abort.log 2>&1; echo "cdp_thread_abort rc=$?" ;;
stagger) run stagger 400 ./tools/stagger_probe 32768x32768 8192x65536 ;;
deferweak)
  for W in "8192 0" "11648 2" "16384 4" "23040 8"; do
    set -- $W; N=$1; P=$2; D=$O/defer_h${N}_p${P}; mkdir -p $D
    run defer_h${N}_p${P} 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/defer_profile.py --kind hilbert --n $N --rank-block $P --dtype f64 --cycles 10 --events $D/events.json
    python3 tools/defer_profile.py --kind hilbert --n $N --rank-block $P --dtype f64 --trace $D/prof/run_kernel_trace.csv --events $D/events.json --json $O/r04_defer_cycle_hilbert${N}_p${P}_f64.json --launches $O/r04_defer_cycle_hilbert${N}_p${P}_f64_launches.csv > $D/summary.txt 2>&1
    cat $D/summary.txt
  done ;;
l2)
  for W in "32768 0" "65536 8"; do
    set -- $W; N=$1; P=$2; D=$O/l2_r${N}_p${P}; mkdir -p $D
    run l2_tcc_defer_${N} 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d $D/tcc_defer -o run -- python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype f64 --cycles 2
    run l2_tcp_defer_${N} 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_ACCESSES_sum --output-format csv -d $D/tcp_defer -o run -- python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype f64 --cycles 2
    run l2_tcc_every_${N} 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d $D/tcc_every -o run -- python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype f64 --every-ab 0 --steps 8 --passes 1
    run l2_tcp_every_${N} 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_ACCESSES_sum --output-format csv -d $D/tcp_every -o run -- python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype f64 --every-ab 0 --steps 8 --passes 1
    python3 tools/sq_counters.py $D/tcc_defer/run_counter_collection.csv $D/tcp_defer/run_counter_collection.csv $D/tcc_every/run_counter_collection.csv $D/tcp_every/run_counter_collection.csv --json=$O/r04_l2_random${N}_p${P}_f64.json
  done ;;
storeab)
  # the cached fp64 storing round (5 pending) on the weak-scaled rank blocks:
  # rows x piece tile (probe builds, tools/defer_shape_probe.sh) x workgroup cap
  for W in "16384 4" "11648 2" "23040 8" "8192 0"; do
    set -- $W; N=$1; P=$2
    for V in default s5r4 s5t0 s5t16; do
      L=eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; [ $V = default ] && L=eigen_value_amd/lib/libsimilarity_transform.so
      EIGEN_VALUE_LIB=$L run storeab_h${N}_p${P}_$V 240 python3 tools/defer_profile.py --kind hilbert --n $N --rank-block $P --dtype f64 --cycles 40 --passes 5 --caps-ab "0,4,4,3,3,0,3;0,4,4,3,3,0,2;0,4,4,3,3,0,4;0,4,4,3,3,0,0" --ab-json $O/r04_storeab_h${N}_p${P}_$V.json
      grep "median" $O/storeab_h${N}_p${P}_$V.log | sed "s/^/$V /"
    done
  done ;;
capsdrop)
  # the workgroup caps of the read-only deferred rounds against none (the
  # storing round keeps its own): entries inside the box-to-box spread go
  run capsdrop_f64_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f64 --cycles 40 --passes 7 --caps-ab "0,4,4,3,3,0,0;0,0,0,0,0,0,0" --ab-json $O/r04_capsdrop_hilbert8192_f64.json
  run capsdrop_f64_8192_p8 300 python3 tools/defer_profile.py --kind hilbert --n 23040 --rank-block 8 --dtype f64 --cycles 40 --passes 7 --caps-ab "0,4,4,3,3,0,0;0,0,0,0,0,0,0" --ab-json $O/r04_capsdrop_hilbert23040_p8_f64.json
  run capsdrop_f64_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f64 --cycles 6 --passes 7 --caps-ab "0,5,4,4,4,0,3;0,0,0,0,0,0,3" --ab-json $O/r04_capsdrop_random32768_f64.json
  run capsdrop_f64_65536_p8 300 python3 tools/defer_profile.py --kind random --n 65536 --rank-block 8 --dtype f64 --cycles 6 --passes 7 --caps-ab "0,5,4,4,4,0,3;0,0,0,0,0,0,3" --ab-json $O/r04_capsdrop_random65536_p8_f64.json
  run capsdrop_f32_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f32 --cycles 8 --passes 7 --caps-ab "0,6,5,4,5,0,3;0,0,0,0,0,0,3" --ab-json $O/r04_capsdrop_random32768_f32.json
  grep -h median $O/capsdrop_*.log ;;
samegpu) run rccl_same_gpu 150 python3 tools/rccl_same_gpu_probe.py --ranks 2 --timeout 30 ; cat $O/rccl_same_gpu.log ;;
ntstore)
  # the non-temporal storing round's piece tile (probe builds) x its cap
  for W in "32768 0 f64 0,5,4,4,4,0" "65536 8 f64 0,5,4,4,4,0" "32768 0 f32 0,6,5,4,5,0"; do
    set -- $W; N=$1; P=$2; DT=$3; C=$4
    for V in default tsnt4 tsnt8 tsnt16 tsnt32; do
      L=eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; [ $V = default ] && L=eigen_value_amd/lib/libsimilarity_transform.so
      EIGEN_VALUE_LIB=$L run ntstore_r${N}_p${P}_${DT}_$V 240 python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype $DT --cycles 6 --passes 5 --caps-ab "$C,3;$C,0;$C,4" --ab-json $O/r04_ntstore_r${N}_p${P}_${DT}_$V.json
      grep "median" $O/ntstore_r${N}_p${P}_${DT}_$V.log | sed "s/^/$V /"
    done
  done ;;
gather) run gather_overhead 300 python3 tools/gather_overhead.py; cat $O/gather_overhead.log | grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Librccl" ;;
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
    python3 tools/pmc_traffic.py --workload ${K}${N}_${DT} --n $N --elem $E --dtype $T --fetch $D/pmc_fetch/run_counter_collection.csv --write $D/pmc_write/run_counter_collection.csv --trace $D/prof/run_kernel_trace.csv --out $O/r04_${K}${N}_${DT}_pmc.json
    cp $D/prof/run_kernel_stats.csv $O/r04_${K}${N}_${DT}_kernel_stats.csv
  done ;;
torchrun8)
  # the driver's N > 1 launch line, rehearsed: torch.distributed.run with 8
  # ranks, all on cuda:0 over gloo (--one-gpu: plumbing, not scaling data)
  run torchrun8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 8 --steps 5 --warmup 1 --backend gloo --one-gpu
  grep -v "^\[W\|socket.cpp\|amdgpu.ids" $O/torchrun8.log | tail -c 3000 ;;
ragged)
  # the weak P = 2 block's ragged last 8 KB piece: rank-0 blocks of P = 2
  # partitions with whole (11264, 12288) and ragged (11648) 8 KB pieces per row
  for N in 11648 11264 12288 8192; do
    P=2; [ $N = 8192 ] && P=0
    run ragged_h${N}_p${P} 240 python3 tools/defer_profile.py --kind hilbert --n $N --rank-block $P --dtype f64 --every-ab "0;0" --steps 100 --passes 5 --ab-json $O/r04_ragged_h${N}_p${P}.json
    grep median $O/ragged_h${N}_p${P}.log
  done ;;
hostasan) LEAKS=0 run host_asan 120 bash tools/host_asan.sh run; tail -40 $O/host_asan.log | grep -v "^$" | tail -30 ;;
everyr2)
  # the every-round cached launch (the headline): 1 row (shipped) vs 2 rows
  # per workgroup (probe build), each under workgroup caps and piece tiles
  for V in default er2; do
    L=eigen_value_amd/lib/variants/$V/libsimilarity_transform.so; [ $V = default ] && L=eigen_value_amd/lib/libsimilarity_transform.so
    EIGEN_VALUE_LIB=$L run everyr2_$V 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f64 --every-ab "2;2:0:3;2:0:4;2:0:6;2:4:4;2:8:4;2:16:0" --steps 100 --passes 7 --ab-json $O/r04_everyr2_hilbert8192_f64_$V.json
    grep median $O/everyr2_$V.log | sed "s/^/$V /"
  done ;;
pitch)
  for PT in 4 8; do for RO in 0 1; do
    PP_PT=$PT PP_RO=$RO PP_PADS=0,32,64,128,512 run pitch_probe_t${PT}_ro${RO} 300 ./tools/pitch_probe 8192x65536 16384x32768 32768x32768 8192x8192
    cat $O/pitch_probe_t${PT}_ro${RO}.log
  done; done ;;
nttile)
  # the every-round non-temporal launch's piece tile (st_set_every_tile via
  # --every-ab "0:T"): shipped 4 against 8 / 16 / row-major, on the north
  # star, configs[4] and the configs[3] rank blocks
  for W in "32768 0 f64" "65536 8 f64" "65536 4 f64" "32768 0 f32"; do
    set -- $W; N=$1; P=$2; DT=$3
    run nttile_r${N}_p${P}_${DT} 300 python3 tools/defer_profile.py --kind random --n $N --rank-block $P --dtype $DT --every-ab "0;0:8;0:16;0:1;0:4" --steps 20 --passes 5 --ab-json $O/r04_nttile_r${N}_p${P}_${DT}.json
    grep median $O/nttile_r${N}_p${P}_${DT}.log
  done ;;
pitchflat)
  # k_flat's own every-round walk (tiles of 4 row groups, as shipped) with the
  # row pitch padded by 0 / 32 / 64 doubles at the same bytes
  for V in ${PITCH_VARIANTS:-flat_map_sweep flat_map_sweep_pad32 flat_map_sweep_pad64}; do
    FMS_EVERY=1 FMS_PT=4 run pitchflat_$V 300 ./tools/$V f64 32768 8192x65536 16384x32768 16384x65536
    grep -v "^$" $O/pitchflat_$V.log | sed "s/^/$V /"
  done ;;
fuzz) run fuzz_parity 900 python3 -u tools/fuzz_parity.py --cases 300 --json $O/r04_fuzz_parity.json; tail -3 $O/fuzz_parity.log ;;
commtests) run comm_tests 300 python -u -m pytest tests/test_gpu_fullsize.py -k "prompt or deadline" -v --timeout 200 --timeout-method thread; tail -6 $O/comm_tests.log ;;
tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread ;;
bench) run bench 600 python bench.py ;;
prof)
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu
  cp $O/prof/run_kernel_stats.csv $O/r04_bench_default_${S:-s}_kernel_stats.csv ;;
smoke) run smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
esac; done
echo "== session done"
