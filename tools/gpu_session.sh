#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel trace.
# Usage (through gpurun, from the repo root): bash tools/gpu_session.sh TAG [steps...]
#   steps: tests smoke bench prof pmc tune (default: tests smoke bench prof)
# Every GPU step has its own time limit; a crash/abort/timeout ends the
# session (test assertion failures, exit 1, do not).
set -u
TAG=${1:-run}; shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
RTAG=${RTAG:-r03}   # round prefix of the files meant for profiles/
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 15 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: $name exited $rc" | tee -a "$OUT/session.log"
    exit $rc
  fi
  return $rc
}

rocm-smi --showproductname > "$OUT/device.txt" 2>&1 || true
nproc > "$OUT/host.txt"; lscpu | grep -E 'Model name|^CPU\(s\)' >> "$OUT/host.txt" || true

for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
    bench) step bench 600 python bench.py ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu ;;
    pmc)
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu ;;
    tune)  step tune 600 ./tools/tune_fused ;;
    sweep) step sweep_dir 600 ./tools/sweep_dir ${SWEEP_ARGS:-2048 4096 6144 8192 12288 16384 24576 32768} ;;
    hilbert)
      make -s -C tools bench_hilbert
      step bench_hilbert_f32 300 ./tools/bench_hilbert f32
      step bench_hilbert_f64 300 ./tools/bench_hilbert f64 ;;
    kernels)
      make -s -C tools bench_kernels
      step bench_kernels 300 ./tools/bench_kernels ;;
    h2d)
      make -s -C tools h2d_probe
      step h2d_probe 300 ./tools/h2d_probe 64 256 512 2048 ;;
    multi) # the N > 1 bench path rehearsed on one GPU (gloo exchange)
      step bench_p2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --one-gpu
      step bench_p4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 20 --warmup 3 --backend gloo --one-gpu ;;
    overlap) # the overlapped exchange: N = 1 (split launches, empty gather) and the rehearsal
      step bench_overlap_p1 600 python bench.py --overlap --no-cpu --no-north-star --no-headline
      step bench_overlap_p2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --one-gpu --overlap --no-overlap-leg ;;
    spawn) # the N > 1 line without a launcher: two self-spawned ranks on one GPU (gloo)
      step bench_spawn_p2 900 python bench.py --gpus 2 --one-gpu --backend gloo --steps 20 --warmup 3 --no-overlap-leg ;;
    spawn8) # the driver's 8-GPU partition rehearsed: 8 self-spawned ranks on one GPU (gloo)
      step bench_spawn_p8 900 python bench.py --gpus 8 --one-gpu --backend gloo --steps 5 --warmup 1 ;;
    longrow) # configs[3]'s long-row rank blocks: column-block piece orders + the counter list
      rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
      FMS_EVERY=1 FMS_PT=4 FMS_PC=0,16,32,64 step longrow_pc 600 ./tools/flat_map_sweep f64 32768 8192x65536 16384x65536
      # translation and address-unit counters of the every-round launch, square vs long rows
      for SZ in 32768 8192x65536; do
        D="$OUT/longrow_pmc_$SZ"; mkdir -p "$D"
        FMS_EVERY=1 FMS_PT=4 step "lr_tcp_$SZ" 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$D/tcp" -o run -- ./tools/flat_map_sweep f64 $SZ || true
        FMS_EVERY=1 FMS_PT=4 step "lr_ta_$SZ" 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d "$D/sq" -o run -- ./tools/flat_map_sweep f64 $SZ || true
        for P in tcp sq; do
          [ -f "$D/$P/run_counter_collection.csv" ] && python3 tools/sq_counters.py "$D/$P/run_counter_collection.csv" --json="$OUT/${RTAG}_longrow_${P}_$SZ.json" | tee -a "$OUT/session.log"
        done
      done ;;
    capsab) # workgroups-per-CU caps of the deferred launches, A/B in the solve loop
      NT_SPECS="0,0,0,0,0,0,0;0,0,0,0,0,0,3;0,6,5,4,5,0,3;0,5,4,4,4,0,3;0,6,5,4,5,0,4"
      C_SPECS="0,0,0,0,0,0,0;0,4,0,0,3,0,0;0,4,4,4,3,0,0;0,5,5,4,4,0,0;0,4,4,4,3,0,3"
      step capsab_f64_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f64 --cycles 6 --passes 5 --caps-ab "$NT_SPECS" --ab-json "$OUT/capsab_random32768_f64.json"
      step capsab_f32_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f32 --cycles 8 --passes 5 --caps-ab "$NT_SPECS" --ab-json "$OUT/capsab_random32768_f32.json"
      step capsab_f64_65536_p8 300 python3 tools/defer_profile.py --kind random --n 65536 --rank-block 8 --dtype f64 --cycles 6 --passes 5 --caps-ab "$NT_SPECS" --ab-json "$OUT/capsab_random65536_p8_f64.json"
      step capsab_f64_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f64 --cycles 40 --passes 5 --caps-ab "$C_SPECS" --ab-json "$OUT/capsab_hilbert8192_f64.json"
      step capsab_f32_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f32 --cycles 60 --passes 5 --caps-ab "$C_SPECS" --ab-json "$OUT/capsab_hilbert8192_f32.json" ;;
    capsab2) # the shipped caps table against no caps and its neighbours
      NT_SPECS="0,5,4,4,4,0,3;0,0,0,0,0,0,0;0,5,4,4,5,0,3;0,6,4,4,4,0,3;0,5,4,4,4,0,4"
      C_SPECS="0,4,4,4,3,0,3;0,0,0,0,0,0,0;0,4,4,4,3,0,4;0,4,4,3,3,0,3;0,5,4,4,3,0,3"
      F32_SPECS="0,6,5,4,5,0,3;0,0,0,0,0,0,0;0,5,4,4,4,0,3;0,6,5,4,5,0,4"
      step capsab2_f64_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f64 --cycles 6 --passes 5 --caps-ab "$NT_SPECS" --ab-json "$OUT/${RTAG}_capsab2_random32768_f64.json"
      step capsab2_f64_65536_p8 300 python3 tools/defer_profile.py --kind random --n 65536 --rank-block 8 --dtype f64 --cycles 6 --passes 5 --caps-ab "$NT_SPECS" --ab-json "$OUT/${RTAG}_capsab2_random65536_p8_f64.json"
      step capsab2_f32_32768 300 python3 tools/defer_profile.py --kind random --n 32768 --dtype f32 --cycles 8 --passes 5 --caps-ab "$F32_SPECS" --ab-json "$OUT/${RTAG}_capsab2_random32768_f32.json"
      step capsab2_f64_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f64 --cycles 40 --passes 5 --caps-ab "$C_SPECS" --ab-json "$OUT/${RTAG}_capsab2_hilbert8192_f64.json" ;;
    capsab3) # cached blocks: the NP = 0 (post-store) and storing slots
      C_SPECS="0,4,4,3,3,0,3;8,4,4,3,3,0,3;6,4,4,3,3,0,3;0,4,4,3,3,0,2;0,4,4,3,3,0,4;0,3,3,3,3,0,3"
      F32C_SPECS="0,0,0,0,0,0,0;0,0,0,0,0,0,3;0,0,0,0,0,0,4;0,0,0,0,4,0,0;8,0,0,0,0,0,0"
      step capsab3_f64_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f64 --cycles 40 --passes 7 --caps-ab "$C_SPECS" --ab-json "$OUT/${RTAG}_capsab3_hilbert8192_f64.json"
      step capsab3_f64_6144 300 python3 tools/defer_profile.py --kind random --n 6144 --dtype f64 --cycles 60 --passes 7 --caps-ab "$C_SPECS" --ab-json "$OUT/${RTAG}_capsab3_random6144_f64.json"
      step capsab3_f64_p8w 300 python3 tools/defer_profile.py --kind hilbert --n 23040 --rank-block 8 --dtype f64 --cycles 40 --passes 7 --caps-ab "$C_SPECS" --ab-json "$OUT/${RTAG}_capsab3_hilbert23040_p8_f64.json"
      step capsab3_f32_8192 300 python3 tools/defer_profile.py --kind hilbert --n 8192 --dtype f32 --cycles 60 --passes 7 --caps-ab "$F32C_SPECS" --ab-json "$OUT/${RTAG}_capsab3_hilbert8192_f32.json" ;;
    libab) # whole store cycles under probe builds of the library (tools/defer_shape_probe.sh
           # variants in eigen_value_amd/lib/variants/NAME), interleaved with the shipped one
      for rep in 1 2 3; do
        for V in base $LIBAB_VARIANTS; do
          if [ "$V" = base ]; then LIBV=""; else LIBV="eigen_value_amd/lib/variants/$V/libsimilarity_transform.so"; fi
          EIGEN_VALUE_LIB=$LIBV step "libab_${V}_$rep" 200 python3 tools/defer_profile.py --kind ${LIBAB_KIND:-hilbert} --n ${LIBAB_N:-8192} --dtype ${LIBAB_DT:-f64} --cycles ${LIBAB_CYCLES:-40} --passes 3 ${LIBAB_EXTRA:-} --events "$OUT/libab_${V}_$rep.json"
        done
      done
      python3 - "$OUT" <<'PY' | tee -a "$OUT/session.log"
import glob, json, os, sys, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "libab_*.json"))):
    v = os.path.basename(f)[6:].rsplit("_", 1)[0]
    r[v].append(json.load(open(f))["event_ms_per_round"])
for v, xs in r.items():
    xs = sorted(xs)
    print(f"libab {v:16s} ms/round {xs}  median {xs[len(xs) // 2]:.5f}")
PY
      ;;
    ntab) # non-temporal-load masks of the cached fp64 deferred rounds (st_set_defer_ntload),
          # interleaved passes over whole store cycles
      M_SPECS=${NTAB_SPECS:-"0;0x1;0x41;0x5f;0x3;0x43;0x1f"}
      for W in "hilbert 8192 0" "hilbert 8192 2" "hilbert 23040 8" "random 10240 0" "random 12288 0" "random 14336 0" "random 16384 2"; do
        set -- $W; K=$1; N=$2; P=$3
        step "ntab_${K}${N}_p$P" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype f64 --cycles 40 --passes 5 --ntload-ab "$M_SPECS" --ab-json "$OUT/${RTAG}_ntab_${K}${N}_p${P}_f64.json"
        grep ntload "$OUT/ntab_${K}${N}_p$P.log" | tee -a "$OUT/session.log"
      done ;;
    everyab) # cache policy of the every-round flat launch (st_set_every_cache: 1 / 2 / 3 turn
             # the loads' / stores' / both policies over, cached <-> non-temporal),
             # interleaved passes of the bench's timed step
      E_SPECS=${EVERYAB_SPECS:-"0;1;2;3"}
      for W in ${EVERYAB_CASES:-hilbert,8192,0,f64 hilbert,23040,8,f64 hilbert,11648,2,f64 hilbert,16384,4,f64 random,6144,0,f64 random,10240,0,f64 random,12288,0,f64 hilbert,8192,0,f32 random,12288,0,f32 random,16384,0,f32 random,32768,0,f64 random,65536,8,f64 random,32768,0,f32}; do
        set -- ${W//,/ }; K=$1; N=$2; P=$3; D=$4
        step "everyab_${K}${N}_p${P}_$D" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype $D --steps 100 --passes 5 --every-ab "$E_SPECS" --ab-json "$OUT/${RTAG}_everyab_${K}${N}_p${P}_$D.json"
        grep every-cache "$OUT/everyab_${K}${N}_p${P}_$D.log" | tee -a "$OUT/session.log"
      done ;;
    dcab) # the deferred rounds' cache-policy flips on the other forms (st_set_defer_cache):
          # the non-temporal form (loads / stores turned cached) and cached fp32 blocks
      for W in ${DCAB_CASES:-random,32768,0,f64,6,0;0x1;0x3;0x1f;0x40;0x80 random,65536,8,f64,6,0;0x1;0x1f random,32768,0,f32,8,0;0x1;0x3;0x1f hilbert,8192,0,f32,60,0;0x1;0x41;0x5f random,12288,0,f32,30,0;0x1;0x41;0x5f random,16384,0,f32,20,0;0x1;0x41;0x5f}; do
        IFS=, read -r K N P D C M <<< "$W"
        step "dcab_${K}${N}_p${P}_$D" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype $D --cycles $C --passes 5 --defer-cache-ab "$M" --ab-json "$OUT/${RTAG}_dcab_${K}${N}_p${P}_$D.json"
        grep defer-cache "$OUT/dcab_${K}${N}_p${P}_$D.log" | tee -a "$OUT/session.log"
      done ;;
    mfab) # launch shapes of the matrix-free round (st_set_mfree_shape), fresh A_0 per run
      for W in ${MFAB_CASES:-hilbert,8192,0,f64 hilbert,23040,8,f64 random,6144,0,f64 random,10240,0,f64 hilbert,8192,0,f32 random,12288,0,f32 random,16384,0,f32 random,32768,0,f64}; do
        set -- ${W//,/ }; K=$1; N=$2; P=$3; D=$4
        step "mfab_${K}${N}_p${P}_$D" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype $D --steps 100 --passes 5 --mfree-ab "${MFAB_SPECS:-0;1;2;3}" --ab-json "$OUT/${RTAG}_mfab_${K}${N}_p${P}_$D.json"
        grep mfree-shape "$OUT/mfab_${K}${N}_p${P}_$D.log" | tee -a "$OUT/session.log"
      done ;;
    libeab) # the every-round step (the bench's) under probe builds of the library, interleaved
      for rep in 1 2 3; do
        for V in base $LIBAB_VARIANTS; do
          if [ "$V" = base ]; then LIBV=""; else LIBV="eigen_value_amd/lib/variants/$V/libsimilarity_transform.so"; fi
          for W in ${LIBEAB_CASES:-hilbert,8192,0,f64}; do
            set -- ${W//,/ }; K=$1; N=$2; P=$3; D=$4
            EIGEN_VALUE_LIB=$LIBV step "libeab_${V}_${K}${N}_p${P}_${D}_$rep" 200 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype $D --steps 200 --passes 3 --every-ab "${LIBEAB_SPECS:-2}"
            grep every-cache "$OUT/libeab_${V}_${K}${N}_p${P}_${D}_$rep.log" | sed "s/^/libeab $V /" | tee -a "$OUT/session.log"
          done
        done
      done ;;
    ntab3) # the weak-scaled P = 4 block (4096 x 16384 fp64), whose deferred cycle trails 8192^2
      step ntab3_hilbert16384_p4 300 python3 tools/defer_profile.py --kind hilbert --n 16384 --rank-block 4 --dtype f64 --cycles 40 --passes 7 --ntload-ab "0x41;0;0x1;0x5f;0x43;0x4f" --ab-json "$OUT/${RTAG}_ntab3_hilbert16384_p4_f64.json"
      grep ntload "$OUT/ntab3_hilbert16384_p4.log" | tee -a "$OUT/session.log" ;;
    ntab2) # bit 7 of the cached fp64 deferred mask: the storing round's stores non-temporal
      for W in "hilbert 8192 0 0x41;0xc1;0x1;0x81" "hilbert 23040 8 0x41;0xc1" "hilbert 11648 2 0x41;0xc1" "random 10240 0 0x5f;0xdf" "random 12288 0 0x5f;0xdf" "random 6144 0 0;0x80;0x41;0xc1"; do
        set -- $W; K=$1; N=$2; P=$3; M=$4
        step "ntab2_${K}${N}_p$P" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype f64 --cycles 40 --passes 7 --ntload-ab "$M" --ab-json "$OUT/${RTAG}_ntab2_${K}${N}_p${P}_f64.json"
        grep ntload "$OUT/ntab2_${K}${N}_p$P.log" | tee -a "$OUT/session.log"
      done ;;
    cachetests) # the bitwise tests of the cache-policy switches
      step pytest_cache 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rA --timeout 300 --timeout-method thread -k "every_cache or ntload or cache_flip or mfree_shapes" ;;
    capsab4) # cached fp64 caps again, now that rounds load non-temporally (g_defer_ntload)
      C_SPECS="0,4,4,3,3,0,3;0,0,0,0,0,0,0;0,5,4,4,4,0,3;4,4,4,3,3,0,3;0,4,4,3,3,0,4;0,4,4,3,3,0,2;0,5,5,4,4,0,3"
      for W in "hilbert 8192 0" "hilbert 23040 8" "random 12288 0"; do
        set -- $W; K=$1; N=$2; P=$3
        step "capsab4_${K}${N}_p$P" 300 python3 tools/defer_profile.py --kind $K --n $N --rank-block $P --dtype f64 --cycles 40 --passes 5 --caps-ab "$C_SPECS" --ab-json "$OUT/${RTAG}_capsab4_${K}${N}_p${P}_f64.json"
        grep caps "$OUT/capsab4_${K}${N}_p$P.log" | tee -a "$OUT/session.log"
      done ;;
    sq) # SQ instruction / wait counters of the deferred launches (two PMC passes)
      C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      C2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"
      for W in "random 32768 f64" "hilbert 8192 f64"; do
        set -- $W; D="$OUT/sq_$1$2_$3"; mkdir -p "$D"
        step "sq1_$1$2" 120 rocprofv3 --pmc $C1 --output-format csv -d "$D/p1" -o run -- python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 2
        step "sq2_$1$2" 120 rocprofv3 --pmc $C2 --output-format csv -d "$D/p2" -o run -- python3 tools/defer_profile.py --kind $1 --n $2 --dtype $3 --cycles 2
        python3 tools/sq_counters.py "$D/p1/run_counter_collection.csv" "$D/p2/run_counter_collection.csv" --json="$OUT/${RTAG}_sq_counters_defer_$1$2_$3.json" | tee -a "$OUT/session.log"
      done ;;
    weakshape) # piece size (4 / 8 KB) of the every-round launch on the weak-scaled rank blocks
      FMS_EVERY=1 FMS_U1=1 FMS_PT=0,4,8 step weakshape 400 ./tools/flat_map_sweep f64 8192 5824x11648 4096x16384 2880x23040 ;;
    pipe) # the software-pipelined deferred kernel (k_pipe) against k_flat, with a bitwise check
      make -s -C tools store_probe
      SP_CHECK=1 SP_PIPE=1 step pipe_probe 400 ./tools/store_probe 32768 8192x65536 ;;
    storeprobe) # the storing round's shapes and caps (tools/store_probe)
      make -s -C tools store_probe
      SP_CAPS=1 SP_ONLY=store step storeprobe_nt 300 ./tools/store_probe 32768 8192x65536
      SP_CAPS=1 SP_CACHED=1 step storeprobe_cached 200 ./tools/store_probe 8192 ;;
    defer) # the deferred-write rounds over whole store cycles: rocprof + HIP events
      for W in "hilbert 8192 f64" "random 32768 f64" "random 32768 f32"; do
        set -- $W; K=$1; N=$2; DT=$3; D="$OUT/defer_${K}${N}_${DT}"; mkdir -p "$D"
        step "defer_${K}${N}_${DT}" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/prof" -o run -- python3 tools/defer_profile.py --kind $K --n $N --dtype $DT --events "$D/events.json"
        python3 tools/defer_profile.py --kind $K --n $N --dtype $DT --trace "$D/prof/run_kernel_trace.csv" --events "$D/events.json" --json "$D/${RTAG}_defer_cycle_${K}${N}_${DT}.json" --launches "$D/${RTAG}_defer_cycle_${K}${N}_${DT}_launches.csv" | tee -a "$OUT/session.log"
      done ;;
    defer_pmc) # HBM bytes per deferred launch (separate FETCH / WRITE passes)
      for W in "hilbert 8192 f64" "random 32768 f64" "random 32768 f32"; do
        set -- $W; K=$1; N=$2; DT=$3; D="$OUT/defer_pmc_${K}${N}_${DT}"; mkdir -p "$D"
        step "defer_fetch_${K}${N}_${DT}" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run -- python3 tools/defer_profile.py --kind $K --n $N --dtype $DT --cycles 3
        step "defer_write_${K}${N}_${DT}" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/write" -o run -- python3 tools/defer_profile.py --kind $K --n $N --dtype $DT --cycles 3
        python3 tools/defer_profile.py --kind $K --n $N --dtype $DT --fetch "$D/fetch/run_counter_collection.csv" --write "$D/write/run_counter_collection.csv" --json "$D/pmc.json" | tee -a "$OUT/session.log"
      done ;;
    profile_f32) # configs[4]: 32768^2 fp32 every-round flat round, trace + PMC passes
      D="$OUT/random32768_f32"
      step prof_f32 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/prof" -o run -- python3 bench.py --kind random --n 32768 --dtype f32 --steps 50 --warmup 3 --no-cpu --no-north-star --no-headline
      step pmc_fetch_f32 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 bench.py --kind random --n 32768 --dtype f32 --steps 20 --warmup 2 --no-cpu --no-north-star --no-headline
      step pmc_write_f32 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 bench.py --kind random --n 32768 --dtype f32 --steps 20 --warmup 2 --no-cpu --no-north-star --no-headline
      python3 tools/pmc_traffic.py --workload random32768_f32 --n 32768 --elem 4 --dtype float --fetch "$D/pmc_fetch/run_counter_collection.csv" --write "$D/pmc_write/run_counter_collection.csv" --trace "$D/prof/run_kernel_trace.csv" --out "$D/pmc.json" | tee -a "$OUT/session.log" ;;
    split) step split_cost 600 python3 tools/split_cost.py ;;
    fp32)  step fp32_study 600 python3 tools/fp32_study.py --out "$OUT/fp32_study.json" ;;
    profile)
      # one workload per profiled command, so every rocprofv3 summary row
      # belongs to a single launch shape: configs[1] and the north-star size
      for W in ${PROFILE_CASES:-hilbert,8192 random,32768}; do
        set -- ${W//,/ }; K=$1; N=$2; D="$OUT/${K}${N}"
        step "prof_${K}${N}" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/prof" -o run -- python3 bench.py --kind $K --n $N --no-cpu --no-north-star --no-headline
        step "pmc_fetch_${K}${N}" 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 bench.py --kind $K --n $N --steps 20 --warmup 2 --no-cpu --no-north-star --no-headline
        step "pmc_write_${K}${N}" 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 bench.py --kind $K --n $N --steps 20 --warmup 2 --no-cpu --no-north-star --no-headline
        python3 tools/pmc_traffic.py --workload "${K}${N}_f64" --n $N --fetch "$D/pmc_fetch/run_counter_collection.csv" --write "$D/pmc_write/run_counter_collection.csv" --trace "$D/prof/run_kernel_trace.csv" --out "$D/pmc.json" | tee -a "$OUT/session.log"
      done ;;
  esac
done
echo "== session done" | tee -a "$OUT/session.log"
