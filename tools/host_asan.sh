#!/bin/bash
# The library's HOST code under AddressSanitizer + UndefinedBehaviorSanitizer
# (-Xarch_host only: device code is built as shipped; GPU ASan is not
# available on the pool), driven by tests/cpp/capi_sanitize.c.
#   bash tools/host_asan.sh build   # here (about 2.5 min: st_kernels.hip)
#   bash tools/host_asan.sh run     # here (argument / policy paths) or on a
#                                   # GPU box (also the device solve paths)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/tools/asan
if [ "${1:-run}" = build ]; then
  mkdir -p $D
  # the tuning build's ABI (-DST_TUNING_ABI=1): the driver checks the setters too
  FL="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -ffp-contract=off -DST_TUNING_ABI=1 -I$ROOT/include -I$ROOT/eigen_value_amd/csrc"
  SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
  for f in st_kernels st_solve st_multi st_rendezvous; do
    /opt/rocm/bin/hipcc $FL $SAN -c $ROOT/eigen_value_amd/csrc/$f.hip -o $D/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $SAN -o $D/libsimilarity_transform.so \
    $D/st_kernels.o $D/st_solve.o $D/st_multi.o $D/st_rendezvous.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm -f $D/*.o
  /opt/rocm/lib/llvm/bin/clang -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
    -I$ROOT/include $ROOT/tests/cpp/capi_sanitize.c -L$D -lsimilarity_transform \
    -Wl,-rpath,'$ORIGIN' -lpthread -o $D/capi_sanitize
  echo "built $D/capi_sanitize"
else
  # verify_asan_link_order=0: the environment may preload a library first;
  # leaks inside the HIP / HSA / RCCL runtimes (their process-lifetime
  # allocations) are not this library's and are suppressed
  # LEAKS=0 on a GPU box: LeakSanitizer's exit-time stop-the-world hung
  # there behind the HIP runtime's threads (profiles/r04_host_asan_gpu.log)
  printf 'leak:libamdhip64.so\nleak:libhsa-runtime64.so\nleak:librccl.so\n' > $D/lsan.supp
  ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=${LEAKS:-1} \
    LSAN_OPTIONS=suppressions=$D/lsan.supp $D/capi_sanitize
fi
