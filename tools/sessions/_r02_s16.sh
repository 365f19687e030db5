O=gpurun_out/r02_s16; mkdir -p $O
export TMPDIR=/tmp
FMS_PT=0 FMS_MAX_NP=5 FMS_STORE_NP=5 timeout -k 10 300 ./tools/flat_map_sweep f64 32768 > $O/probe.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/defer_profile.py --kind random --n 32768 --dtype f64 --events $O/events.json > $O/prof.log 2>&1 || exit 1
python3 tools/defer_profile.py --kind random --n 32768 --dtype f64 --trace $O/prof/run_kernel_trace.csv --events $O/events.json --json $O/cycle.json
cat $O/probe.log
