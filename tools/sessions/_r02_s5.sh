O=gpurun_out/r02_s5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $O/avail.txt 2>&1
FMS_QUICK=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc1 -o run -- ./tools/flat_map_sweep f64 32768 > $O/pmc1.log 2>&1
echo "pmc1 rc=$?"
FMS_QUICK=1 timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- ./tools/flat_map_sweep f64 32768 > $O/pmc2.log 2>&1
echo "pmc2 rc=$?"
