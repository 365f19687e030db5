O=gpurun_out/r02_s43; mkdir -p $O
timeout -k 10 300 python3 tools/alloc_probe.py --reps 4 > $O/alloc_before.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu --no-headline > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/alloc_probe.py --reps 4 > $O/alloc_after.log 2>&1 || exit 1
grep -h '^{' $O/alloc_before.log $O/alloc_after.log
python3 -c "
import json
d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('north', d['north_star']['ms_per_iteration'], 'c3p1', d['configs3_p1']['ms_per_iteration'], 'head', d['ms_per_step'])"
