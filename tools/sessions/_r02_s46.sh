O=gpurun_out/r02_s46; mkdir -p $O
for C in 0 3; do
  BENCH_COOL_S=$C timeout -k 10 900 python bench.py --no-cpu --no-headline > $O/bench_cool$C.log 2>&1 || exit 1
done
for C in 0 3; do python3 -c "
import json
d=json.loads([l for l in open('$O/bench_cool$C.log') if l.startswith('{')][-1])
print('cool $C', d['ms_per_step'], 'ns', d['north_star']['ms_per_iteration'], 'c4', d['configs4_f32']['ms_per_iteration'], 'c3', d['configs3_p1']['ms_per_iteration'], {k:v['ms_per_iteration'] for k,v in d['configs3_p1']['rank_blocks'].items() if k!='note'}, {k:v['ms_per_iteration'] for k,v in d['deferred_writes'].items()})"; done
