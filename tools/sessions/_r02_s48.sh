O=gpurun_out/r02_s48; mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('head', d['ms_per_step'], 'ns', d['north_star']['ms_per_iteration'], d['north_star'].get('in_process'), 'mf', d['north_star']['matrix_free']['ms_per_iteration'])
print('c4', d['configs4_f32']['ms_per_iteration'], 'c3', d['configs3_p1']['ms_per_iteration'], d['configs3_p1'].get('in_process'))
print({k:v['ms_per_iteration'] for k,v in d['configs3_p1']['rank_blocks'].items() if k!='note'})
print({k:(v['ms_per_iteration'], v.get('events_vs_rocprof'), v['bitwise_equal_to_write_every_round']) for k,v in d['deferred_writes'].items()})
print('cpu', d['cpu_baseline']['ms_per_iteration'], list(d))"
