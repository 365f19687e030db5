O=gpurun_out/r02_s39; mkdir -p $O
timeout -k 10 600 python bench.py --no-cpu --no-north-star --no-headline > $O/bench.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print(d['ms_per_step'], json.dumps(d['weak_rank_blocks'], indent=1))"
