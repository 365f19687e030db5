O=gpurun_out/r02_s38; mkdir -p $O
timeout -k 10 600 python bench.py --no-cpu > $O/bench.log 2>&1 || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print(json.dumps(d['configs3_p1'], indent=1))"
