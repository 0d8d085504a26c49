#!/bin/bash
# Print the result of a tools/gpu_check.sh run.
out=gpurun_out/$1
grep -E "^E  |passed|failed|rc=" $out/tests.log | head -20
python - "$out/bench.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')]
if not l:
    print(open(sys.argv[1]).read()[-1500:]); sys.exit()
d = json.loads(l[-1])
print(f"{d['value']/1e6:.2f} Mops/s  {d['ms_per_step']:.3f} ms/step  commits/step {d['detail']['committed_per_step_rank0']:.0f}",
      {k: round(v, 3) for k, v in d['roofline']['batch_ms'].items()}, "roofline frac", round(d['roofline']['frac'], 4),
      "cpu", d.get('cpu_baseline', {}).get('value'))
PY
f=$(find $out/prof -name "*kernel_stats.csv" 2>/dev/null | head -1)
[ -n "$f" ] && python tools/rocprof_summary.py $f --top ${2:-14}
