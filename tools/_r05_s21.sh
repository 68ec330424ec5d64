# round 5 session 21: the per-config default step counts (DEFAULT_STEPS) — the default line (CPU
# baseline, whole-batch parity), C2 / mgqp / C3 lines, and the 2-rank rehearsal, with run times
set -u
O=gpurun_out/r05_s21
mkdir -p $O
export TMPDIR=/tmp
t() { local name=$1; shift; local t0=$(date +%s); timeout -k 10 900 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(( $(date +%s) - t0 )) s"; [ $rc -eq 0 ] || exit $rc; }
t bench python bench.py
for c in C2 mgqp C3; do t bench_$c python bench.py --config $c --no-cpu --no-c4; done
t dist2 python bench.py --gpus 2
for f in $O/bench*.log $O/dist2.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; h=r.get('hbm', r); print('$f', d['steps'], d['warmup'], round(d['value']/1e9,4), 'G/s', 'kernel', round(h['kernel_ms']*1e3,2), 'frac', round(h['frac'],4), 'pipelined', round(r['pipelined']['frac'],4) if r.get('pipelined') else None, h['traffic_measured_on'])"; done
echo done
