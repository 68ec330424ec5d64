# round 5 session 24: the time-based pre-warm (--prewarm-ms, default 40) — short step counts
# (W 10, K 50) against the defaults and against no pre-warm, C1; the 2-rank rehearsal; C5
set -u
O=gpurun_out/r05_s24
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-c4 --warmup 10 --steps 50 --prewarm-ms 0 > $O/bench_short_nopw_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu --no-c4 --warmup 10 --steps 50 > $O/bench_short_pw_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu --no-c4 > $O/bench_default_$rep.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --gpus 2 --steps 50 --warmup 10 > $O/dist2.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config C5 --no-cpu --no-c4 --kernel-reps 2 > $O/bench_C5.log 2>&1 || exit $?
for f in $O/bench_*.log $O/dist2.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; h=r.get('hbm', r); print('$f', d['steps'], d['warmup'], d.get('prewarm'), round(d['value']/1e9,5), 'G/s', 'kernel', round(h['kernel_ms']*1e3,2))"; done
echo done
