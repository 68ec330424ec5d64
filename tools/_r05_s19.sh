# round 5 session 19: the default line's step counts — (W, K) = (10, 50) against (100, 200) and
# (200, 500), alternating, three runs each (C1, no CPU baseline)
set -u
O=gpurun_out/r05_s19
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for wk in "10 50" "100 200" "200 500"; do
    set -- $wk
    timeout -k 10 300 python bench.py --no-cpu --no-c4 --warmup $1 --steps $2 > $O/bench_w$1_k$2_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'streams1', round(d['value_streams1']/1e9,4), 'kernel', round(r['kernel_ms']*1e3,2))"; done
echo done
