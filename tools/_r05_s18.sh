# round 5 session 18: the bench's kernel duration as the median of five rounds (after 3K untimed launches, each round after five more
# untimed launches): three default runs, against rocprof of the same build
set -u
O=gpurun_out/r05_s18
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --no-c4 > $O/bench_C1_$rep.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --config C2 --no-cpu --no-c4 > $O/bench_C2.log 2>&1 || exit $?
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(r['kernel_ms']*1e3,2), 'us', [round(x*1e3,1) for x in r['kernel_ms_rounds']], 'frac', round(r['frac'],4), round(d['value']/1e9,3), 'G/s')"; done
echo done
