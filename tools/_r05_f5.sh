# round 5 final bench lines with the median-of-rounds kernel timing (library as in r05_f4):
# the default line (CPU baseline and whole-batch parity), the 3-stream trace, and C5's line
set -u
T=r05_f5
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh $T smoke bench trace3 || exit $?
timeout -k 10 600 python bench.py --config C5 --steps 3 --warmup 1 --kernel-reps 3 --no-c4 --cpu-seconds 10 > $O/bench_C5.log 2>&1 || exit $?
for f in $O/bench.log $O/bench_C5.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(r['kernel_ms']*1e3,2), 'us', [round(x*1e3,1) for x in r['kernel_ms_rounds']], 'frac', round(r['frac'],4), d['value'], r['traffic_measured_on'])"; done
echo done
