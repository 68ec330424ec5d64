# round 5 session 23: stream count of the pipelined value at steady-state step counts (C1),
# alternating, two runs each
set -u
O=gpurun_out/r05_s23
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for s in 2 3 4 6; do
    timeout -k 10 300 python bench.py --no-cpu --no-c4 --streams $s > $O/bench_s${s}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms']*1e3,2))"; done
echo done
