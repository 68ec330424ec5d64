# round 5 session 12: C2's kernels in their own object under iterative-minreg (qp_lane_p0.hip):
# the whole GPU suite, then C2 and C1 benches (three runs each)
set -u
O=gpurun_out/r05_s12
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh r05_s12 pytest || exit $?
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --config C2 --no-cpu --no-c4 --steps 30 > $O/bench_C2_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_$rep.log 2>&1 || exit $?
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
