# round 5 session 14: iterative-ilp scheduler knobs on the C1 lane kernel (C1-only A/B builds):
# c1base (the in-tree flags), AMDGPU register-pressure trackers, metric bias 0, memory clauses <= 4
set -u
O=gpurun_out/r05_s14
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in c1base trk bias0 clause4; do
    QPGPU_LIB_PATH=_ab/$v/libqpgpu.so timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
