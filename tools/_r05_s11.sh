# round 5 session 11: the lane kernel under iterative-minreg (C2's best strategy in round 3,
# profiles/r03_s13) against the in-tree iterative-ilp, C2 and C1, alternating
set -u
O=gpurun_out/r05_s11
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base minreg; do
    L=""; [ $v != base ] && L=_ab/$v/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config C2 --no-cpu --no-c4 --steps 30 > $O/bench_C2_${v}_$rep.log 2>&1 || exit $?
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
