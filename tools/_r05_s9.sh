# round 5 session 9: the lane kernel's scheduler strategy — iterative-ilp (in-tree) against
# max-ilp and max-memory-clause (C1 exact, alternating, three runs each)
set -u
O=gpurun_out/r05_s9
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base maxilp maxmem; do
    L=""; [ $v != base ] && L=_ab/$v/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'], 'bitwise', d['cpu_baseline'].get('parity', {}).get('x_bitwise_equal') if d.get('cpu_baseline') else None)"; done
echo done
