# round 5 session 8: the lane kernel without the diagnostic stamp code (nostamp: QPGPU_LANE_STAMPS=0)
# against the in-tree build (stamps compiled in, null-checked at run time), C1 exact, alternating
set -u
O=gpurun_out/r05_s8
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base nostamp; do
    L=""; [ $v = nostamp ] && L=_ab/nostamp/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
