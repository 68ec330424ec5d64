# round 5 session 16: C2's first-scan software-pipelining depth (QPGPU_LANE_SCAN_DEPTH, qp_lane_p0
# A/B builds): 2 (in-tree) against 1, 3 and 4, alternating, three runs each
set -u
O=gpurun_out/r05_s16
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base sd1 sd3 sd4; do
    L=""; [ $v != base ] && L=_ab/$v/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config C2 --no-cpu --no-c4 --steps 30 > $O/bench_C2_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
