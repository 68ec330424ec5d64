# round 5 session 27: C2 with the CI copy by LDS-DMA after the setup (QPGPU_LANE_DMA_P0=1,
# qp_lane_p0 A/B build) against the in-tree first-scan fill, default step counts, alternating
set -u
O=gpurun_out/r05_s27
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base dmap0; do
    L=""; [ $v != base ] && L=_ab/$v/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config C2 --no-cpu --no-c4 > $O/bench_C2_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(r['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,4), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
