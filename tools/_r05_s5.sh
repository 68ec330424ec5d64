# round 5 session 5: the cooperative finish (qp_lane): full GPU suite on the in-tree
# build (coop on), then kernel times against the same build with QPGPU_LANE_COOP=0 (nocoop: exact
# TU, nocoopf: fast TU), C1 and C2, alternating, and the phase stamps
set -u
O=gpurun_out/r05_s5
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh r05_s5 pytest smoke || exit $?
for rep in 1 2; do
  for c in C1 C2; do
    for v in coop nocoop; do
      L=""; [ $v = nocoop ] && L=_ab/nocoop/libqpgpu.so
      QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --no-cpu --no-c4 --steps 30 > $O/bench_${c}_${v}_$rep.log 2>&1 || exit $?
      L=""; [ $v = nocoop ] && L=_ab/nocoopf/libqpgpu.so
      QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --fast --no-cpu --no-c4 --steps 30 > $O/bench_${c}_${v}f_$rep.log 2>&1 || exit $?
    done
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
timeout -k 10 300 python tools/stamps.py general qp_major > $O/stamps_coop.log 2>&1 || exit $?
QPGPU_LIB_PATH=_ab/nocoop/libqpgpu.so timeout -k 10 300 python tools/stamps.py general qp_major > $O/stamps_nocoop.log 2>&1 || exit $?
head -12 $O/stamps_coop.log; head -12 $O/stamps_nocoop.log
echo done
