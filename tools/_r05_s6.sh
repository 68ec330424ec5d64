# round 5 session 6: round B (CE) landing after J = L^-T and the solve (in-tree) against right
# after the Cholesky (celate0 / celate0f), C1 and C4 exact and fast, alternating; GPU suite first
set -u
O=gpurun_out/r05_s6
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh r05_s6 pytest || exit $?
for rep in 1 2 3; do
  for v in late early; do
    L=""; [ $v = early ] && L=_ab/celate0/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
    L=""; [ $v = early ] && L=_ab/celate0f/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --fast --no-cpu --no-c4 --steps 30 > $O/bench_C1_${v}f_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s', 'consistent', d['outputs_consistent'])"; done
timeout -k 10 300 python tools/stamps.py general qp_major > $O/stamps_late.log 2>&1 || exit $?
QPGPU_LIB_PATH=_ab/celate0/libqpgpu.so timeout -k 10 300 python tools/stamps.py general qp_major > $O/stamps_early.log 2>&1 || exit $?
head -12 $O/stamps_late.log; head -12 $O/stamps_early.log
echo done
