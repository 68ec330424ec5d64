# round 5 session 13: the wave kernel's scheduler strategy — LLVM's default (in-tree) against
# iterative-minreg and iterative-maxocc, mgqp level and C3 (bitwise builds), alternating
set -u
O=gpurun_out/r05_s13
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base wminreg wmaxocc; do
    L=""; [ $v != base ] && L=_ab/$v/libqpgpu.so
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config mgqp --no-cpu --no-c4 --steps 20 > $O/bench_mgqp_${v}_$rep.log 2>&1 || exit $?
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --config C3 --no-cpu --no-c4 --steps 10 --warmup 3 > $O/bench_C3_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e6,3), 'M/s', 'consistent', d['outputs_consistent'])"; done
echo done
