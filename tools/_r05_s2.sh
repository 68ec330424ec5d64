# round 5 session 2: (a) the loop-top exit under the iterative-ILP scheduler —
# taken (ilpx1), compiled in but never taken (ilpx2), default scheduler (defx1), in-tree build;
# (b) the exact C1 kernel's phase stamps and SQ counters; (c) the pre-select-in-scan A/B
# (presel: exact build, preself: fast build): parity, then C1 / C2 kernel times
set -u
O=gpurun_out/r05_s2
mkdir -p $O
export TMPDIR=/tmp
for v in intree ilpx1 ilpx2 defx1; do
  if [ $v = intree ]; then L=""; else L=_ab/$v/libqpgpu.so; fi
  QPGPU_LIB_PATH=$L timeout -k 10 300 python tools/fast_worst.py general 8 0 16 1001 816 > $O/worst_$v.log 2>&1
  rc=$?; echo "worst $v rc=$rc"; head -4 $O/worst_$v.log | tail -1
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 300 python tools/stamps.py general qp_major > $O/stamps_exact.log 2>&1 || exit $?
timeout -k 10 300 python tools/stamps.py box qp_major > $O/stamps_exact_box.log 2>&1 || exit $?
cat $O/stamps_exact.log
for v in presel preself; do
  QPGPU_LIB_PATH=_ab/$v/libqpgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "full_size or edge or config_parity or batch_tail or c4_shard or fast" > $O/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -3 $O/parity_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for rep in 1 2; do
  for c in C1 C2; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-c4 --steps 30 > $O/bench_${c}_base_$rep.log 2>&1 || exit $?
    QPGPU_LIB_PATH=_ab/presel/libqpgpu.so timeout -k 10 300 python bench.py --config $c --no-cpu --no-c4 --steps 30 > $O/bench_${c}_presel_$rep.log 2>&1 || exit $?
    QPGPU_LIB_PATH=_ab/preself/libqpgpu.so timeout -k 10 300 python bench.py --config $c --fast --no-cpu --no-c4 --steps 30 > $O/bench_${c}_preself_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); o=d.get('other_arithmetic',{}); print('$f', d['config']['kernel'], round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s; other', o.get('kernel'), round(o.get('kernel_ms',0)*1e3,2))"; done
CFG=C1 bash tools/gpu_session.sh r05_s2 sqcfg || exit $?
echo done
