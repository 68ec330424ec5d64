# round 5 session 26: bitwise shared reciprocals in the exact lane kernel's setup (QPGPU_LANE_BRCP,
# C1-only A/B builds brcp1 / brcp0 from the same source): C1 parity of brcp1, then C1 benches at
# the default step counts, alternating, three runs each
set -u
O=gpurun_out/r05_s26
mkdir -p $O
export TMPDIR=/tmp
QPGPU_LIB_PATH=_ab/brcp1/libqpgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "full_size_c1 or c4_shard" --timeout 300 --timeout-method thread > $O/parity_brcp1.log 2>&1; echo "parity rc=$?"; tail -n 3 $O/parity_brcp1.log
for rep in 1 2 3; do
  for v in brcp0 brcp1; do
    QPGPU_LIB_PATH=_ab/$v/libqpgpu.so timeout -k 10 300 python bench.py --no-cpu --no-c4 > $O/bench_C1_${v}_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(r['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,4), 'G/s', 'consistent', d['outputs_consistent'])"; done
echo done
