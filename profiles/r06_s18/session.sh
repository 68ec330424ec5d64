O=gpurun_out/r06_s18
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/occ2/libqpgpu.so step parity_occ2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "full_size_c1 or (edge_parity and lane) or C1_general"
for r in 1 2; do
  step c1_base_$r 300 python -u bench.py --no-cpu --no-c4
  QPGPU_LIB_PATH=_ab/occ2/libqpgpu.so step c1_occ2_$r 300 python -u bench.py --no-cpu --no-c4
done
step c4_base 300 python -u bench.py --no-cpu --batch 1048576 --steps 100 --warmup 20
QPGPU_LIB_PATH=_ab/occ2/libqpgpu.so step c4_occ2 300 python -u bench.py --no-cpu --batch 1048576 --steps 100 --warmup 20
