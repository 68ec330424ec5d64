O=gpurun_out/r06_s7
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/v1/libqpgpu.so step pytest_v1 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k "large" tests/test_gpu_parity.py::test_c5_bench_problems_parity tests/test_gpu_parity.py::test_large_config_parity tests/test_gpu_parity.py::test_size_class_boundaries
for r in 1 2; do for v in v0 v1 v2 v3; do
  QPGPU_LIB_PATH=_ab/$v/libqpgpu.so step c5_${v}_$r 300 python -u tools/c5_exact_cost.py 4096 3 default
done; done
