O=gpurun_out/r06_s8
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step pytest_all 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
QPGPU_LIB_PATH=_ab/tol7/libqpgpu.so step pytest_tol7 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k "large"
QPGPU_LIB_PATH=_ab/stamps/libqpgpu.so step stamps_mgqp 300 python -u tools/stamps_wave.py 14 10 28 65536
QPGPU_LIB_PATH=_ab/stamps/libqpgpu.so step stamps_C3 300 python -u tools/stamps_wave.py 30 6 60 65536
