O=gpurun_out/r06_s17
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/lane14/libqpgpu.so step parity_lane14 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "mgqp_L0 and None"
QPGPU_LIB_PATH=_ab/lane14/libqpgpu.so step bench_mgqp_lane14 300 python -u bench.py --config mgqp
