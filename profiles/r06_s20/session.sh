O=gpurun_out/r06_s20
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/shu32/libqpgpu.so step shadow_tests_u32 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -k "shadow"
step c5_u8 400 python -u bench.py --config C5 --no-cpu
QPGPU_LIB_PATH=_ab/shu16/libqpgpu.so step c5_u16 400 python -u bench.py --config C5 --no-cpu
QPGPU_LIB_PATH=_ab/shu32/libqpgpu.so step c5_u32 400 python -u bench.py --config C5 --no-cpu
step c5_noshadow 400 python -u bench.py --config C5 --no-cpu --no-shadow
