O=gpurun_out/r06_s4
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step pytest_large 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k "large" tests/test_gpu_parity.py::test_c5_bench_problems_parity tests/test_gpu_parity.py::test_large_config_parity tests/test_gpu_parity.py::test_size_class_boundaries tests/test_gpu_parity.py::test_edge_parity
step cert_c5 300 python -u tools/cert_probe.py $O/cert_c5.json C5
QPGPU_LIB_PATH=_ab/stamps0/libqpgpu.so WDETAIL=0 step stamps0_C5_4096 300 python -u tools/stamps_wave.py 256 0 512 4096
step latency 120 tools/latency_parts 2000
