O=gpurun_out/r06_s2
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step cert_c5 300 python -u tools/cert_probe.py $O/cert_c5.json C5
step cert_fuzz 300 python -u tools/cert_probe.py $O/cert_fuzz.json fuzz
step pytest_large 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k "large" tests/test_gpu_parity.py::test_c5_bench_problems_parity tests/test_gpu_parity.py::test_large_config_parity tests/test_gpu_parity.py::test_size_class_boundaries
step latency 120 tools/latency_parts 2000
