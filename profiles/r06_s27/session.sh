O=gpurun_out/r06_s27
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-250; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step dropin_tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_dropin.py
step pytest 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step dropin_latency 300 tools/dropin_latency 2000 500
step latency_parts 300 tools/latency_parts 2000
