O=gpurun_out/r06_s11
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step pytest_all 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step latency_parts 300 tools/latency_parts 2000
step dropin_latency 300 tools/dropin_latency 2000 500
