O=gpurun_out/r06_s6
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step latency_parts 300 tools/latency_parts 1000
STAMPS_B=1 step stamps_one_qp 120 python -u tools/stamps.py general qp_major
STAMPS_B=64 step stamps_one_wave 120 python -u tools/stamps.py general qp_major
step bench_C1 600 python -u bench.py
step bench_C5 900 python -u bench.py --config C5
