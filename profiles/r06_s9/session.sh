# the final tree as the driver runs it, plus every config's bench line
O=gpurun_out/r06_s9
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-600; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
for c in C2 mgqp C3; do step bench_$c 600 python -u bench.py --config $c; done
step bench_C5 900 python -u bench.py --config C5
