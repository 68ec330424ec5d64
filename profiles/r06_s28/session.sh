O=gpurun_out/r06_s28
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/gocc3/libqpgpu.so step c5_gocc3 400 python -u bench.py --config C5 --no-cpu
step c5_base 400 python -u bench.py --config C5 --no-cpu
