O=gpurun_out/r06_s22
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -22 $O/$name.log | cut -c1-200; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/stamps/libqpgpu.so step stamps_C5_4096 300 python -u tools/stamps_wave.py 256 0 512 4096
