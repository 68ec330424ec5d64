O=gpurun_out/r06_s3
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 $O/$name.log; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step cert_c5 300 python -u tools/cert_probe.py $O/cert_c5.json C5
step cert_fuzz 300 python -u tools/cert_probe.py $O/cert_fuzz.json fuzz
step pytest_all 1500 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for v in 0 1 2; do
  QPGPU_LIB_PATH=_ab/stamps$v/libqpgpu.so WDETAIL=$v step stamps${v}_C5_4096 300 python -u tools/stamps_wave.py 256 0 512 4096
  QPGPU_LIB_PATH=_ab/stamps$v/libqpgpu.so WDETAIL=$v step stamps${v}_C5_160 300 python -u tools/stamps_wave.py 256 0 512 160
done
