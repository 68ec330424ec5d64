O=gpurun_out/r06_s15
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
QPGPU_LIB_PATH=_ab/p0dma2/libqpgpu.so step pytest_dma2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "box or C2 or edge or full_size or fuzz" tests/test_gpu_fuzz.py -k "not large"
for r in 1 2; do for v in p0base p0dma1 p0dma2; do
  QPGPU_LIB_PATH=_ab/$v/libqpgpu.so step c2_${v}_$r 300 python -u bench.py --config C2 --no-cpu
done; done
