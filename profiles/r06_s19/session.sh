O=gpurun_out/r06_s19
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-400; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step shadow_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -k "shadow"
step large_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fuzz.py -k "large"
step bench_C5_shadow 400 python -u bench.py --config C5 --no-cpu
step bench_C5_noshadow 400 python -u bench.py --config C5 --no-cpu --no-shadow
