# C5 on the final tree: bench line (whole-batch parity), kernel trace, HBM counters; drop-in latency
O=gpurun_out/r06_f5
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step bench_C5 900 python -u bench.py --config C5
step prof_C5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C5 -o k -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 --kernel-reps 2 --kernel-rounds 1
step pmcf_C5 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_C5 -o k -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu --kernel-reps 1 --kernel-rounds 1 --prewarm-ms 0
step pmcw_C5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_C5 -o k -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu --kernel-reps 1 --kernel-rounds 1 --prewarm-ms 0
step dropin_latency 300 tools/dropin_latency 2000 500
QPGPU_LIB_PATH=_ab/occ3/libqpgpu.so step mgqp_occ3 300 python -u bench.py --config mgqp --no-cpu
QPGPU_LIB_PATH=_ab/occ4off/libqpgpu.so step mgqp_occ4off 300 python -u bench.py --config mgqp --no-cpu
step mgqp_base 300 python -u bench.py --config mgqp --no-cpu
