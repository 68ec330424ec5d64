# the final tree (round 6): GPU suite, smoke, every config's bench line, rocprof traces, HBM counters, drop-in latency
O=gpurun_out/r06_f7
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo STOP; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
step prof_C1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C1 -o k -- python3 bench.py --no-cpu --no-c4
for c in C1 C2 mgqp C3; do
  [ $c = C1 ] || step bench_$c 600 python -u bench.py --config $c
  step pmcf_$c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$c -o k -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 5 --kernel-rounds 1 --prewarm-ms 0
  step pmcw_$c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$c -o k -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 5 --kernel-rounds 1 --prewarm-ms 0
done
step bench_C5 900 python -u bench.py --config C5
step prof_C5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C5 -o k -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 --kernel-reps 2 --kernel-rounds 1
step pmcf_C5 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_C5 -o k -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu --kernel-reps 1 --kernel-rounds 1 --prewarm-ms 0
step pmcw_C5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_C5 -o k -- python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu --kernel-reps 1 --kernel-rounds 1 --prewarm-ms 0
step dropin_latency 300 tools/dropin_latency 2000 500
step latency_parts 300 tools/latency_parts 2000
