# round 5 session 22: rocprof of sustained serialized runs (--streams 1, the per-config default
# step counts), steady-state kernel durations from the trace's last dispatches (tools/trace_steady.py)
set -u
O=gpurun_out/r05_s22
mkdir -p $O
export TMPDIR=/tmp
for c in C1 C2 mgqp C3; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o k -- python3 bench.py --config $c --no-cpu --no-c4 --streams 1 > $O/prof_$c.log 2>&1 || exit $?
  echo "== $c"; python3 tools/trace_steady.py $O/prof_$c/k_kernel_trace.csv qp_ 100 | tee $O/steady_$c.txt
  python3 -c "import json; d=json.loads(open('$O/prof_$c.log').read().strip().splitlines()[-1]); r=d['roofline']; h=r.get('hbm', r); print('bench kernel_ms', round(h['kernel_ms']*1e3,2), 'us', [round(x*1e3,1) for x in h['kernel_ms_rounds']])" | tee -a $O/steady_$c.txt
done
echo done
