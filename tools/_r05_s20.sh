# round 5 session 20: sustained load before the timed regions — (W, K) and the kernel-duration
# warm-up (--kernel-warmup launches), C1, alternating, two runs each; then rocprof of a sustained
# serialized run for comparison
set -u
O=gpurun_out/r05_s20
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "10 50 -1" "200 500 -1" "200 500 300" "1000 2000 300" "1000 2000 1000"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --no-cpu --no-c4 --warmup $1 --steps $2 --kernel-warmup $3 > $O/bench_w$1_k$2_kw$3_$rep.log 2>&1 || exit $?
  done
done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'streams1', round(d['value_streams1']/1e9,4), 'kernel', round(r['kernel_ms']*1e3,2), [round(x*1e3,1) for x in r['kernel_ms_rounds']])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sust -o c1 -- python3 bench.py --no-cpu --no-c4 --streams 1 --warmup 500 --steps 1000 > $O/prof_sust.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r05_s20/prof_sust/c1_kernel_stats.csv")):
    if "qp_lane" in r["Name"]:
        print(r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, "us")
PY
echo done
