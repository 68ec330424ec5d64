# round 5 final tree: the GPU suite, the smoke and the default bench line exactly as the driver
# runs them (python bench.py, no flags)
set -u
T=r05_f6
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh $T pytest smoke bench || exit $?
python3 -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'], 'pipelined', r['pipelined']['frac'], 'traffic', r['traffic_measured_on'], 'parity', d['cpu_baseline']['parity']['meets_north_star'], d['cpu_baseline']['parity']['qps'])"
echo done
