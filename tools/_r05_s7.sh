# round 5 session 7: C5 with two deferred add_constraint sweeps (qp_wave.hip, QPGPU_WAVE_TOLLOOP
# bit 3): the tolerance-path parity tests, the C5 bench line, its PMC traffic and rocprof stats
set -u
T=r05_s7
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -rf --timeout 600 --timeout-method thread -k "c5 or panel or large_config or generic_beyond or edge_parity" > $O/pytest_tol.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_tol.log
if [ $rc -ne 0 ]; then exit $rc; fi
CFGS="C5" bash tools/gpu_session.sh $T benchfull pmccfg profcfg || exit $?
python3 -c "import json; d=json.load(open('$O/pmc_traffic.json')); [print(k, v['write_kib'], v['hbm_bytes_per_launch']/1e9) for k, v in d.items()]"
echo done
