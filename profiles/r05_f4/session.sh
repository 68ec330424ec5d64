# round 5 final build (+ per-device locked LDS grants in the wave launcher): GPU suite, smoke, the default bench line,
# the 3-stream trace, rocprof stats and PMC traffic per config (bitwise kernels; the fast kernels
# from the same passes)
set -u
T=r05_f4
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh $T pytest smoke bench trace3 || exit $?
CFGS="C2" bash tools/gpu_session.sh $T benchfull || exit $?
CFGS="C1 C2 mgqp C3" bash tools/gpu_session.sh $T profcfg pmccfg || exit $?
for c in C1 C2 mgqp C3; do
  K=$(python3 -c "import sys; sys.path.insert(0, 'motion-generation-using-quadratic-programs_amd'); import bench, qpgpu; c = bench.CONFIGS['$c']; print(qpgpu.kernel_name(c[1], c[2], c[3], fast=True))")
  python3 tools/pmc_traffic.py "$O/pmc_fetch_$c" "$O/pmc_write_$c" $c 65536 "$K" "$O/pmc_traffic.json" > $O/pmc_fast_$c.log 2>&1
done
echo done
