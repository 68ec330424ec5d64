# round 5 session 1: parity gate (plain per-QP bar), exact-build default lines, trace of the
# 3-stream run, rocprof stats and PMC traffic of the exact C1 kernel
set -u
T=r05_s1
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh $T pytest smoke bench trace3 || exit $?
CFGS="C2 mgqp C3 C5" bash tools/gpu_session.sh $T benchfull || exit $?
timeout -k 10 600 python bench.py --fast --steps 20 --warmup 5 --no-c4 > $O/bench_C1_fast.log 2>&1 || exit $?
CFGS="C1" bash tools/gpu_session.sh $T profcfg pmccfg || exit $?
echo done
