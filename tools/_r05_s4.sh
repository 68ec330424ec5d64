# round 5 session 4: the product with the DMA path's warm-up dropped and the fast build's
# loop-top exit on: full GPU suite, smoke, default bench, C1 / C2 PMC traffic (exact and fast
# kernels of the same passes), rocprof stats of C1 / C2
set -u
T=r05_s4
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_session.sh $T pytest smoke bench || exit $?
CFGS="C1 C2" bash tools/gpu_session.sh $T pmccfg profcfg || exit $?
for c in C1 C2; do
  K=$(python3 -c "import sys; sys.path.insert(0, 'motion-generation-using-quadratic-programs_amd'); import qpgpu; print(qpgpu.kernel_name(7, 6 if '$c' == 'C1' else 0, 14, fast=True))")
  python3 tools/pmc_traffic.py "$O/pmc_fetch_$c" "$O/pmc_write_$c" $c 65536 "$K" "$O/pmc_traffic.json" > $O/pmc_fast_$c.log 2>&1
done
echo done
