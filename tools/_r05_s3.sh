# round 5 session 3: (a) the round-4 lane source (64dd725^, loop-top exit) rebuilt: iterative-ILP
# (oldilp), the same with every s_waitcnt forced to zero (oldilpwz), default scheduler (olddef);
# (b) FETCH_SIZE calibration incl. the 4-B line touches; (c) C1 traffic attribution: where the
# warm-up of CI rows 5-6 / ci0 happens (base: after CE -> AGPR; warm0: none; warm2: last step)
set -u
O=gpurun_out/r05_s3
mkdir -p $O
export TMPDIR=/tmp
for v in oldilp oldilpwz olddef; do
  QPGPU_LIB_PATH=_ab/$v/libqpgpu.so timeout -k 10 300 python tools/fast_worst.py general 8 0 16 1001 816 > $O/worst_$v.log 2>&1
  rc=$?; echo "worst $v rc=$rc"; head -4 $O/worst_$v.log | tail -1
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
bash tools/gpu_session.sh r05_s3 calib || exit $?
cat $O/pmc_calibration.json
for v in base warm0 warm2; do
  if [ $v = base ]; then L=""; else L=_ab/$v/libqpgpu.so; fi
  QPGPU_LIB_PATH=$L timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o k -- python3 bench.py --no-cpu --no-c4 --streams 1 --steps 5 --warmup 1 --kernel-reps 3 > $O/pmc_$v.log 2>&1 || exit $?
  python3 - $O/pmc_$v <<'PY'
import csv, glob, statistics, sys
vals = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f)) if "qpk::qp_lane_kernel" in r["Kernel_Name"]]
print(sys.argv[1], "FETCH_SIZE KiB median", statistics.median(vals), "-> MB /0.501", 1024 * statistics.median(vals) / 0.501 / 1e6)
PY
done
for rep in 1 2; do
  for v in base warm0 warm2; do
    if [ $v = base ]; then L=""; else L=_ab/$v/libqpgpu.so; fi
    QPGPU_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-c4 --steps 30 > $O/bench_${v}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v', round(d['roofline']['kernel_ms']*1e3,2), 'us', round(d['value']/1e9,3), 'G/s')"
  done
done
echo done
