#!/bin/bash
# One GPU session on the gpurun box: parity tests, smoke, bench, rocprofv3 kernel trace and
# HBM counters.  Every GPU step has its own time limit; a crash / timeout (exit code other than
# 0 or 1) ends the session immediately.
#   usage: tools/gpu_session.sh TAG [steps...]   steps: pytest smoke bench prof pmc
set -u
TAG=${1:-session}
shift
STEPS=${*:-"pytest smoke bench prof pmc"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 limit=$2
  shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with rc=$rc"
    exit $rc
  fi
}
for s in $STEPS; do
  case $s in
    pytest) run pytest 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchfull)
      # every config's line with its CPU baseline (bounded sample) and parity sample
      for c in ${CFGS:-C1 C2 mgqp C3}; do run benchfull_$c 900 python bench.py --config $c --steps 20 --cpu-seconds 10; done
      case " ${CFGS:-C1 C2 mgqp C3 C5} " in *" C5 "*) run benchfull_C5 900 python bench.py --config C5 --steps 3 --warmup 1 --kernel-reps 3 --cpu-seconds 10 ;; esac ;;
    c5res)
      # C5 with fewer resident QPs (Infinity-Cache residency experiment): one warm input set,
      # batch B (160 QPs x 1.5 MiB of CI + J ~ 240 MiB fits the 256 MiB Infinity Cache)
      for b in ${C5B:-160 256 512 4096}; do run bench_C5_b$b 600 python bench.py --config C5 --batch $b --input-sets 1 --no-cpu --no-c4 --steps 3 --warmup 1 --kernel-reps 2 --streams 1; done ;;
    fastdiag)
      for v in ${VARIANTS}; do QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run fastdiag_$v 600 python tools/fast_diag.py C1 C2; done ;;
    profcfg)
      # rocprofv3 kernel trace + stats of one config's bench (serialized launches), per config
      for c in ${CFGS:-C1}; do
        case $c in C5) xa="--steps 3 --warmup 1 --kernel-reps 2";; C3) xa="--steps 5 --warmup 1 --kernel-reps 3";; *) xa="--steps 20 --warmup 5";; esac
        run prof_$c 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o k -- python3 bench.py --config $c --no-cpu --no-c4 --streams 1 $xa
      done ;;
    benchtiled) run bench_tiled64 600 python bench.py --layout tiled64 --no-cpu --no-c4 --steps 20 ;;
    benchfam)
      for f in ${FAMILIES:-lane subgroup}; do for l in qp_major tiled64; do run bench_${f}_$l 600 python bench.py --family $f --layout $l --no-cpu --no-c4; done; done ;;
    benchall)
      for c in C1 C2 mgqp C3; do run bench_$c 600 python bench.py --config $c --no-cpu --no-c4 --steps 20; done
      run bench_C5 600 python bench.py --config C5 --no-cpu --no-c4 --steps 3 --warmup 1 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c1 -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-c4 --streams 1 ;;
    profmgqp) run profmgqp 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmgqp" -o mgqp -- python3 tools/bench_mgqp.py --steps 3 --no-host --no-cpu ;;
    benchmgqp) run benchmgqp 600 python tools/bench_mgqp.py ;;
    benchmgqpw) run benchmgqp_wide 600 python tools/bench_mgqp.py --wide ;;
    pmc)
      run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o c1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1
      run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o c1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1
      python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" C1 65536 "$(python3 -c 'import sys; sys.path.insert(0,"motion-generation-using-quadratic-programs_amd"); import qpgpu; import os; print(qpgpu.kernel_name(7,6,14,fast=bool(os.environ.get("FAST"))))')" "$OUT/pmc_traffic.json" ;;
    stamps) for l in qp_major tiled64; do run stamps_general_$l 300 python tools/stamps.py general $l; run stamps_box_$l 300 python tools/stamps.py box $l; done ;;
    dist2) run dist2 600 python bench.py --gpus 2 --steps 10 --warmup 2 ;;
    dist2c1) run dist2c1 600 python bench.py --gpus 2 --config C1 --steps 10 --warmup 2 ;;
    trace3)
      # the default bench line's run (3 streams) under a kernel trace: do the timed steps' launches
      # overlap (ms_per_step below the kernel's own duration)?  tools/trace_overlap.py
      run trace3 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace3" -o c1 -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-c4
      python3 tools/trace_overlap.py "$OUT/trace3/c1_kernel_trace.csv" qp_lane 5 20 "$OUT/trace3_overlap.json" > "$OUT/trace3_overlap.log" 2>&1; cat "$OUT/trace3_overlap.log" ;;
    profC3) run profC3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profC3" -o c3 -- python3 bench.py --config C3 --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 3 ;;
    profC5) run profC5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profC5" -o c5 -- python3 bench.py --config C5 --steps 3 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 2 ;;
    pmcC5)
      run pmcC5_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcC5_fetch" -o c5 -- python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1
      run pmcC5_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcC5_write" -o c5 -- python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1
      python3 tools/pmc_traffic.py "$OUT/pmcC5_fetch" "$OUT/pmcC5_write" C5 4096 "$(python3 -c 'import sys; sys.path.insert(0,"motion-generation-using-quadratic-programs_amd"); import qpgpu; print(qpgpu.kernel_name(256,0,512))')" "$OUT/pmc_traffic.json" ;;
    benchcold)
      for c in C1 C2 mgqp C3; do run benchcold_$c 600 python bench.py --config $c --no-cpu --no-c4 --steps 20; done
      run benchcold_C5 600 python bench.py --config C5 --no-cpu --no-c4 --steps 3 --warmup 1 --kernel-reps 3 ;;
    fastcheck)
      # the QPGPU_FLAG_FAST lane build: parity against the oracle (1e-10, decisions), then C1 / C2
      # benches of both builds on the same box
      run fastdiag 600 python tools/fast_diag.py --fast C1 C2
      run stamps_fast 300 python tools/stamps.py general qp_major fast
      run stamps_exact 300 python tools/stamps.py general qp_major
      for c in ${CONFIGS:-C1 C2}; do
        run bench_${c}_exact 600 python bench.py --config $c --no-cpu --no-c4 --exact --steps ${ABSTEPS:-30}
        run bench_${c}_fast 600 python bench.py --config $c --no-cpu --no-c4 --fast --steps ${ABSTEPS:-30}
      done ;;
    latency)
      run latency 300 tools/dropin_latency 2000 500 ;;
    ab)
      # A/B of the in-tree build against _ab/<variant>/libqpgpu.so (tools/ab_build.sh), per config
      for c in ${CONFIGS:-C1 C2}; do
        run bench_${c}_base 600 python bench.py --config $c --no-cpu --no-c4 --steps ${ABSTEPS:-30}
        for v in ${VARIANTS}; do
          QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run bench_${c}_$v 600 python bench.py --config $c --no-cpu --no-c4 --steps ${ABSTEPS:-30}
        done
      done ;;
    abpar)
      # parity of an A/B variant: the full-size C1/C2 and edge-case parity tests against it
      for v in ${VARIANTS}; do
        QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run parity_$v 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "full_size or edge or config_parity or batch_tail or c4_shard"
      done ;;
    abstamps)
      # per-phase stamps (tools/stamps.py) of the in-tree build and each A/B variant
      run stamps_base 300 python tools/stamps.py ${KIND:-general}
      for v in ${VARIANTS}; do QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run stamps_$v 300 python tools/stamps.py ${KIND:-general}; done ;;
    wavecheck)
      # qp_wave changes: parity on every wave-covered shape, then C3 / mgqp-level benches and stamps
      run wave_parity 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -rf -k "wave or config_parity or large_config or panel or edge or tail"
      run bench_C3 600 python bench.py --config C3 --no-cpu --no-c4 --steps 10 --warmup 3
      run bench_mgqp 600 python bench.py --config mgqp --no-cpu --no-c4 --steps 20
      # stamps need the per-phase clocks compiled in: SRC=qp_wave tools/ab_build.sh stamps -DQPGPU_WAVE_STAMPS=1
      if [ -f _ab/stamps/libqpgpu.so ]; then QPGPU_LIB_PATH=_ab/stamps/libqpgpu.so run stamps_C3 300 python tools/stamps_wave.py 30 6 60 65536; fi ;;
    abwstamps)
      run wstamps_base 300 python tools/stamps_wave.py ${WSHAPE:-30 6 60 65536}
      for v in ${VARIANTS}; do QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run wstamps_$v 300 python tools/stamps_wave.py ${WSHAPE:-30 6 60 65536}; done ;;
    sqcfg)
      # SQ counters of one config's kernel (CFG, default C3): instruction mix and issue share
      c=${CFG:-C3}
      run sqA_$c 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/sqA_$c" -o c1 -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1
      run sqB_$c 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sqB_$c" -o c1 -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1
      run sqC_$c 600 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d "$OUT/sqC_$c" -o c1 -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1
      python3 tools/sqsum.py "$OUT" > "$OUT/sqsum_$c.log" 2>&1; cat "$OUT/sqsum_$c.log" ;;
    abpmc)
      # FETCH_SIZE of the C1 kernel for the in-tree build and each A/B variant (one pass each)
      run pmcab_base 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcab_base" -o c1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1
      for v in ${VARIANTS}; do QPGPU_LIB_PATH=_ab/$v/libqpgpu.so run pmcab_$v 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcab_$v" -o c1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-c4 --streams 1; done
      for d in "$OUT"/pmcab_*/; do python3 - "$d" <<'PY'
import csv, statistics, sys
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1] + "c1_counter_collection.csv")) if "qp_lane" in r["Kernel_Name"]]
print(sys.argv[1], "FETCH_SIZE KiB median", statistics.median(vals), "-> bytes x2", 2 * 1024 * statistics.median(vals))
PY
      done ;;
    calib)
      # FETCH_SIZE / WRITE_SIZE calibration for the solver's access patterns (tools/fetch_probe.hip)
      run calib_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o probe -- ./tools/fetch_probe
      run calib_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o probe -- ./tools/fetch_probe
      python3 tools/pmc_calib.py "$OUT/calib_fetch" "$OUT/calib_write" "$OUT/pmc_calibration.json" ;;
    pmccfg)
      # FETCH_SIZE and WRITE_SIZE passes of one config's bench (CFG), one pass per counter
      for c in ${CFGS:-C1}; do
        case $c in C5) xa="--steps 2 --warmup 1 --kernel-reps 1";; C3) xa="--steps 3 --warmup 1 --kernel-reps 2";; *) xa="--steps 5 --warmup 1 --kernel-reps 3";; esac
        run pmc_fetch_$c 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$c" -o k -- python3 bench.py --config $c --no-cpu --no-c4 --streams 1 $xa
        run pmc_write_$c 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$c" -o k -- python3 bench.py --config $c --no-cpu --no-c4 --streams 1 $xa
        read B K < <(python3 -c "import sys; sys.path.insert(0, 'motion-generation-using-quadratic-programs_amd'); import bench, qpgpu; c = bench.CONFIGS['$c']; import os; print(c[4], qpgpu.kernel_name(c[1], c[2], c[3], fast=bool(os.environ.get('FAST'))))")
        python3 tools/pmc_traffic.py "$OUT/pmc_fetch_$c" "$OUT/pmc_write_$c" $c $B "$K" "$OUT/pmc_traffic.json"
      done ;;
    listctr) rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "listctr rc=$?" ;;
    sq)
      for f in ${FAMILIES:-lane subgroup}; do
        run sqA_$f 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/sqA_$f" -o c1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-c4 --family $f --layout ${LAYOUT:-qp_major}
        run sqB_$f 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sqB_$f" -o c1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-c4 --family $f --layout ${LAYOUT:-qp_major}
        run sqC_$f 600 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d "$OUT/sqC_$f" -o c1 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-c4 --family $f --layout ${LAYOUT:-qp_major}
      done ;;
  esac
done
echo "session $TAG done"
