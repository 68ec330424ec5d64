# round 5 session 15: LDS and wait counters of the C1 lane kernel (one --pmc pass each), to look
# for LDS bank conflicts and where the waves wait
set -u
O=gpurun_out/r05_s15
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > $O/avail.txt 2>&1; echo "list rc=$?"
grep -o "SQ_[A-Z_]*LDS[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_INSTS_[A-Z_]*" $O/avail.txt | sort -u > $O/sq_names.txt
cat $O/sq_names.txt | tr '\n' ' '; echo
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o c1 -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-c4 --streams 1 --kernel-reps 1 > $O/$name.log 2>&1; echo "$name rc=$?"; }
run lds1 SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS || exit 1
run wait1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ["lds1", "wait1"]:
    f = glob.glob(f"gpurun_out/r05_s15/{d}/*counter_collection.csv")
    if not f: print(d, "no csv"); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "qp_lane_kernel<7, 14, 1, true, 6>" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(d, k, "per dispatch", sum(v) / max(1, len(v)))
PY
echo done
