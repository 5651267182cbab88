#!/bin/bash
# PMC passes (one counter group per run) over a microbenchmark binary: BIN ARGS
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
BIN=$1; shift
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $CTRS --output-format csv -d "$REPO/gpurun_out/pmc_mb_$i" -o run -- $BIN "$@" > gpurun_out/pmc_mb_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_mb_$i.log; exit 1; }
done
python3 - "$REPO/gpurun_out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc_mb_*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r.get("Kernel_Name", "")[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in sorted(agg.items()):
    print(n)
    for k, v in sorted(d.items()):
        print("   %-24s %14.1f  (n=%d)" % (k, sum(v) / len(v), len(v)))
PY
