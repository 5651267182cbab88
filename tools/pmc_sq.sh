#!/bin/bash
# SQ counters for the engine kernels (one --pmc pass, no trace domains)
REPO="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$REPO"; export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
rm -rf "$REPO/gpurun_out/pmc_sq"
timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d "$REPO/gpurun_out/pmc_sq" -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-sample 0 --no-check --ingest-mode ${MODE:-2} --decode-steps 0 --h2d-steps 0 ${BENCH_EXTRA} > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc_sq.log
python3 - "$REPO/gpurun_out/pmc_sq" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True)
print(f)
if f:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        n = r.get("Kernel_Name", "")
        if "fw::" in n:
            agg[n[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, d in agg.items():
        print(n, {k: sum(v) / len(v) for k, v in d.items()})
PY
exit $rc
