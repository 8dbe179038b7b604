#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmcq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 scripts/qr_tsqrt_only.py"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcq/p1 -o run -- $P > gpurun_out/pmcq/p1.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmcq/p2 -o run -- $P > gpurun_out/pmcq/p2.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/pmcq/p3 -o run -- $P > gpurun_out/pmcq/p3.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2", "p3"):
    for f in glob.glob(f"gpurun_out/pmcq/{p}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:40]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in acc.items():
            if "qr_" not in k: continue
            print(p, k, {c: f"{sum(v)/len(v):.3g}" for c, v in d.items()})
PY
exit $rc
