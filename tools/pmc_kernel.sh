#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over any python command, summarised for
# the dispatches whose kernel name contains FILTER.  GPU only; outputs under gpurun_out/.
# Usage: bash tools/pmc_kernel.sh TAG FILTER python tools/xyz.py args...
export TMPDIR=/tmp
TAG=$1; FILTER=$2; shift 2
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$TAG$i -o p -- \
      "$@" > gpurun_out/pmc_$TAG$i.log 2>&1 || echo "pass $i failed rc=$?"
done
python - "$TAG" "$FILTER" <<'PY'
import csv, glob, sys, collections
tag, filt = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/pmc_{tag}*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:32s} {tot[k] / max(n[k], 1):16.1f}  (n={n[k]})")
PY
