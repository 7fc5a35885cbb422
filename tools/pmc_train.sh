# HBM traffic per dispatch of the training step's kernels (config 3): separate FETCH_SIZE and
# WRITE_SIZE passes over bench.py --train (its eager attribution step between GPU spins),
# summarised by tools/pmc_traffic.py; "wgrad_kernel" aggregates every weight-gradient kernel
# (ring, register-staged, patch and halo forms; not the split reductions), matching bench.py's launch label.  GPU only.
export TMPDIR=/tmp
set -e
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmct_$C -o p -- \
      python bench.py --train --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/pmct_$C.log 2>&1
done
python tools/pmc_traffic.py gpurun_out/pmct_FETCH_SIZE/p_counter_collection.csv \
    gpurun_out/pmct_WRITE_SIZE/p_counter_collection.csv gpurun_out/pmc_traffic_train.json 16 256 \
    > gpurun_out/pmc_traffic_train.txt
python - <<'PY'
import json
p = "gpurun_out/pmc_traffic_train.json"
d = json.load(open(p))
k = d["kernels"]
sel = [v for n, v in k.items() if n.startswith("wgrad_") and "reduce" not in n]
nf = sum(v["dispatches_fetch_pass"] for v in sel)
nw = sum(v["dispatches_write_pass"] for v in sel)
fb = sum(v["fetch_bytes_per_dispatch"] * v["dispatches_fetch_pass"] for v in sel) / max(nf, 1)
wb = sum(v["write_bytes_per_dispatch"] * v["dispatches_write_pass"] for v in sel) / max(nw, 1)
k["wgrad_kernel"] = {"dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
                     "fetch_bytes_per_dispatch": round(fb), "write_bytes_per_dispatch": round(wb),
                     "hbm_bytes_per_dispatch": round(fb + wb),
                     "note": "average over every weight-gradient dispatch of one eager step"}
d["source"] += "; eager training step of bench.py --train (B16, 256x256)"
json.dump(d, open(p, "w"), indent=1)
print("wgrad_kernel", k["wgrad_kernel"])
PY
rm -rf gpurun_out/pmct_FETCH_SIZE gpurun_out/pmct_WRITE_SIZE
