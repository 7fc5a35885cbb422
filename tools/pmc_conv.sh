# PMC passes over one conv shape (tools/conv_probe.py --only); GPU only.  Usage: bash tools/pmc_conv.sh TAG "<probe args>"
export TMPDIR=/tmp
TAG=$1; shift
P="python tools/conv_probe.py $* --iters 20"
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
         "FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$TAG$i -o p -- $P > gpurun_out/pmc_$TAG$i.log 2>&1 || echo "pass $i failed rc=$?"
done
