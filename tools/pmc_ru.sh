export TMPDIR=/tmp
P="python tools/ru_probe.py --iters 10"
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/rpmc$i -o p -- $P > gpurun_out/rpmc$i.log 2>&1 || echo "pass $i failed"
done
