#!/bin/bash
# PMC counters of the polyphase weight-gradient kernel (64^2 B16 shape), one pass each
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_ws2a -o a -- python3 $R/tools/wgrad_probe.py --cin 192 --cout 192 --hw 64 --ksize 5 --stride 2 --batch 16 --iters 3 > $R/gpurun_out/pmc_ws2a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/pmc_ws2b -o b -- python3 $R/tools/wgrad_probe.py --cin 192 --cout 192 --hw 64 --ksize 5 --stride 2 --batch 16 --iters 3 > $R/gpurun_out/pmc_ws2b.log 2>&1
cd $R
python3 tools/pmc_db.py gpurun_out/pmc_ws2a/a_results.db --match wgrad_s2 > gpurun_out/pmc_ws2.txt
python3 tools/pmc_db.py gpurun_out/pmc_ws2b/b_results.db --match wgrad_s2 >> gpurun_out/pmc_ws2.txt
rm -rf gpurun_out/pmc_ws2a gpurun_out/pmc_ws2b
timeout -k 10 60 python -u tools/wgrad_probe.py --cin 192 --cout 192 --hw 64 --ksize 5 --stride 2 --batch 16 --iters 20 >> gpurun_out/pmc_ws2.txt 2>&1
timeout -k 10 60 python -u tools/wgrad_probe.py --cin 192 --cout 192 --hw 32 --ksize 5 --stride 2 --batch 16 --iters 20 >> gpurun_out/pmc_ws2.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "wgrad" >> gpurun_out/pmc_ws2.txt 2>&1
timeout -k 10 300 python -u bench.py --train --steps 10 --no-cpu-baseline > gpurun_out/r04_c3_ws2b.json 2> gpurun_out/r04_c3_ws2b.err
