# Round-end check on one box: the full -m gpu suite, smoke(), then the bench lines of
# tools/round_lines.sh.  GPU only; outputs under gpurun_out/.
set -e
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final_gputest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
bash tools/round_lines.sh
