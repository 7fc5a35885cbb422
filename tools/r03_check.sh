# Round-3 GPU session: the -m gpu suite (new north-star / config-1 / config-3 tests first),
# smoke(), then the default bench line (config 2 + dp_train) and the config-1 line.
# Outputs under gpurun_out/; stops at the first step that crashes or times out.
export TMPDIR=/tmp
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests/test_gpu_northstar.py tests/test_gpu_train.py tests/test_gpu_layers.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/${TAG}_new.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 300 python bench.py --alpha > gpurun_out/${TAG}_c1.json 2> gpurun_out/${TAG}_c1.err
