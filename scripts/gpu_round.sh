# One GPU session: every GPU test, smoke(), the headline bench (ENet -> BEV) (with its config-4 DeepLab sub-record).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/round
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > gpurun_out/round/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/round/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/round/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.txt 2>&1 || { cat gpurun_out/round/smoke.txt; exit 1; }
cat gpurun_out/round/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/round/bench.json 2> gpurun_out/round/bench.err || exit 1
echo done
