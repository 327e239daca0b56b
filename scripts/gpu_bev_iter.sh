# ENet/BEV parity tests + the headline bench line (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bev
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bev/pytest.log 2>&1 || { tail -30 gpurun_out/bev/pytest.log; exit 1; }
tail -2 gpurun_out/bev/pytest.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bev/bench.json 2> gpurun_out/bev/bench.err || exit 1
echo done
