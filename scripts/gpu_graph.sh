# HIP-graph replay of the bench step: parity test, then eager vs captured bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/graph
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "captured or multistream" --timeout 120 --timeout-method thread > gpurun_out/graph/pytest.log 2>&1 || { tail -30 gpurun_out/graph/pytest.log; exit 1; }
tail -3 gpurun_out/graph/pytest.log
for g in 0 1 0 1; do
  timeout -k 10 120 python bench.py --graph $g --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/graph/g$g.json 2> gpurun_out/graph/g$g.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/graph/g$g.json')); print('graph', $g, d['value'], d['ms_per_step'])"
done
for s in 1 4; do
  timeout -k 10 120 python bench.py --graph 1 --streams $s --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/graph/s$s.json 2> gpurun_out/graph/s$s.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/graph/s$s.json')); print('graph streams', $s, d['value'], d['ms_per_step'])"
done
echo done
