set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1 || { tail -30 gpurun_out/g1_pytest.log; exit 1; }
tail -3 gpurun_out/g1_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1_smoke.log 2>&1 || { tail -5 gpurun_out/g1_smoke.log; exit 1; }
tail -1 gpurun_out/g1_smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/g1_bench20_$i.log 2>&1 || { tail -20 gpurun_out/g1_bench20_$i.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/g1_bench20_$i.log').read().strip().splitlines()[-1]); r=d['roofline']
print('value', d['value']/1e6, 'ms', d['ms_per_step'], 'kern', r['kernel_ms'], 'eager', d['eager_loop']['ms_per_step'], d['config']['launch'])"
done
timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/g1_bench1000.log 2>&1 || { tail -20 gpurun_out/g1_bench1000.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/g1_bench1000.log').read().strip().splitlines()[-1]); r=d['roofline']
print('value', d['value']/1e6, 'ms', d['ms_per_step'], 'kern', r['kernel_ms'], 'eager', d['eager_loop']['ms_per_step'])"
