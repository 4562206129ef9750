set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/graph_latency.py > gpurun_out/lat_default.log 2>&1 || { tail -20 gpurun_out/lat_default.log; exit 1; }
cat gpurun_out/lat_default.log
timeout -k 10 200 python tools/graph_latency.py --spin > gpurun_out/lat_spin.log 2>&1 || { tail -20 gpurun_out/lat_spin.log; exit 1; }
cat gpurun_out/lat_spin.log
