# the parity tests with the nearest-realisation records, then the MULTI
# kernel's HBM traffic with and without the contact Info (separate PMC passes)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/near.log 2>&1
r=$?; cp gpurun_out/parity_margins.json gpurun_out/parity_margins_near.json; tail -2 gpurun_out/near.log
[ $r -le 1 ] || exit $r
for m in noinfo info; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mt_$m/trace -o run --output-format csv -- python3 tools/multi_traffic.py $m > gpurun_out/mt_$m.trace.log 2>&1 || exit 5
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/mt_$m/fetch -o run --output-format csv -- python3 tools/multi_traffic.py $m > gpurun_out/mt_$m.fetch.log 2>&1 || exit 6
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/mt_$m/write -o run --output-format csv -- python3 tools/multi_traffic.py $m > gpurun_out/mt_$m.write.log 2>&1 || exit 7
done
exit $r
