# the MULTI kernel's lane-consecutive QP load/store against the previous build
# (brax_amd/_lib_prev): the final states bit for bit (Info off and on, cutoff
# 0 and 36), its time and HBM traffic with Info off (separate PMC passes),
# then the parity tests (binding nearest-realisation gates)
set -o pipefail
mkdir -p gpurun_out/ab_mu; export TMPDIR=/tmp
for m in noinfo info; do for c in 0 36; do
  BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 120 python -u tools/multi_traffic.py $m $c gpurun_out/ab_mu/prev_${m}_$c.npz > gpurun_out/ab_mu/run.log 2>&1 || exit 3
  timeout -k 10 120 python -u tools/multi_traffic.py $m $c gpurun_out/ab_mu/new_${m}_$c.npz >> gpurun_out/ab_mu/run.log 2>&1 || exit 3
done; done
python - <<'PY' > gpurun_out/ab_mu/bitcmp.log 2>&1
import numpy as np
ok = True
for m in ('noinfo', 'info'):
  for c in (0, 36):
    a = np.load(f'gpurun_out/ab_mu/prev_{m}_{c}.npz'); b = np.load(f'gpurun_out/ab_mu/new_{m}_{c}.npz')
    for k in a.files:
      eq = np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))
      ok &= eq
      print(m, c, k, a[k].shape, 'bit-identical' if eq else 'DIFFERS')
print('ALL BIT-IDENTICAL' if ok else 'MISMATCH')
PY
cat gpurun_out/ab_mu/bitcmp.log
for v in prev new; do
  if [ $v = prev ]; then L=brax_amd/_lib_prev/libbrax_amd.so; else L=brax_amd/_lib/libbrax_amd.so; fi
  BRAX_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mt2_$v/trace -o run --output-format csv -- python3 tools/multi_traffic.py noinfo > gpurun_out/mt2_$v.trace.log 2>&1 || exit 5
  BRAX_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/mt2_$v/fetch -o run --output-format csv -- python3 tools/multi_traffic.py noinfo > gpurun_out/mt2_$v.fetch.log 2>&1 || exit 6
  BRAX_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/mt2_$v/write -o run --output-format csv -- python3 tools/multi_traffic.py noinfo > gpurun_out/mt2_$v.write.log 2>&1 || exit 7
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/near2.log 2>&1
r=$?; cp gpurun_out/parity_margins.json gpurun_out/parity_margins_near2.json; tail -3 gpurun_out/near2.log
exit $r
