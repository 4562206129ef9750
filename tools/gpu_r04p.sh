# the blob header passed by value in the kernel arguments against the previous
# build (brax_amd/_lib_prev): Ant / Humanoid / HalfCheetah rollouts and the
# MULTI kernel's states bit for bit, then the A/B bench (tools/ab_libs.sh)
set -o pipefail
mkdir -p gpurun_out/ab_mu; export TMPDIR=/tmp
for m in noinfo info; do
  BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 120 python -u tools/multi_traffic.py $m 36 gpurun_out/ab_mu/prev_$m.npz > gpurun_out/ab_mu/run.log 2>&1 || exit 3
  timeout -k 10 120 python -u tools/multi_traffic.py $m 36 gpurun_out/ab_mu/new_$m.npz >> gpurun_out/ab_mu/run.log 2>&1 || exit 3
done
python - <<'PY' > gpurun_out/ab_mu/bitcmp_hdr.log 2>&1
import numpy as np
ok = True
for m in ('noinfo', 'info'):
  a = np.load(f'gpurun_out/ab_mu/prev_{m}.npz'); b = np.load(f'gpurun_out/ab_mu/new_{m}.npz')
  for k in a.files:
    eq = np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)); ok &= eq
    print('multi', m, k, 'bit-identical' if eq else 'DIFFERS')
print('MULTI ALL BIT-IDENTICAL' if ok else 'MULTI MISMATCH')
PY
cat gpurun_out/ab_mu/bitcmp_hdr.log | tail -1
bash tools/gpu_ab_prev.sh hdr
