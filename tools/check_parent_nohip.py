"""`bench.py --gpus N` parent on a box with fewer GPUs: the RCCL spawn branch
must refuse (rc 2) without initialising HIP in the parent. Runs bench.main's
spawn decision in this process, then lists this process's open /dev/kfd
descriptors (HIP's init opens it) and what the GPU count came from.

    python tools/check_parent_nohip.py 2
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def kfd_fds():
  out = []
  for fd in os.listdir('/proc/self/fd'):
    try:
      if os.readlink(f'/proc/self/fd/{fd}').startswith('/dev/kfd'):
        out.append(fd)
    except OSError:
      pass
  return out


def main():
  n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
  import bench
  env = {k: os.environ.get(k) for k in ('HIP_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES',
                                        'CUDA_VISIBLE_DEVICES')}
  print('visibility env', env, 'visible_gpus()', bench.visible_gpus(os.environ),
        'kfd topology GPU nodes', bench.visible_gpus({}), flush=True)
  rc = bench.spawn_ranks(n, ['--gpus', str(n)])
  fds = kfd_fds()
  print('spawn_ranks rc', rc, 'parent /dev/kfd fds', fds, flush=True)
  ok = rc == 2 and not fds
  print('OK' if ok else 'FAIL')
  sys.exit(0 if ok else 1)


if __name__ == '__main__':
  main()
