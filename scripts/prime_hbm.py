"""First touch of a GPU's HBM by a process of its own: most of the free memory allocated in 1 GiB blocks, written
(hipMemset) and freed.  On a fresh box the first process to use the HBM ran ~13 % slow throughout (the bench's first
process: 1.38-1.47 G templates/s against 1.58-1.61 for the next; after this, 1.611 — DESIGN.md "Performance").
bench.py runs it before it touches the GPU.  usage: prime_hbm.py [DEVICE] [KEEP_FREE_GIB] [WRITE (1)]"""
import ctypes
import sys
import time


def main():
  dev = int(sys.argv[1]) if len(sys.argv) > 1 else 0
  keep = int(sys.argv[2]) if len(sys.argv) > 2 else 8
  write = (sys.argv[3] if len(sys.argv) > 3 else '1') != '0'   # 0: allocate and free only
  hip = ctypes.CDLL('libamdhip64.so.7')
  if hip.hipSetDevice(dev) != 0:
    print('prime_hbm: no device {}'.format(dev), flush=True)
    return 0
  free, total = ctypes.c_size_t(), ctypes.c_size_t()
  hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
  n = max(0, int(free.value >> 30) - keep)
  t0 = time.perf_counter()
  ptrs = []
  for _ in range(n):
    p = ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30)) != 0:
      break
    if write:
      hip.hipMemset(p, 0, ctypes.c_size_t(1 << 30))
    ptrs.append(p)
  hip.hipDeviceSynchronize()
  for p in ptrs:
    hip.hipFree(p)
  print('prime_hbm: device {}: {} GiB written in {:.1f} s'.format(dev, len(ptrs), time.perf_counter() - t0),
        flush=True)
  return 0


if __name__ == '__main__':
  sys.exit(main())
