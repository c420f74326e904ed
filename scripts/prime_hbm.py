"""Allocate most of the GPU's HBM in 1 GiB blocks, write every block (hipMemset), free them, exit: a fresh box's first
touch of its HBM, done by a process of its own (calibration: does the first bench process's slowdown come from it?)."""
import ctypes
import sys
import time


def main():
  gb = int(sys.argv[1]) if len(sys.argv) > 1 else 250
  hip = ctypes.CDLL('libamdhip64.so.7')
  t0 = time.perf_counter()
  ptrs = []
  for _ in range(gb):
    p = ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 30)) != 0:
      break
    hip.hipMemset(p, 0, ctypes.c_size_t(1 << 30))
    ptrs.append(p)
  hip.hipDeviceSynchronize()
  t1 = time.perf_counter()
  for p in ptrs:
    hip.hipFree(p)
  print('primed {} GiB in {:.1f} s'.format(len(ptrs), t1 - t0), flush=True)


if __name__ == '__main__':
  main()
