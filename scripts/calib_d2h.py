"""D2H calibration for the end-to-end leg: device arena -> page-locked host staging, as mh_output_fetch does it
(hipMemcpyAsync on one or two streams), for several chunk sizes.  Prints one JSON line:
{"one_stream": {chunk_MiB: GB/s}, "two_streams": {...}, "sdma": env HSA_ENABLE_SDMA}.
Run it twice (default and HSA_ENABLE_SDMA=0: blit-kernel copies instead of the DMA engines) to compare."""
import json
import os
import time

import torch


def main():
  dev = torch.device('cuda:0')
  total = 4 << 30
  src = torch.empty(total, dtype=torch.uint8, device=dev)
  src.fill_(7)
  s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
  out = {'sdma': os.environ.get('HSA_ENABLE_SDMA', 'default'), 'one_stream': {}, 'two_streams': {}}
  for mib in (16, 64, 256):
    n = mib << 20
    pins = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    for mode in ('one_stream', 'two_streams'):
      for rep in range(2):   # the first pass warms the mappings
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        moved = 0
        for off in range(0, total - 2 * n + 1, 2 * n):
          if mode == 'one_stream':
            with torch.cuda.stream(s1):
              pins[0].copy_(src[off:off + n], non_blocking=True)
              pins[1].copy_(src[off + n:off + 2 * n], non_blocking=True)
            s1.synchronize()
          else:
            with torch.cuda.stream(s1):
              pins[0].copy_(src[off:off + n], non_blocking=True)
            with torch.cuda.stream(s2):
              pins[1].copy_(src[off + n:off + 2 * n], non_blocking=True)
            s1.synchronize()
            s2.synchronize()
          moved += 2 * n
        dt = time.perf_counter() - t0
      out[mode][mib] = round(moved / dt / 1e9, 2)
    del pins
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
