"""HBM bandwidth probe: write-only fill and read+write copy of FASTQ-arena-sized buffers (torch kernels)."""
import torch

n = 4_350_000_000
a = torch.empty(n, dtype=torch.uint8, device='cuda')
b = torch.empty(n, dtype=torch.uint8, device='cuda')
a.fill_(1)
b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn, nbytes in (('fill', lambda: a.fill_(126), n), ('copy', lambda: b.copy_(a), 2 * n),
                         ('sum', lambda: a.view(torch.int64).sum(), n)):
  fn()
  torch.cuda.synchronize()
  e0.record()
  for _ in range(5):
    fn()
  e1.record()
  torch.cuda.synchronize()
  ms = e0.elapsed_time(e1) / 5
  print('{:5s} {:8.3f} ms  {:7.1f} GB/s'.format(name, ms, nbytes / ms / 1e6), flush=True)
