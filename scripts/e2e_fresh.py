"""The bench's end-to-end leg (bench.end_to_end: generate-reads on the synthetic chr1, files in, /dev/null out) in a
process of its own, to set the bench's in-process number (after the WGS steps) against a fresh command.
--torch: torch's HIP runtime first; --frag GB: that much device memory allocated in 2 GiB pieces and freed first (as
the WGS steps leave the allocator).  One JSON line."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
  argv = sys.argv[1:]
  use_torch = '--torch' in argv
  frag = int(argv[argv.index('--frag') + 1]) if '--frag' in argv else 0
  if use_torch:
    import torch
    torch.empty(1, device='cuda')
  sys.argv = [sys.argv[0]]
  import bench
  from mitty_amd import synth
  from mitty_amd.readmodel import get_read_model
  a = bench.parse()
  seq, recs, _ = synth.genome_regions(synth.genome_contigs(1.0), [0], workers=1)[0]
  _, model = get_read_model(a.model + '.pkl')
  if frag:
    from mitty_amd import _native
    _native.lib()   # the library's runtime (or torch's, loaded first)
    hip = ctypes.CDLL('libamdhip64.so.7')
    ptrs = []
    for _ in range(frag // 2):
      p = ctypes.c_void_p()
      if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(2 << 30)) != 0:
        break
      ptrs.append(p)
    for p in ptrs:
      hip.hipFree(p)
  e = bench.end_to_end(a, seq, recs, model, None)
  print(json.dumps({'torch_first': use_torch, 'frag_gb': frag, 'seconds': round(e['seconds'], 3),
                    'Mtps': round(e['value'] / 1e6, 1), 'split_s': e['split_s'],
                    'output_d2h_ms': (e.get('stages_ms') or {}).get('output_d2h'),
                    'gz_seconds': round(e['gz']['seconds'], 3), 'gz_Mtps': round(e['gz']['value'] / 1e6, 1)}),
        flush=True)


if __name__ == '__main__':
  main()
