"""D2H of the FASTQ arenas as the end-to-end writer does it (mh_output_fetch / _async into PinnedBuffer slots), against
torch copies in the same process, to find why the e2e leg moved 17.4 GB at ~28 GB/s while scripts/calib_d2h.py
measured ~56 GB/s.  Prints one JSON line of GB/s per variant."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  # --torch: torch's HIP runtime first (then the library runs on it: one libamdhip64 per process) and torch's own
  # copies measured too; without it the library runs on /opt/rocm's runtime, as in bench.py
  use_torch = '--torch' in sys.argv
  if use_torch:
    import torch
    torch.empty(1, device='cuda')
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  p, passes = _native.read_model_params(150, 30.0)
  L = 60_000_000
  seq = synth.contig(L, 7)
  copies = synth.copies_soa(synth.variants(seq, 8))
  eng = Engine(0)
  out = {}
  try:
    eng.load_region(0, ('1', 0, L), seq)
    units = [(k, 0, k % 2, 1000 + k) for k in range(4)]
    eng.run_units(units, lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'S')
    u1, u2 = eng.ctx.output_size()
    out['arena_bytes'] = [u1, u2]
    CH = 64 << 20
    pins = [[_native.PinnedBuffer(), _native.PinnedBuffer()] for _ in range(2)]
    for s in pins:
      s[0].reserve(CH)
      s[1].reserve(CH)

    def run(name, fn, both=True):
      for rep in range(2):
        eng.ctx.sync()
        t0 = time.perf_counter()
        moved = fn(both)
        dt = time.perf_counter() - t0
      out[name] = round(moved / dt / 1e9, 2)

    def sync_fetch(both):
      moved = 0
      for k, off in enumerate(range(0, min(u1, u2) - CH, CH)):
        eng.ctx.fetch_range_pinned(pins[k % 2], off, CH, off, CH if both else 0)
        moved += CH * (2 if both else 1)
      return moved

    def async_fetch(both):
      moved, pend = 0, None
      for k, off in enumerate(range(0, min(u1, u2) - CH, CH)):
        t, _ = eng.ctx.fetch_range_async(pins[k % 2], off, CH, off, CH if both else 0)
        if pend is not None:
          eng.ctx.fetch_wait(pend)
        pend = t
        moved += CH * (2 if both else 1)
      eng.ctx.fetch_wait(pend)
      return moved

    def async_timed(both):   # as the e2e leg runs it: stage timing on (each fetch is an 'output_d2h' stage)
      eng.ctx.enable_timing(True)
      try:
        return async_fetch(both)
      finally:
        eng.ctx.enable_timing(False)

    def async_writer(both):   # ... and each chunk handed to the two file-writer threads (/dev/null)
      from mitty_amd.lib.fastq_stream import PairWriter
      from mitty_amd.lib.fastq_stream import FastqSink
      sinks = [FastqSink('/dev/null', 1, 1, False), FastqSink('/dev/null', 1, 1, False)]
      pw = PairWriter(sinks)
      moved, pend = 0, None
      try:
        for k, off in enumerate(range(0, min(u1, u2) - CH, CH)):
          pw.wait(k % 2)
          t, (d1, d2) = eng.ctx.fetch_range_async(pins[k % 2], off, CH, off, CH if both else 0)
          if pend is not None:
            eng.ctx.fetch_wait(pend[0])
            pw.submit(*pend[1:])
          pend = (t, k % 2, [d1, d2 if both else None])
          moved += CH * (2 if both else 1)
        eng.ctx.fetch_wait(pend[0])
        pw.submit(*pend[1:])
        pw.close()
      finally:
        for x in sinks:
          x.close()
      return moved

    run('sync_two_files', sync_fetch)
    run('async_two_timed', async_timed)
    run('async_two_writer', async_writer)
    run('sync_one_file', sync_fetch, False)
    run('async_two_files', async_fetch)
    run('async_one_file', async_fetch, False)
    if not use_torch:
      raise StopIteration
    src = torch.empty(4 << 30, dtype=torch.uint8, device='cuda')
    src.fill_(3)
    tp = [torch.empty(CH, dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def torch_copy(both):
      moved = 0
      for k in range(0, (4 << 30) // CH - 1, 2):
        tp[0].copy_(src[k * CH:(k + 1) * CH], non_blocking=True)
        if both:
          tp[1].copy_(src[(k + 1) * CH:(k + 2) * CH], non_blocking=True)
        torch.cuda.synchronize()
        moved += CH * (2 if both else 1)
      return moved

    run('torch_two', torch_copy)
    run('torch_one', torch_copy, False)
    for s in pins:
      s[0].free()
      s[1].free()
  except StopIteration:
    pass
  finally:
    eng.close()
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
