"""Device deflate calibration: where k_bgzf_blocks' time goes.  FASTQ made by the engine on a synthetic contig (random
bases: the bench's chr1 data, not the repeated golden file) is deflated from the arena (mh_output_bgzf_range), timed
per call; with --prof the library is the DF_PROF build (make -C mitty_amd/csrc prof) and the per-phase shader-clock
sums of every wave's lane 0 are printed as fractions (mh_deflate.hip: staging, CRC, parse, count, keep, hash-in,
codes, token load, encode, end), with parse steps and matches per slice.  One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PHASES = ['staging', 'crc', 'parse', 'count', 'keep', 'hash_in', 'codes', 'tok_load', 'encode', 'end']


def main():
  prof = '--prof' in sys.argv
  if prof:
    os.environ['MH_LIB'] = os.path.join(REPO, 'mitty_amd', '_lib', 'prof', 'libmitty_hip.so')
  import ctypes
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  p, passes = _native.read_model_params(150, 30.0)
  L = 30_000_000
  seq = synth.contig(L, 7)
  copies = synth.copies_soa(synth.variants(seq, 8))
  eng = Engine(0)
  out = {'prof_build': prof}
  try:
    eng.load_region(0, ('1', 0, L), seq)
    eng.run_units([(k, 0, k % 2, 1000 + k) for k in range(4)], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'S')
    u1, _ = eng.ctx.output_size()
    n = min(u1, 1 << 30)
    pin = _native.PinnedBuffer()
    ts = []
    z = b''
    for rep in range(3):
      eng.ctx.sync()
      if prof and rep == 2:
        buf = (ctypes.c_ulonglong * 16)()
        _native.lib().mh_df_prof(buf)   # zero: the last call alone
      t0 = time.perf_counter()
      z = eng.ctx.bgzf_range(0, 0, n, pin)
      ts.append(time.perf_counter() - t0)
    out.update(input_bytes=n, output_bytes=len(z), ratio=round(n / len(z), 3), seconds=[round(t, 4) for t in ts],
               GBps_incl_d2h=round(n / min(ts) / 1e9, 2))
    if prof:
      buf = (ctypes.c_ulonglong * 16)()
      _native.lib().mh_df_prof(buf)
      v = list(buf)
      tot = sum(v[:10])
      out['phase_frac'] = {k: round(v[i] / tot, 4) for i, k in enumerate(PHASES)}
      waves = max(1, v[12])
      out['clocks_per_slice'] = round(tot / waves)
      out['steps_per_slice'] = round(v[10] / waves, 1)
      out['matches_per_slice'] = round(v[11] / waves, 1)
      out['clocks_per_step'] = {k: round(v[i] / max(1, v[10]), 1) for i, k in enumerate(PHASES) if 2 <= i <= 8}
    pin.free()
  finally:
    eng.close()
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
