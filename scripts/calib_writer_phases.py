"""Writer calibration: where k_emit_tiles' time goes, from the DF_PROF/EW_PROF build (make -C mitty_amd/csrc prof):
per 32-template tile, the shader clocks of wave 0's formatting, waves 1-3's gathers, each side's wait at the tile's
barrier, the seam sweep and the chunk sweep (mh_emit.hip EW_PROF).  Units of a synthetic contig (random bases, the
bench's variant density) sampled and emitted by the engine; the second pass alone is counted.  One JSON line."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
SLOTS = ['format_w0', 'gather_w123', 'barrier_w0', 'barrier_w123', 'cr_rows', 'seam_sweep', 'chunk_sweep']


def main():
  os.environ['MH_LIB'] = os.path.join(REPO, 'mitty_amd', '_lib', 'prof', 'libmitty_hip.so')
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  p, _ = _native.read_model_params(150, 30.0)
  L = 60_000_000
  seq = synth.contig(L, 7)
  copies = synth.copies_soa(synth.variants(seq, 8))
  eng = Engine(0)
  buf = (ctypes.c_ulonglong * 16)()
  out = {}
  try:
    eng.load_region(0, ('1', 0, L), seq)
    for rep in range(2):
      eng.ctx.reset_output()
      eng.ctx.sync()
      _native.lib().mh_ew_prof(buf)   # zero
      eng.run_units([(k, 0, k % 2, 1000 + k) for k in range(4)], lambda r, c: copies[c], p, 150, mdl['cum_tlen'],
                    'S')
      eng.ctx.sync()
    _native.lib().mh_ew_prof(buf)
    v = list(buf)
    tiles = max(1, v[7])
    per = {k: v[i] / tiles for i, k in enumerate(SLOTS)}
    per['gather_w123'] /= 3
    per['barrier_w123'] /= 3
    for k in ('cr_rows', 'seam_sweep', 'chunk_sweep'):
      per[k] /= 4   # (every wave)
    out['tiles'] = tiles
    out['clocks_per_tile'] = {k: round(x, 1) for k, x in per.items()}
    out['critical_w0'] = round(per['format_w0'] + per['barrier_w0'] + per['cr_rows'] + per['seam_sweep'] +
                               per['chunk_sweep'], 1)
  finally:
    eng.close()
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  main()
