"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors and the CPU oracle.

Bar: bit-exact (integer / byte work).  Sizes: golden fixtures (reference-captured), oracle comparisons up to a few
Mbp, and size-independent properties at larger sizes.
"""
import gzip
import os
import re

import numpy as np
import pytest

from tests import golden_io as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def native():
  from mitty_amd import _native
  if _native.device_count() == 0:
    pytest.fail('no HIP device: GPU tests must run on an MI355X')
  return _native


@pytest.fixture(scope='module')
def ctx(native):
  c = native.Context(0)
  yield c
  c.close()


# ---- template sampling (illumina.generate_reads) ---------------------------------------------------------------
def test_templates_golden(native):
  from mitty_amd.simulation import illumina
  t = G.templates()
  keys = sorted({k.rsplit('|', 1)[0] for k in t.files})
  assert len(keys) == 12
  for key in keys:
    m, seed, p_min, p_max = key.split('|')
    rm = illumina.read_model_params(G.model(m), 30.0)
    r = illumina.generate_reads(rm, int(p_min), int(p_max), int(seed))
    assert np.array_equal(r[0]['file_order'], t[key + '|fo0']), key
    assert np.array_equal(r[0]['pos'], t[key + '|pos0']), key
    assert np.array_equal(r[1]['pos'], t[key + '|pos1']), key
    assert r[0]['file_order'].dtype == np.int8 and r[0]['pos'].dtype == np.int64 and r[0]['len'].dtype == np.uint32
    assert np.array_equal(r[1]['file_order'], 1 - t[key + '|fo0'])


@pytest.mark.parametrize('span,seed', [(3_000_000, 7), (20_000_000, 99), (61_000, 4294967295), (41, 3), (1, 5)])
@pytest.mark.parametrize('model', G.MODELS)
def test_templates_vs_oracle(native, model, span, seed):
  """Larger spans than the golden set (exercise the shuffle decode / permutation at millions of draws)."""
  from mitty_amd.simulation import illumina
  from oracle import oracle as O
  mdl = G.model(model)
  rm = illumina.read_model_params(mdl, 30.0)
  r = illumina.generate_reads(rm, 1000, 1000 + span, seed)
  fo, p0, p1 = O.generate_templates(rm['p'], int(rm['rlen']), mdl['cum_tlen'], 1000, 1000 + span, seed)
  assert np.array_equal(r[0]['file_order'], fo)
  assert np.array_equal(r[0]['pos'], p0)
  assert np.array_equal(r[1]['pos'], p1)


DEC_MODES = {'sequential': 1, 'force_fixup': 2, 'force_geo': 4, 'all': 7}


@pytest.mark.parametrize('mode', sorted(DEC_MODES))
def test_templates_forced_fallbacks_vs_oracle(native, mode):
  """The exact fallbacks that keep the templates bit-exact when the fast path cannot, each forced through the C ABI
  (mh_set_decode_mode) on a 12 Mbp unit (illumina.py:66-76): the block-sequential decode (k_shuffle_decode2), the
  single-stream decode + per-unit permutation fix-up (k_shuffle_decode, finish_unit), and every geometric draw
  recomputed by the host libm (finish_unit's exact path).  Array-equal to the oracle; the fix-up modes must have run."""
  from mitty_amd.simulation import illumina
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  rm = illumina.read_model_params(mdl, 30.0)
  ctx = illumina.device_context()
  fix0 = ctx.fixup_count()
  ctx.set_decode_mode(DEC_MODES[mode])
  try:
    r = illumina.generate_reads(rm, 500, 500 + 12_000_000, 2024)
  finally:
    ctx.set_decode_mode(0)
  fixed = ctx.fixup_count() - fix0
  fo, p0, p1 = O.generate_templates(rm['p'], int(rm['rlen']), mdl['cum_tlen'], 500, 500 + 12_000_000, 2024)
  assert np.array_equal(r[0]['pos'], p0) and np.array_equal(r[1]['pos'], p1)
  assert np.array_equal(r[0]['file_order'], fo)
  assert fixed == (0 if mode == 'sequential' else 1)


@pytest.mark.parametrize('mode', sorted(DEC_MODES))
def test_batched_units_forced_fallbacks_vs_oracle(native, mode):
  """The same forced fallbacks on a batched multi-unit job (the batch permutation, the asynchronous per-unit tails
  resolved by the emission): every unit's FASTQ equal to the oracle's, every unit redone by the fix-up modes."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 30.0)
  L = 3_000_000
  seq = synth.contig(L, 71)
  copies = synth.copies_soa(synth.variants(seq, 72))
  units = _native.work_units(5, [2], passes)
  eng = Engine(0)
  try:
    eng.ctx.set_decode_mode(DEC_MODES[mode])
    eng.load_region(0, ('7', 0, L), seq)
    res = eng.run_units([(ps, ri, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)], lambda r, c: copies[c], p,
                        150, mdl['cum_tlen'], 'SYN')
    d1, d2 = eng.ctx.fetch_output()
    fix = eng.ctx.fixup_count()
  finally:
    eng.close()
  o1, o2 = [], []
  for ps, (ri, cpy, sd) in enumerate(units):
    k, b1, b2 = O.generate_unit_soa(seq, 0, copies[cpy], p, 150, mdl['cum_tlen'], sd, 'SYN:0:{}'.format(ps), '7', cpy)
    assert res[ps][1] == k and k > 1000
    o1.append(b1)
    o2.append(b2)
  G.check_same(d1, b''.join(o1))
  G.check_same(d2, b''.join(o2))
  assert fix == (0 if mode == 'sequential' else len(units))


def test_templates_high_coverage_vs_oracle(native):
  """p close to 0.1 (coverage 60, 2x150 -> passes 4, p = 0.025 ... use a direct p) and tiny rlen."""
  from mitty_amd.simulation import illumina
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  for p in (0.1, 0.0999, 0.05, 0.4, 0.9):
    rm = {'p': p, 'rlen': 30, 'cum_tlen': mdl['cum_tlen']}
    r = illumina.generate_reads(rm, 0, 400_000, 11)
    fo, p0, p1 = O.generate_templates(p, 30, mdl['cum_tlen'], 0, 400_000, 11)
    assert np.array_equal(r[0]['pos'], p0) and np.array_equal(r[1]['pos'], p1)
    assert np.array_equal(r[0]['file_order'], fo)


def test_seed_out_of_range(native):
  from mitty_amd.simulation import illumina
  rm = illumina.read_model_params(G.model('hiseq-X-v2.5-Garvan'), 30.0)
  with pytest.raises(ValueError):
    illumina.generate_reads(rm, 0, 1000, 1 << 32)
  with pytest.raises(ValueError):
    illumina.generate_reads(rm, 0, 1000, -1)


# ---- splice / read derivation (rpc) ----------------------------------------------------------------------------
def _seqs():
  from mitty_amd.lib import fasta
  return {'syn': fasta.read_fasta(G.path('data/syn.fa')), 'tiny': fasta.read_fasta(G.path('data/tiny.fasta'))}


def test_node_lists_golden(native):
  from mitty_amd.lib import vcfio
  from mitty_amd.simulation import rpc
  seqs = _seqs()
  for key, d in G.load_json('nodes.json').items():
    tag = key.split('|')[0]
    chrom, s0, e = d['region']
    vl = [vcfio.Variant(*v) for v in d['variants']]
    nodes = rpc.create_node_list(seqs[tag][chrom][s0:e].decode(), s0 + 1, vl)
    assert [list(n.tuple()) for n in nodes] == d['nodes'], key


def test_reads_golden(native):
  from mitty_amd.lib import vcfio
  from mitty_amd.simulation import rpc
  seqs = _seqs()
  nodes_g = G.load_json('nodes.json')
  reads = G.load_json('reads.json.gz')
  total = 0
  for key, rows in reads.items():
    d = nodes_g[key]
    tag = key.split('|')[0]
    chrom, s0, e = d['region']
    nodes = rpc.create_node_list(seqs[tag][chrom][s0:e].decode(), s0 + 1, [vcfio.Variant(*v) for v in d['variants']])
    pl = [r[0] for r in rows]
    ll = [r[1] for r in rows]
    got, n0, n1 = rpc.generate_reads_batch(pl, ll, nodes)
    for r, g, a, b in zip(rows, got, n0, n1):
      assert [r[2], r[3]] == [int(a), int(b)], (key, r[:2])
      assert [r[4], r[5], r[6], r[7]] == [g[0], g[1], g[2], g[3]], (key, r[:2])
    total += len(rows)
  assert total > 5000


def test_reference_rpc_known_answers(native):
  """mitty/test/simulation/test_rpc.py:111-180 restated against the device path."""
  from mitty_amd.lib import vcfio
  from mitty_amd.simulation import rpc
  ref_seq = open(G.path('data/tiny.fasta')).readlines()[1]
  vdf = vcfio.load_variant_file(G.path('data/tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))
  nodes = rpc.create_node_list(ref_seq, 1, vdf[0]['v'][1])
  assert len(nodes) == 9
  assert nodes[0] == (1, 1, '=', 4, 'ATGA', None)
  assert nodes[3] == (9, 9, 'I', 3, 'TTT', 3)
  assert nodes[5] == (14, 14, 'D', 2, '', -2)
  assert nodes[7] == (21, 25, 'D', 4, '', -4)
  assert nodes[8] == (22, 25, '=', 1, 'C', None)
  nse = rpc.get_begin_end_nodes(np.arange(1, 16), 10, nodes)
  assert nse[0].tolist() == [0, 0, 0, 0, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 6]
  assert nse[1].tolist() == [3, 3, 4, 4, 4, 6, 6, 6, 6, 6, 6, 6, 8, 8, 8]
  assert rpc.generate_read(1, 10, 0, 3, nodes) == (1, '4=1X3=2I', [0, 3], 'ATGATGTATT')
  assert rpc.generate_read(6, 10, 2, 6, nodes) == (6, '3=3I3=2D1=', [3, -2], 'GTATTTTCCG')
  assert rpc.generate_read(10, 10, 3, 6, nodes) == (9, '2I3=2D5=', [3, -2], 'TTTCCGGAGG')
  assert rpc.generate_read(13, 10, 4, 8, nodes) == (10, '2=2D7=4D1=', [-2, -4], 'CCGGAGGCGC')
  assert rpc.generate_read(15, 8, 6, 8, nodes) == (14, '7=4D1=', [-4], 'GGAGGCGC')
  assert rpc.generate_read(9, 2, 3, 3, nodes) == (8, '>0:2I', [3], 'TT')
  nodes0 = rpc.create_node_list(ref_seq, 1, vdf[0]['v'][0])
  assert rpc.generate_read(5, 10, 0, 1, nodes0) == (5, '9=1X', [0], 'CGTATCCAAT')
  assert rpc.generate_read(6, 10, 0, 2, nodes0) == (6, '8=1X1=', [0], 'GTATCCAATG')


def test_survey_edge_cases(native):
  """SURVEY.md Appendix B1-B5 node-list quirks."""
  from mitty_amd.lib.vcfio import Variant
  from mitty_amd.simulation import rpc
  ref = 'ACGTACGTAC' * 3
  nodes = rpc.create_node_list(ref, 1, [Variant(27, 'CGTACG', 'C', 'D', 5)])           # B1
  assert [n.tuple()[:4] for n in nodes] == [(1, 1, '=', 27), (27, 33, 'D', 5)]
  ref = 'ACGTA' + 'C' * 25
  nodes = rpc.create_node_list(ref, 1, [Variant(5, 'A', 'A' + 'T' * 20, 'I', 20)])     # B2
  assert rpc.generate_read(6, 5, 1, 1, nodes) == (5, '>0:5I', [20], 'TTTTT')
  assert rpc.generate_read(8, 5, 1, 1, nodes) == (5, '>2:5I', [20], 'TTTTT')
  assert rpc.generate_read(3, 5, 0, 1, nodes) == (3, '3=2I', [20], 'GTATT')
  assert rpc.generate_read(20, 8, 1, 2, nodes) == (6, '6I2=', [20], 'TTTTTTCC')
  ref = 'ACGTACGTACGTACGTACGTACGTAC'
  vl = [Variant(5, 'ACGT', 'A', 'D', 3), Variant(6, 'C', 'T', 'X', 0), Variant(9, 'A', 'T', 'X', 0),
        Variant(9, 'A', 'AG', 'I', 1)]                                                       # B3
  nodes = rpc.create_node_list(ref, 1, vl)
  assert [n.tuple()[:4] for n in nodes] == [(1, 1, '=', 5), (5, 9, 'D', 3), (6, 9, 'X', 1), (7, 10, '=', 17)]


# ---- end to end --------------------------------------------------------------------------------------------------
@pytest.mark.parametrize('model', G.MODELS)
def test_e2e_fastq_byte_identical_to_reference(native, model, tmp_path):
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  c = G.load_json('e2e_config.json')[model]
  mod, mdl = get_read_model(model + '.pkl')
  f1, f2 = str(tmp_path / 'r1.fq'), str(tmp_path / 'r2.fq')
  readgenerate.process_multi_threaded(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], f1, f2, threads=2, seed=c['seed'])
  G.check_same(open(f1, 'rb').read(), G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)))
  G.check_same(open(f2, 'rb').read(), G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model)))


def test_e2e_single_file_and_cli(native, tmp_path):
  """--fastq2 omitted: file 1 only (readgenerate.py:244-245), through the click CLI."""
  from click.testing import CliRunner
  from mitty_amd.cli import cli
  c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
  f1 = str(tmp_path / 'r1.fq')
  res = CliRunner().invoke(cli, ['generate-reads', G.path(c['fasta']), G.path(c['vcf']), c['sample'],
                                 G.path(c['bed']), 'hiseq-X-v2.5-Garvan.pkl', str(c['coverage']), str(c['seed']), f1])
  assert res.exit_code == 0, res.output + repr(res.exception)
  G.check_same(open(f1, 'rb').read(), G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz'))


def _lockstep_reader(f1, f2):
  """A consumer of a FIFO pair that alternates record by record (pysam.FastxFile zip, readcorrupt.py:49-53)."""
  import threading
  got = ([], [])

  def run():
    with open(f1, 'rb') as a, open(f2, 'rb') as b:
      while True:
        x = b''.join(a.readline() for _ in range(4))
        y = b''.join(b.readline() for _ in range(4))
        if not x and not y:
          return
        got[0].append(x)
        got[1].append(y)
  t = threading.Thread(target=run, daemon=True)
  t.start()
  return t, got


def _fifo_producer(path, data):
  import threading
  def run():
    with open(path, 'wb') as fp:   # one open, as `tee > tf1` does
      fp.write(data[:1])
      fp.flush()
      fp.write(data[1:])
  t = threading.Thread(target=run, daemon=True)
  t.start()
  return t


@pytest.mark.timeout(120)
def test_generate_reads_into_fifos_and_gz(native, tmp_path):
  """generate-reads writing both files into FIFOs read in lockstep (examples/reads/run.sh:13-16), with small flushes
  so several pieces cross the pipes; then '.gz' names: BGZF files that decompress to the golden bytes."""
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  model = '1kg-pcr-free'
  c = G.load_json('e2e_config.json')[model]
  mod, mdl = get_read_model(model + '.pkl')
  f1, f2 = str(tmp_path / 'tf1'), str(tmp_path / 'tf2')
  os.mkfifo(f1)
  os.mkfifo(f2)
  t, got = _lockstep_reader(f1, f2)
  readgenerate.process_multi_threaded(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], f1, f2, seed=c['seed'], flush_bytes=50_000)
  t.join(60)
  G.check_same(b''.join(got[0]), G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)))
  G.check_same(b''.join(got[1]), G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model)))
  z1, z2 = str(tmp_path / 'r1.fq.gz'), str(tmp_path / 'r2.fq.gz')
  readgenerate.process_multi_threaded(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], z1, z2, seed=c['seed'], flush_bytes=50_000)
  for z, k in ((z1, 1), (z2, 2)):
    raw = open(z, 'rb').read()
    assert raw[:4] == b'\x1f\x8b\x08\x04' and raw[-28:] == bytes.fromhex(
      '1f8b08040000000000ff0600424302001b0003000000000000000000')   # BGZF blocks + EOF marker
    G.check_same(gzip.decompress(raw), G.fastq_bytes('e2e_{}.r{}.fq.gz'.format(model, k)))


@pytest.mark.timeout(120)
def test_corrupt_reads_fifo_in_fifo_out(native, tmp_path):
  """corrupt-reads --rng mitty with both inputs on single-open FIFO producers (gzip bytes, like `<(cat < tf1)` of a
  gzip stream) and both outputs on FIFOs read in lockstep: byte-identical to the reference's processes=1 output."""
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readcorrupt
  model = 'hiseq-X-v2.5-Garvan'
  mod, mdl = get_read_model(model + '.pkl')
  fi1, fi2, fo1, fo2 = (str(tmp_path / n) for n in ('i1', 'i2', 'o1', 'o2'))
  for f in (fi1, fi2, fo1, fo2):
    os.mkfifo(f)
  p1 = _fifo_producer(fi1, open(G.path('corrupt_in_{}.r1.fq.gz'.format(model)), 'rb').read())
  p2 = _fifo_producer(fi2, open(G.path('corrupt_in_{}.r2.fq.gz'.format(model)), 'rb').read())
  t, got = _lockstep_reader(fo1, fo2)
  readcorrupt.multi_process(mod, mdl, fi1, fo1, fi2, fo2, processes=1, seed=7, chunk_bytes=3001,
                            flush_bytes=20_000)
  p1.join(30)
  p2.join(30)
  t.join(60)
  G.check_same(b''.join(got[0]), G.fastq_bytes('corrupt_{}.r1.fq.gz'.format(model)), 'corrupt file 1')
  G.check_same(b''.join(got[1]), G.fastq_bytes('corrupt_{}.r2.fq.gz'.format(model)), 'corrupt file 2')


def _unit_vs_oracle(length, seed, model, n_seed=1, rate=1.3e-3, start0=0, cpys=(0, 1), emit_mode=0):
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model(model)
  p, _ = _native.read_model_params(mdl['mean_rlen'], 30.0)
  seq = synth.contig(length, n_seed)
  recs = synth.variants(seq, n_seed + 1, rate=rate)
  copies = synth.copies_soa(recs, start0, length)
  ref = seq[start0:]
  eng = Engine(0)
  eng.ctx.set_emit_mode(emit_mode)
  try:
    eng.load_region(0, ('7', start0, length), ref)
    for cpy in cpys:
      eng.ctx.reset_output()
      n, kept, b1, b2 = eng.run_unit(3, 0, cpy, seed + cpy, copies[cpy], p, mdl['mean_rlen'], mdl['cum_tlen'], 'SYN')
      d1, d2 = eng.ctx.fetch_output()
      k, o1, o2 = O.generate_unit_soa(ref, start0, copies[cpy], p, int(mdl['mean_rlen']), mdl['cum_tlen'], seed + cpy,
                                      'SYN:0:3', '7', cpy)
      assert kept == k
      G.check_same(d1, o1, 'file 1 differs (copy {})'.format(cpy))
      G.check_same(d2, o2, 'file 2 differs (copy {})'.format(cpy))
  finally:
    eng.close()
  return kept


@pytest.mark.parametrize('emit_mode', [0, 1])
@pytest.mark.parametrize('model', G.MODELS)
def test_unit_vs_oracle_2mbp(native, model, emit_mode):
  assert _unit_vs_oracle(2_000_000, 7, model, emit_mode=emit_mode) > 10000


@pytest.mark.parametrize('emit_mode', [0, 1])
def test_unit_vs_oracle_dense_variants_offset_region(native, emit_mode):
  _unit_vs_oracle(1_500_000, 4000000000, 'hiseq-X-v2.5-Garvan', n_seed=5, rate=8e-3, start0=123_457,
                  emit_mode=emit_mode)


def test_unit_vs_oracle_very_dense_slot_overflow(native):
  """~1 variant per 8 bp: some qnames exceed the 256-byte slot, the unit falls back to the LDS-image writer."""
  _unit_vs_oracle(300_000, 11, '1kg-pcr-free', n_seed=13, rate=0.12, cpys=(0,))


def test_unit_vs_oracle_no_variants(native):
  _unit_vs_oracle(600_000, 1, '1kg-pcr-free', n_seed=9, rate=0.0)


@pytest.mark.parametrize('emit_mode', [0, 1])
def test_unit_vs_oracle_nine_digit_positions(native, emit_mode):
  """A 2 Mbp region starting at 150,000,000 of a 152 Mbp contig: every POS has 9 digits (both writers)."""
  assert _unit_vs_oracle(152_000_000, 8, '1kg-pcr-free', n_seed=17, start0=150_000_000, cpys=(1,),
                         emit_mode=emit_mode) > 10000


def test_batched_units_vs_oracle(native):
  """Several units sampled in one batch (jump-ahead segments for every stream, concurrent decodes, the batch-wide
  permutation sort of mh_sort.h), emitted in the reference's unit order: the arena equals the oracle's per-unit FASTQ
  concatenated."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 30.0)
  regions = [('5', 0, 9_000_000), ('6', 250_000, 4_000_000)]
  seqs = [synth.contig(9_000_000, 21), synth.contig(4_000_000, 22)]
  copies = [synth.copies_soa(synth.variants(seqs[0], 23), 0, 9_000_000),
            synth.copies_soa(synth.variants(seqs[1], 24), 250_000, 4_000_000)]
  units = _native.work_units(99, [2, 2], passes)
  eng = Engine(0)
  try:
    for ri, (reg, s) in enumerate(zip(regions, seqs)):
      eng.load_region(ri, reg, s[reg[1]:reg[2]])
    res = eng.run_units([(ps, ri, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)],
                        lambda r, c: copies[r][c], p, 150, mdl['cum_tlen'], 'SYN')
    d1, d2 = eng.ctx.fetch_output()
    fix = eng.ctx.fixup_count()
  finally:
    eng.close()
  o1, o2, total = [], [], 0
  for ps, (ri, cpy, sd) in enumerate(units):
    reg = regions[ri]
    k, b1, b2 = O.generate_unit_soa(seqs[ri][reg[1]:reg[2]], reg[1], copies[ri][cpy], p, 150, mdl['cum_tlen'], sd,
                                    'SYN:0:{}'.format(ps), reg[0], cpy)
    assert res[ps][1] == k
    o1.append(b1)
    o2.append(b2)
  G.check_same(d1, b''.join(o1))
  G.check_same(d2, b''.join(o2))
  assert fix <= 1   # (the exact fallbacks are forced and pinned in test_*_forced_fallbacks_vs_oracle)


def test_prefetched_haplotypes_vs_build(native):
  """Engine.run_units(prefetch=...) as `bench.py --prefetch` runs it: the next batch's haplotypes spliced by the
  context's prefetch thread on its own stream (mh_prefetch_haplotypes_vset) while the current batch is sampled and
  written, and the next step's first batch as a fresh build kept across drop_haplotypes.  Two steps of three batches:
  every batch's FASTQ equal to the same run with every haplotype built at its batch's start, the first step equal to
  the oracle's; a prefetch into a live slot is refused."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 10.0)
  lens = [3_000_000, 2_000_000, 2_500_000]
  regions = [(str(7 + i), 0, L) for i, L in enumerate(lens)]
  seqs = [synth.contig(L, 51 + i) for i, L in enumerate(lens)]
  copies = [synth.copies_soa(synth.variants(s, 61 + i)) for i, s in enumerate(seqs)]
  units = _native.work_units(77, [2] * len(lens), passes)
  job = [(ps, ri, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)]
  batches = [[u for u in job if u[1] == ri] for ri in range(len(lens))]

  def run(prefetch):
    eng = Engine(0)
    outs = []
    try:
      for ri, (reg, sq) in enumerate(zip(regions, seqs)):
        eng.load_region(ri, reg, sq)
        for cpy in (0, 1):
          eng.upload_variants(ri, cpy, copies[ri][cpy])
      for step in range(2):
        eng.drop_haplotypes()
        for i, batch in enumerate(batches):
          last = i + 1 == len(batches)
          nxt = batches[0] if last else batches[i + 1]
          eng.ctx.reset_output()
          res = eng.run_units(batch, lambda r, c: copies[r][c], p, 150, mdl['cum_tlen'], 'PF',
                              prefetch=nxt if prefetch else None,
                              prefetch_next_step=last, prefetch_after=0)
          outs.append((res, eng.ctx.fetch_output()))
      if prefetch:
        live = eng._haps[(0, 0)][0]
        with pytest.raises(ValueError):   # (MH_E_ARG: a live slot)
          eng.ctx.prefetch_haplotypes_vset([live], [0], [1], [eng._vsets[(0, 0)]])
    finally:
      eng.close()
    return outs

  a, b = run(True), run(False)
  assert len(a) == len(b) == 2 * len(batches)
  for (ra, (a1, a2)), (rb, (b1, b2)) in zip(a, b):
    assert ra == rb
    G.check_same(a1, b1)
    G.check_same(a2, b2)
  for i, batch in enumerate(batches):   # the first step against the oracle
    o1, o2 = [], []
    for ps, ri, cpy, sd in batch:
      k, x1, x2 = O.generate_unit_soa(seqs[ri], 0, copies[ri][cpy], p, 150, mdl['cum_tlen'], sd, 'PF:0:{}'.format(ps),
                                      regions[ri][0], cpy)
      o1.append(x1)
      o2.append(x2)
    G.check_same(a[i][1][0], b''.join(o1))
    G.check_same(a[i][1][1], b''.join(o2))
    assert a[i][1][0] == a[len(batches) + i][1][0]   # (the second step repeats the first)


def test_lsd_sort_repeated_batches(native):
  """The permutation sort (mh_sort.h) over batches of different sizes and then the first batch again: its look-back
  status words sit inside the sort's buffer at an offset that moves with the batch size, so a batch size seen before
  must not find stale status there (round 4: a timed-out look-back scan on the bench's second step).  The repeat's
  templates equal the first run's, and every batch's equal a one-unit-at-a-time run's."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  L = 4_000_000
  seq = synth.contig(L, 41)
  copies = synth.copies_soa(synth.variants(seq, 42))
  batches = [[(0, 0, 0, 501), (1, 0, 1, 502), (2, 0, 0, 503)], [(3, 0, 1, 601)], [(4, 0, 0, 701), (5, 0, 1, 702)]]
  got = {}
  for mode in ('batch', 'single'):
    eng = Engine(0)
    try:
      eng.load_region(0, ('2', 0, L), seq)
      runs = []
      for k, b in enumerate(batches + [batches[0]]):
        eng.haplotypes([(ri, cpy) for _, ri, cpy, _ in b])
        slots = [eng.haplotype(ri, cpy, copies[cpy])[0] for _, ri, cpy, _ in b]
        if mode == 'batch':
          ns = eng.ctx.sample_units([100 * k + i for i in range(len(b))], slots, [u[3] for u in b], p, 150,
                                    mdl['cum_tlen'])
        else:
          ns = [eng.ctx.sample_units([100 * k + i], [sl], [u[3]], p, 150, mdl['cum_tlen'])[0]
                for i, (sl, u) in enumerate(zip(slots, b))]
        runs.append([eng.ctx.templates_export(100 * k + i) for i in range(len(b))])
        assert min(ns) > 1000
      got[mode] = runs
    finally:
      eng.close()
  for a, b in zip(got['batch'][0], got['batch'][-1]):
    for x, y in zip(a, b):
      assert np.array_equal(x, y)
  for ra, rb in zip(got['batch'], got['single']):
    for a, b in zip(ra, rb):
      for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_async_tail_equals_sync_templates(native):
  """mh_sample_units_async: the units' tails queued on the second stream and resolved one by one, in any order (a
  count, an export — any non-emission entry point resolves every pending set — or the next batch's sampling), give
  the same template sets as mh_sample_units."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 30.0)
  L = 6_000_000
  seq = synth.contig(L, 31)
  copies = synth.copies_soa(synth.variants(seq, 32))
  units = [(0, c, 4100 + k) for k, c in enumerate([0, 1, 0, 1, 1])]
  eng = Engine(0)
  try:
    eng.load_region(0, ('3', 0, L), seq)
    eng.haplotypes([(0, 0), (0, 1)])
    slots = [eng.haplotype(0, c, copies[c])[0] for _, c, _ in units]
    seeds = [sd for _, _, sd in units]
    ns = eng.ctx.sample_units(list(range(5)), slots, seeds, p, 150, mdl['cum_tlen'])
    want = [eng.ctx.templates_export(i) for i in range(5)]
    assert min(ns) > 1000
    for rep in range(2):
      eng.ctx.sample_units_async(list(range(10, 15)), slots, seeds, p, 150, mdl['cum_tlen'])
      if rep == 0:
        for i in (2, 0, 4):   # out of order, one at a time
          assert eng.ctx.template_count(10 + i) == ns[i]
        got = [eng.ctx.templates_export(10 + i) for i in range(5)]   # (resolves 1 and 3 too)
      else:   # nothing resolved before the next batch's sampling: its start resolves them
        eng.ctx.sample_units_async(list(range(20, 25)), slots, seeds, p, 150, mdl['cum_tlen'])
        got = [eng.ctx.templates_export(10 + i) for i in range(5)] + \
              [eng.ctx.templates_export(20 + i) for i in range(5)]
      for k, g in enumerate(got):
        w = want[k % 5]
        assert len(g[0]) == ns[k % 5]
        for a, b in zip(g, w):
          assert np.array_equal(a, b), (rep, k)
  finally:
    eng.close()


def test_resident_variants_and_buffer_reuse(native):
  """Haplotypes spliced from resident variant sets (mh_upload_variants) equal the host-array path, and rebuilding
  after a drop (the released buffers are reused, holding another copy's bytes) gives the same nodes, bytes and
  FASTQ."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  L = 12_000_000
  seq = synth.contig(L, 11)
  copies = synth.copies_soa(synth.variants(seq, 12))
  eng = Engine(0)
  try:
    eng.load_region(0, ('1', 0, L), seq)

    def run(order):
      out = {}
      for cpy in order:
        n, kept, b1, b2 = eng.run_unit(0, 0, cpy, 777 + cpy, copies[cpy], p, 150, mdl['cum_tlen'], 'SYN')
        slot, n_nodes, _, _ = eng.haplotype(0, cpy, copies[cpy])
        out[cpy] = (eng.ctx.get_nodes(slot, n_nodes), eng.ctx.fetch_output(0, b1, 0, b2))
        eng.ctx.reset_output()
      eng.drop_haplotypes()
      return out

    host = run([0, 1])
    for cpy in (0, 1):
      eng.upload_variants(0, cpy, copies[cpy])
    dev = run([1, 0])
    dev2 = run([0, 1])
    with pytest.raises(_native.NativeError, match='unknown variant set'):
      eng.ctx.build_haplotype_vset(5, 0, 1, 99)
    bad = dict(copies[0])
    bad['op'] = bad['op'].copy()
    bad['op'][0] = ord('Q')
    with pytest.raises(ValueError, match='Complex variants'):
      eng.ctx.upload_variants(98, bad)
    eng.drop_variants()
  finally:
    eng.close()
  for cpy in (0, 1):
    (ps, pr, op, ol, hap), (d1, d2) = host[cpy]
    for other in (dev[cpy], dev2[cpy]):
      (ps2, pr2, op2, ol2, hap2), (e1, e2) = other
      assert np.array_equal(ps, ps2) and np.array_equal(pr, pr2) and np.array_equal(op, op2)
      assert np.array_equal(ol, ol2)
      G.check_same(hap, hap2, 'hap copy {}'.format(cpy))
      G.check_same(d1, e1, 'fastq1 copy {}'.format(cpy))
      G.check_same(d2, e2, 'fastq2 copy {}'.format(cpy))


def test_two_lane_splice_matches_one_lane(native):
  """Both copies spliced side by side (mh_build_haplotypes_vset: second stream, second host thread, its own scratch)
  give the nodes, haplotype bytes and FASTQ of one-at-a-time builds (mh_build_haplotype_vset per copy), over two
  contigs and a rebuild after a drop."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  seqs = [synth.contig(3_000_000, 51), synth.contig(2_000_000, 52)]
  copies = [synth.copies_soa(synth.variants(sq, 53 + i)) for i, sq in enumerate(seqs)]
  units = [(0, 0, 0, 61), (1, 0, 1, 62), (2, 1, 0, 63), (3, 1, 1, 64)]
  keys = [(ri, cpy) for ri in (0, 1) for cpy in (0, 1)]

  def run(one_lane):
    eng = Engine(0)
    try:
      for ri, sq in enumerate(seqs):
        eng.load_region(ri, (str(ri + 1), 0, len(sq)), sq)
        for cpy in (0, 1):
          eng.upload_variants(ri, cpy, copies[ri][cpy])
      out = []
      for _ in range(2):
        eng.drop_haplotypes()
        eng.ctx.reset_output()
        if one_lane:   # every copy built alone first, so run_units' two-lane build finds nothing to do
          for ri, cpy in keys:
            eng.haplotype(ri, cpy, None)
        else:
          eng.haplotypes(keys)
        res = eng.run_units(units, lambda ri, c: copies[ri][c], p, 150, mdl['cum_tlen'], 'SYN')
        nodes = [eng.ctx.get_nodes(*eng.haplotype(ri, cpy, None)[:2]) for ri, cpy in keys]
        out.append((res, nodes, eng.ctx.fetch_output()))
      return out
    finally:
      eng.close()

  a, b = run(True), run(False)
  for (ra, na, (a1, a2)), (rb, nb, (b1, b2)) in zip(a, b):
    assert ra == rb
    for x, y in zip(na, nb):
      for u, v in zip(x, y):
        assert np.array_equal(np.asarray(u), np.asarray(v)) if not isinstance(u, bytes) else u == v
    G.check_same(a1, b1, 'fastq1')
    G.check_same(a2, b2, 'fastq2')


def test_pipelined_jobs_match_isolated_runs(native):
  """Jobs queued back to back (the next job's haplotype rebuild and sampling run while the previous job's FASTQ
  writers are still queued, reusing released haplotype buffers) give the same bytes as each job run alone."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  L = 8_000_000
  seq = synth.contig(L, 31)
  copies = synth.copies_soa(synth.variants(seq, 32))
  jobs = [[(0, 0, 0, 11), (1, 0, 1, 12), (2, 0, 0, 13), (3, 0, 1, 14)],
          [(0, 0, 1, 21), (1, 0, 0, 22)],
          [(0, 0, 0, 31), (1, 0, 1, 32), (2, 0, 1, 33)]]

  def run(pipelined):
    eng = Engine(0)
    try:
      eng.load_region(0, ('1', 0, L), seq)
      for cpy in (0, 1):
        eng.upload_variants(0, cpy, copies[cpy])
      outs = []
      for units in jobs:
        eng.drop_haplotypes()
        res = eng.run_units(units, lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'SYN')
        if not pipelined:
          outs.append((res, eng.ctx.fetch_output()))
          eng.ctx.reset_output()
        else:
          outs.append((res, None))
      if pipelined:   # everything appended to the arenas; one fetch at the end
        return [r for r, _ in outs], eng.ctx.fetch_output()
      return [r for r, _ in outs], (b''.join(o[0] for _, o in outs), b''.join(o[1] for _, o in outs))
    finally:
      eng.close()

  res_a, (a1, a2) = run(False)
  res_b, (b1, b2) = run(True)
  assert res_a == res_b
  G.check_same(b1, a1, 'fastq1')
  G.check_same(b2, a2, 'fastq2')


def test_deferred_prepare_matches_waiting_prepare(native):
  """mh_emit_prepare with null outputs (no host round trip; totals read back when the writer is queued), with
  outputs (the waiting form) and no prepare at all (emit_reads measures itself) give the same bytes and counts, and
  the waiting form's returned totals are the writer's."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  L = 3_000_000
  seq = synth.contig(L, 41)
  copies = synth.copies_soa(synth.variants(seq, 42))
  units = [(0, 0, 51), (1, 1, 52), (2, 0, 53), (3, 1, 54)]

  def run(form):
    eng = Engine(0)
    try:
      eng.load_region(0, ('1', 0, L), seq)
      res = []
      for ps, cpy, sd in units:
        slot = eng.haplotype(0, cpy, copies[cpy])[0]
        eng.ctx.sample_units([ps], [slot], [sd], p, 150, mdl['cum_tlen'])
        eng.ctx.use_templates(ps)
        stub = 'SYN:0:{}'.format(ps)
        got = None
        if form == 'wait':
          got = eng.ctx.emit_prepare(slot, stub, '1', cpy, True, unit_key=sd)
        elif form == 'deferred':
          assert eng.ctx.emit_prepare(slot, stub, '1', cpy, True, unit_key=sd, wait=False) is None
        r = eng.ctx.emit_reads(slot, stub, '1', cpy, True, unit_key=sd)
        if got is not None:
          assert got == r
        res.append(r)
      return res, eng.ctx.fetch_output()
    finally:
      eng.close()

  res_w, (w1, w2) = run('wait')
  for form in ('deferred', 'none'):
    res_d, (d1, d2) = run(form)
    assert res_w == res_d and all(r[0] > 1000 for r in res_w)
    G.check_same(d1, w1, 'fastq1 ' + form)
    G.check_same(d2, w2, 'fastq2 ' + form)


# ---- the bench configuration (BASELINE configs[1]) at full size -----------------------------------------------------
CHR1 = 249_250_621
CHR1_SEED = 12345


@pytest.fixture(scope='module')
def chr1_unit(native):
  """One chr1-sized work unit (249 Mbp, copy 1, ~7.48 M draws, ~5.9 M kept templates) of the bench workload, run once
  on the GPU perfect and once with fused corruption: both FASTQ arenas, the node list and the haplotype."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  seq = synth.contig(CHR1, 1)
  copies = synth.copies_soa(synth.variants(seq, 2))
  out = {'seq': seq, 'copies': copies, 'p': p, 'model': mdl}
  for corrupt in (False, True):
    eng = Engine(0)
    try:
      if corrupt:
        eng.ctx.set_corruption(True, mdl['cum_bq_mat'], 10 ** (-np.arange(100) / 10), 7)
      eng.load_region(0, ('1', 0, CHR1), seq)
      n, kept, b1, b2 = eng.run_unit(0, 0, 1, CHR1_SEED, copies[1], p, 150, mdl['cum_tlen'], 'SYN')
      key = 'corrupt' if corrupt else 'perfect'
      out[key] = eng.ctx.fetch_output()
      out[key + '_counts'] = (n, kept, b1, b2)
      if not corrupt:
        slot, n_nodes, p_min, p_max = eng.haplotype(0, 1, copies[1])
        out['nodes'] = eng.ctx.get_nodes(slot, n_nodes)
        out['span'] = (p_min, p_max)
    finally:
      eng.close()
  return out


@pytest.fixture(scope='module')
def chr1_oracle(chr1_unit):
  """The same unit through the CPU oracle (~15-20 s on one core)."""
  from oracle import oracle as O
  u = chr1_unit
  return O.generate_unit_soa(u['seq'], 0, u['copies'][1], u['p'], 150, u['model']['cum_tlen'], CHR1_SEED, 'SYN:0:0',
                             '1', 1)


def test_chr1_templates_vs_oracle(native, chr1_unit):
  """The whole template arrays of a chr1-length unit (7.48 M geometric draws, the full Fisher-Yates decode and
  permutation, k_decode_tail) equal the oracle's (illumina.py:66-76)."""
  from mitty_amd.simulation import illumina
  from oracle import oracle as O
  mdl = chr1_unit['model']
  p_min, p_max = chr1_unit['span']
  rm = illumina.read_model_params(mdl, 30.0)
  r = illumina.generate_reads(rm, p_min, p_max, CHR1_SEED)
  fo, p0, p1 = O.generate_templates(rm['p'], 150, mdl['cum_tlen'], p_min, p_max, CHR1_SEED)
  assert len(p0) > 6_000_000
  assert np.array_equal(r[0]['file_order'], fo)
  assert np.array_equal(r[0]['pos'], p0)
  assert np.array_equal(r[1]['pos'], p1)


def test_chr1_unit_fastq_vs_oracle(native, chr1_unit, chr1_oracle):
  """Both FASTQ files of the full chr1 unit byte-identical to the oracle: 9-digit POS (SplitWriter::put_u's nd > 8
  branch) and 7-digit cnt (digit_sum offsets past 999,999 kept templates) are exercised throughout."""
  k, o1, o2 = chr1_oracle
  n, kept, b1, b2 = chr1_unit['perfect_counts']
  d1, d2 = chr1_unit['perfect']
  assert kept == k and kept > 1_000_000
  assert (len(d1), len(d2)) == (b1, b2)
  G.check_same(d1, o1, 'chr1 file 1')
  G.check_same(d2, o2, 'chr1 file 2')
  last = d1[d1.rindex(b'\n@', 0, len(d1) - 1) + 2:].split(b'\n')[0].decode()
  assert last.startswith('SYN:0:0:{}|'.format(kept)) and len(str(kept)) == 7
  assert re.search(rb'\|[01]\|[1-9][0-9]{8}\|150\|', d1[-50_000_000:])   # 9-digit positions


def _line_fields_equal(a, b, fields):
  """FASTQ texts a, b: same line structure, and lines whose index mod 4 is in `fields` byte-equal."""
  A, B = np.frombuffer(a, np.uint8), np.frombuffer(b, np.uint8)
  assert len(A) == len(B)
  nl = np.flatnonzero(A == 10)
  assert np.array_equal(nl, np.flatnonzero(B == 10))
  starts = np.concatenate([[0], nl[:-1] + 1])
  for f in fields:
    s, e = starts[f::4], nl[f::4]
    for c in range(0, len(s), 1 << 20):
      cs, ce = s[c:c + (1 << 20)], e[c:c + (1 << 20)]
      ln = ce - cs
      idx = np.repeat(cs - np.concatenate([[0], np.cumsum(ln)[:-1]]), ln) + np.arange(int(ln.sum()))
      if not np.array_equal(A[idx], B[idx]):
        bad = int(np.nonzero(A[idx] != B[idx])[0][0])
        raise AssertionError('field {} differs near byte {}'.format(f, int(idx[bad])))


def test_chr1_corrupted_qnames_vs_oracle(native, chr1_unit, chr1_oracle):
  """BASELINE configs[2]: the chr1 unit with fused BQ corruption keeps every qname (and the '+' lines) byte-equal to
  the CPU oracle's; sequences and qualities keep their lengths; qualities are no longer all '~'."""
  _, o1, o2 = chr1_oracle
  c1, c2 = chr1_unit['corrupt']
  assert chr1_unit['corrupt_counts'] == chr1_unit['perfect_counts']
  _line_fields_equal(c1, o1, (0, 2))
  _line_fields_equal(c2, o2, (0, 2))
  assert c1 != o1 and c2 != o2


def test_chr1_scale_properties(native, chr1_unit):
  """Size-independent checks over every record of the first 40 MB: qnames parse, cnt runs 1, 2, ..., the CIGAR
  consumes the read length, qualities are '~', and each read equals the haplotype slice its qname implies (POS mapped
  to a sample coordinate through the node list; mate on strand 1 reverse-complemented)."""
  from mitty_amd.simulation.readgenerate import parse_qname
  ps, pr, op, ol, hap = chr1_unit['nodes']
  p_min = int(ps[0])
  d1 = chr1_unit['perfect'][0][:40_000_000]
  eq = (op == ord('=')) | (op == ord('X'))
  eq_pr, eq_ps, eq_len = pr[eq], ps[eq], np.where(op[eq] == ord('X'), 1, ol[eq])
  comp = bytes.maketrans(b'ATCGN', b'TAGCN')
  lines = d1.split(b'\n')
  n_rec = (len(lines) - 1) // 4
  assert n_rec > 50000
  checked = 0
  for i in range(n_rec - 1):
    qn, s, q = lines[4 * i][1:].decode(), lines[4 * i + 1], lines[4 * i + 3]
    assert int(qn.split('|')[0].split(':')[3]) == i + 1
    assert len(q) == 150 and set(q) == {ord('~')}
    r = parse_qname(qn)[0]
    if r.special_cigar is not None or len(s) != 150:
      continue
    consumed = sum(int(a) for a, o in re.findall(r'(\d+)([=XID])', r.cigar) if o in '=XI')
    assert consumed == 150
    if re.match(r'\d+([=XID])', r.cigar).group(1) not in '=X':   # a read starting inside an insertion
      continue
    k = int(np.searchsorted(eq_pr, r.pos, 'right')) - 1
    assert eq_pr[k] <= r.pos < eq_pr[k] + eq_len[k]
    samp = int(eq_ps[k]) + r.pos - int(eq_pr[k])
    want = bytes(hap[samp - p_min:samp - p_min + 150])
    got = s if r.strand == 0 else s.translate(comp)[::-1]
    assert got == want, (i, qn)
    checked += 1
  assert checked > 0.9 * n_rec


# ---- corruption (Philox mode) ----------------------------------------------------------------------------------
def test_corruption_statistics(native, tmp_path):
  """Qnames unchanged; qualities follow the model's per-position BQ distribution; substitution rate follows the
  phred error probability; substitutions are to a different base."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  seq = synth.contig(3_000_000, 3)
  copies = synth.copies_soa(synth.variants(seq, 4))
  outs = []
  for corrupt in (False, True):
    eng = Engine(0)
    try:
      if corrupt:
        eng.ctx.set_corruption(True, mdl['cum_bq_mat'], 10 ** (-np.arange(100) / 10), 7)
      eng.load_region(0, ('1', 0, len(seq)), seq)
      eng.run_unit(0, 0, 0, 77, copies[0], p, 150, mdl['cum_tlen'], 'S')
      outs.append(eng.ctx.fetch_output())
    finally:
      eng.close()
  (a1, a2), (c1, c2) = outs
  for a, c, mate in ((a1, c1, 0), (a2, c2, 1)):
    la, lc = a.split(b'\n'), c.split(b'\n')
    assert len(la) == len(lc)
    assert la[0::4] == lc[0::4]                      # qnames untouched
    seq_a, seq_c, qual = la[1::4], lc[1::4], lc[3::4]
    n = len(qual) - 1
    Q = np.frombuffer(b''.join(qual[:n]), np.uint8).reshape(n, 150).astype(np.int64) - 33
    SA = np.frombuffer(b''.join(seq_a[:n]), np.uint8).reshape(n, 150)
    SC = np.frombuffer(b''.join(seq_c[:n]), np.uint8).reshape(n, 150)
    # BQ histogram at a few positions vs the model's pmf
    for pos in (0, 75, 149):
      pmf = np.diff(np.concatenate([[0.0], mdl['cum_bq_mat'][mate, pos, :]]))
      h = np.bincount(Q[:, pos], minlength=94)[:94] / n
      assert np.abs(h - pmf).max() < 0.02, (mate, pos)
    err = SA != SC
    exp = (10 ** (-Q / 10.0)).mean()
    assert abs(err.mean() - exp) < 0.1 * exp + 1e-4
    changed = SC[err]
    assert not np.any(changed == SA[err])


@pytest.mark.parametrize('model', G.MODELS)
def test_corruption_direct_writer_matches_lds_writer(native, monkeypatch, model):
  """Fused corruption in the direct writer (B corrupted in LDS, per-record quality strings) gives the bytes of the
  LDS-image writer (same Philox counters), golden synthetic genome with lowercase / IUPAC / N bytes included."""
  from mitty_amd import _native
  from mitty_amd.engine import Engine
  from mitty_amd.lib import fasta as mfasta, vcfio
  mdl = G.model(model)
  rlen = int(mdl['mean_rlen'])
  p, _ = _native.read_model_params(rlen, 30.0)
  vdf = vcfio.load_variants_soa(G.path('data/syn.vcf'), 'S1', G.path('data/syn.bed'))
  seqs = mfasta.read_fasta(G.path('data/syn.fa'))
  outs = []
  # (the direct writer and the LDS-image writer + the in-place pass, mh_set_emit_mode(1))
  for lds in (False, True):
    eng = Engine(0)
    try:
      eng.ctx.set_emit_mode(1 if lds else 0)
      eng.ctx.set_corruption(True, mdl['cum_bq_mat'], 10 ** (-np.arange(100) / 10), 9)
      for ri in range(len(vdf)):
        chrom, s0, e = vdf[ri]['region']
        eng.load_region(ri, vdf[ri]['region'], mfasta.fetch(seqs, chrom, s0, e))
        for cpy in range(len(vdf[ri]['copies'])):
          eng.run_unit(ri, ri, cpy, 1000 + 10 * ri + cpy, vdf[ri]['copies'][cpy], p, rlen, mdl['cum_tlen'], 'S1')
      outs.append(eng.ctx.fetch_output())
    finally:
      eng.close()
  (l1, l2) = outs[-1]
  assert len(l1) > 10000
  for k, (d1, d2) in enumerate(outs[:-1]):
    G.check_same(d1, l1, 'fastq1 (variant {})'.format(k))
    G.check_same(d2, l2, 'fastq2 (variant {})'.format(k))


@pytest.mark.parametrize('tables,write2', [('lds', True), ('global', True), ('lds', False), ('stress', True),
                                           ('rlen250', True)])
def test_philox_corruption_vs_numpy_restatement(native, monkeypatch, tables, write2):
  """Philox-mode corruption (the writer's len(seq) layout + k_cr_inplace) byte for byte against the numpy
  restatement of the draw scheme with full 53-bit uniforms (tests/philox_ref.py) applied to the perfect reads of the
  same sampling.  No N in the genome, so every template is kept and cnt - 1 is the template index; the bucket table
  from LDS and from global memory (MH_CR_GLOBAL), one and two FASTQ files.  'stress': a BQ table of 93 random
  thresholds per position, so ~9 % of draws land in a bucket holding one — waves with more flagged draws than the
  row pass's LDS item list (its per-lane fallback), walks of several entries and the exact decisions all run.
  'rlen250': 2x250 reads of 1kg-pcr-free (16 full blocks and a short one of 10 bases per read)."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from tests import philox_ref
  if tables == 'global':
    monkeypatch.setenv('MH_CR_GLOBAL', '1')
  mdl = G.model('1kg-pcr-free' if tables == 'rlen250' else 'hiseq-X-v2.5-Garvan')
  rlen = int(mdl['mean_rlen'])
  cum = mdl['cum_bq_mat']
  if tables == 'stress':
    cum = np.sort(np.random.default_rng(5).random(cum.shape), axis=2)
    cum[:, :, -1] = 1.0
  p, _ = _native.read_model_params(rlen, 30.0)
  seq = synth.contig(400_000, 5, n_gaps=False)
  copies = synth.copies_soa(synth.variants(seq, 6))
  phred = 10 ** (-np.arange(100) / 10)
  outs = []
  for corrupt in (False, True):
    eng = Engine(0)
    try:
      if corrupt:
        eng.ctx.set_corruption(True, cum, phred, 3_000_000_099)
      eng.load_region(0, ('1', 0, len(seq)), seq)
      eng.run_unit(0, 0, 1, 4711, copies[1], p, rlen, mdl['cum_tlen'], 'S', write_fastq2=write2)
      outs.append(eng.ctx.fetch_output())
    finally:
      eng.close()
  (a1, a2), (c1, c2) = outs
  files = ((a1, c1), (a2, c2)) if write2 else ((a1, c1),)
  n_sub = 0
  for f, (a, c) in enumerate(files):
    la, lc = a.split(b'\n'), c.split(b'\n')
    assert len(la) == len(lc) and len(la) > 20000
    assert la[0::4] == lc[0::4]
    ts = [int(q.split(b'|', 1)[0].rsplit(b':', 1)[1]) - 1 for q in la[0:-1:4]]
    assert ts == list(range(len(ts)))                       # every template kept
    want_s, want_q = philox_ref.corrupt_reads(la[1::4][:len(ts)], ts, f, cum, phred, 3_000_000_099, 4711)
    assert lc[1::4][:len(ts)] == want_s
    assert lc[3::4][:len(ts)] == want_q
    n_sub += sum(x != y for x, y in zip(la[1::4], want_s))
  assert n_sub > 100


# ---- multi-GPU slices ---------------------------------------------------------------------------
@pytest.mark.parametrize('corrupt', [False, True])
def test_emit_slices_concatenate_to_unit(native, corrupt):
  """mh_emit_reads_range over consecutive slices, each numbered from the kept count of the slices before it
  (mh_count_kept), concatenates to the whole-unit emission byte for byte (corruption keyed by the unit index)."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(150, 30.0)
  seq = synth.contig(2_500_000, 31)
  copies = synth.copies_soa(synth.variants(seq, 32))
  eng = Engine(0)
  try:
    if corrupt:
      eng.ctx.set_corruption(True, mdl['cum_bq_mat'], 10 ** (-np.arange(100) / 10), 5)
    eng.load_region(0, ('1', 0, len(seq)), seq)
    slot = eng.haplotype(0, 0, copies[0])[0]
    n = int(eng.ctx.sample_units([0], [slot], [4242], p, 150, mdl['cum_tlen'])[0])
    eng.ctx.use_templates(0)
    kept, b1, b2 = eng.ctx.emit_reads(slot, 'S:0:1', '1', 0, True, 4242)
    whole = eng.ctx.fetch_output()
    eng.ctx.reset_output()
    assert eng.ctx.count_kept(slot, 0, n) == kept
    cuts = [0, 1, 1, 777, n // 3, n - 5, n]
    base = 0
    for a, b in zip(cuts[:-1], cuts[1:]):
      k, _, _ = eng.ctx.emit_reads(slot, 'S:0:1', '1', 0, True, 4242, t_range=(a, b), cnt_base=base)
      assert k == eng.ctx.count_kept(slot, a, b)
      base += k
    assert base == kept
    assert eng.ctx.fetch_output() == whole
  finally:
    eng.close()


def _gpu_rank(rank, world, port, layout, outdir, bam=False, spill_dir=None):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd import distributed as D
    from mitty_amd.readmodel import get_read_model
    c = G.load_json('e2e_config.json')['1kg-pcr-free']
    mod, mdl = get_read_model('1kg-pcr-free.pkl')
    extra = {}
    if bam:   # the configs[4] BAM leg: every rank sorts and writes one coordinate range
      extra = dict(bam_fname=os.path.join(outdir, 'g.bam'), bam_header_text='@HD\tVN:1.0\tSO:coordinate\n',
                   bam_refs=[('1', 50000), ('2', 20000), ('3', 8000)], bam_capacity=bam if bam is not True else 0,
                   bam_spill_dir=spill_dir)
    D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                 c['coverage'], os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'),
                                 seed=c['seed'], backend=D.DeviceBackend(0), layout=layout, **extra)
  finally:
    dist.destroy_process_group()


def _packing_worker(_rank, port):
  """(a fresh process: torch's HIP runtime first, as in every torch.distributed rank)"""
  import torch
  import torch.distributed as dist
  from mitty_amd import _native as native, distributed as D, synth
  from mitty_amd.readmodel import get_read_model
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  p, _ = native.read_model_params(150, 30.0)
  seq = synth.contig(400_000, 31)
  soa = synth.copies_soa(synth.variants(seq, 32))
  be = D.DeviceBackend(0)
  try:
    be.load_region(0, ('4', 0, len(seq)), seq)
    unit = (0, 0, 1, 123456)
    ns = be.sample([unit, unit], lambda r, c: soa[c], p, 150, mdl['cum_tlen'], 'mitty', which=[0])
    n = ns[0]
    assert n > 10000 and ns[1] is None

    def emitted(k):
      _, r1, r2 = be.emit(k, 'S:0:0', '4', 1, True, unit[3], None, 0)
      return be.fetch(r1, r2)
    want = emitted(0)
    buf = torch.empty(17 * n, dtype=torch.uint8, device='cuda')
    assert be.pack_device(0, n, buf.data_ptr()) == n
    be.unpack_device(1, n, 150, buf.data_ptr())
    assert emitted(1) == want
    host = np.zeros(17 * n, np.uint8)
    be.pack_host(0, n, host)
    assert np.array_equal(host, buf.cpu().numpy())
    be.unpack_host(1, n, 150, host)
    assert emitted(1) == want
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port), rank=0, world_size=1)
    try:
      be.share(0, n, 0, 150)
    finally:
      dist.destroy_process_group()
    assert emitted(0) == want
  finally:
    be.close()


def test_template_broadcast_packing_round_trip(native):
  """The sliced multi-GPU layout's broadcast unit (DeviceBackend.share): a sampled unit's templates packed into one
  device buffer (pos0 | pos1 | fo0 at 0 / 8n / 16n, the RCCL payload) and into a host buffer (the gloo payload),
  imported into another template set, emit the same FASTQ bytes as the sampled set; share() itself under a one-rank
  gloo group.  Runs in a spawned process (torch and libmitty_hip in one process need torch loaded first)."""
  from tests._spawn import spawn_with_port
  spawn_with_port(_packing_worker, lambda port: (port,), 1)


@pytest.mark.parametrize('layout', ['lpt', 'slice'])
def test_distributed_two_ranks_one_gpu(native, tmp_path, layout):
  """Two ranks (gloo for the int64 exchanges, both on GPU 0) write the reference --threads 1 files."""
  from tests._spawn import spawn_with_port
  spawn_with_port(_gpu_rank, lambda port: (2, port, layout, str(tmp_path)), 2)
  G.check_same(open(tmp_path / 'r1.fq', 'rb').read(), G.fastq_bytes('e2e_1kg-pcr-free.r1.fq.gz'))
  G.check_same(open(tmp_path / 'r2.fq', 'rb').read(), G.fastq_bytes('e2e_1kg-pcr-free.r2.fq.gz'))


@pytest.mark.parametrize('world,layout,cap,disk', [(2, 'lpt', 0, False), (2, 'slice', 300_000, False),
                                                  (3, 'lpt', 200_000, True)])
def test_distributed_bam_ranks_one_gpu(native, tmp_path, world, layout, cap, disk):
  """configs[4] across ranks without a merging rank: 2 or 3 ranks (gloo, all on GPU 0) each build the BAM records of
  their pieces on the device and partition them by coordinate range (mh_bam_partition); the all-to-all moves every
  record to its range's rank, which sorts its range (ties by global input order), deflates the blocks that start in
  it on the device (mh_bam_write_part) and contributes its BAI plan.  BAM and BAI equal the one-GPU god-aligner's
  file (mh_bam_write_gpu over the same FASTQ, one store) byte for byte, and the records and index the oracle's; with
  bounded range stores (cap) spilling to host memory or to temporary files (disk)."""
  from tests._spawn import spawn_with_port
  from oracle import god
  one, many = tmp_path / 'one', tmp_path / 'many'
  one.mkdir()
  many.mkdir()
  spill = str(tmp_path / 'spill') if disk else None
  if disk:
    os.mkdir(spill)
  spawn_with_port(_gpu_rank, lambda port: (world, port, layout, str(many), cap or True, spill), world)
  f1, f2 = G.fastq_bytes('e2e_1kg-pcr-free.r1.fq.gz'), G.fastq_bytes('e2e_1kg-pcr-free.r2.fq.gz')
  G.check_same(open(many / 'r1.fq', 'rb').read(), f1)
  # the one-store reference: the god-aligner's own GPU writer over the same FASTQ
  from mitty_amd.engine import Engine
  eng = Engine(0)
  try:
    eng.ctx.bam_set_refs(['1', '2', '3'], [50000, 20000, 8000])
    eng.ctx.bam_add_fastq(f1, f2)
    eng.ctx.bam_write_gpu(str(one / 'g.bam'), '@HD\tVN:1.0\tSO:coordinate\n', bai_path=str(one / 'g.bam.bai'))
  finally:
    eng.close()
  a, b = open(one / 'g.bam', 'rb').read(), open(many / 'g.bam', 'rb').read()
  assert a == b
  assert open(one / 'g.bam.bai', 'rb').read() == open(many / 'g.bam.bai', 'rb').read()
  _, recs, vo, vend = god.record_voffsets(b)
  want = god.sorted_stream(god.god_records(f1, f2, {'1': 0, '2': 1, '3': 2}))
  assert len(recs) == len(want) > 1000 and recs == [god.encode(r) for r in want]
  assert open(many / 'g.bam.bai', 'rb').read() == god.bai(3, [god.decode(r) for r in recs], vo, vend)
  assert not [f for f in os.listdir(many) if '.part' in f]
  if disk:
    assert os.listdir(spill) == []   # (the spill files were unlinked when mapped)


# ---- god-aligner BAM -------------------------------------------------------------------------
def _god_setup(tmp_path):
  fa = tmp_path / 'ref.fa'
  fa.write_text('')
  (tmp_path / 'ref.fa.ann').write_text('1 1 11\n0 1 (null)\n0 50000 0\n0 2 (null)\n0 20000 0\n0 3 (null)\n0 8000 0\n')
  return str(fa)


def _god_check(bam, fq1, fq2, max_templates=None, sample='Seven'):
  """The BAM file against the oracle: header bytes, sorted record stream, BAI over the file's own offsets."""
  from oracle import god
  from mitty_amd.benchmarking import god_aligner as ga
  data = open(bam, 'rb').read()
  header, recs, vo, vend = god.record_voffsets(data)
  sq = G.load_json('god_header.json')
  import base64
  import sys
  text = ga.header_text({'HD': {'VN': '1.0'},
                         'PG': [{'CL': ' '.join(sys.argv), 'ID': 'mitty-god-aligner', 'PN': 'god-aligner',
                                 'VN': ga.__version__}],
                         'RG': [{'ID': base64.b64encode(' '.join(sys.argv).encode('ascii')), 'SM': sample}],
                         'SQ': sq})
  assert header == god.header_bytes(text, sq)
  want = god.sorted_stream(god.god_records(fq1, fq2, {'1': 0, '2': 1, '3': 2}, max_templates))
  assert len(recs) == len(want)
  assert recs == [god.encode(r) for r in want]
  dec = [god.decode(r) for r in recs]
  assert open(bam + '.bai', 'rb').read() == god.bai(len(sq), dec, vo, vend)
  return dec


def _god_inputs(model, tmp_path):
  """The e2e FASTQ pair without templates whose sequence and quality lengths differ (a read cut by a deletion that
  runs past the region end keeps rlen qualities, readgenerate.py:229): pysam's quality setter raises ValueError on
  those (god_aligner.py:166-170), so the reference god-aligner cannot take them; test_god_aligner_rejects_* covers
  that error."""
  b1, b2 = G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)), G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model))
  l1, l2 = b1.split(b'\n'), b2.split(b'\n')
  keep = [i for i in range(0, len(l1) - 1, 4)
          if len(l1[i + 1]) == len(l1[i + 3]) and len(l2[i + 1]) == len(l2[i + 3])]
  c1 = b''.join(b'\n'.join(l1[i:i + 4]) + b'\n' for i in keep)
  c2 = b''.join(b'\n'.join(l2[i:i + 4]) + b'\n' for i in keep)
  f1, f2 = tmp_path / 'in1.fq', tmp_path / 'in2.fq'
  f1.write_bytes(c1)
  f2.write_bytes(c2)
  return str(f1), str(f2), c1, c2


def _nt16_fold(seq):
  """A sequence as a BAM record stores it (4-bit codes: case folded, unknown letters -> N)."""
  codes = '=ACMGRSVTWYHKDBN'
  return ''.join(c.upper() if c.upper() in codes else 'N' for c in seq)


@pytest.mark.parametrize('model', G.MODELS)
def test_god_aligner_bam_vs_oracle(native, model, tmp_path):
  from mitty_amd.benchmarking import god_aligner as ga
  fa = _god_setup(tmp_path)
  fq1, fq2, b1, b2 = _god_inputs(model, tmp_path)
  bam = str(tmp_path / 'g.bam')
  st = ga.process_multi_threaded(fa, bam, fq1, fq2, threads=3)
  dec = _god_check(bam, b1, b2)
  assert st['records'] == 2 * (b1.count(b'\n') // 4)
  # every record of god.json (captured from the reference's write_perfect_reads) is in the BAM
  have = {(d['qname'], d['is_read1']): d for d in dec}
  hit = 0
  for qn, recs in G.load_json('god.json'):
    for r in recs:
      if (qn, r['is_read1']) in have:
        got = have[(qn, r['is_read1'])]
        want = dict(r, seq=_nt16_fold(r['seq']))
        assert {k: got[k] for k in want} == want
        hit += 1
  assert hit > 0
  # small input chunks (records carried across calls), level 0 and 9, give the same records
  for chunk, level in ((7001, 0), (65536, 9)):
    bam2 = str(tmp_path / 'g{}.bam'.format(chunk))
    ga.process_multi_threaded(fa, bam2, fq1, fq2, threads=2, chunk_bytes=chunk, level=level)
    _god_check(bam2, b1, b2)


@pytest.mark.parametrize('gpu_bgzf', [False, True])
@pytest.mark.parametrize('model', G.MODELS)
def test_god_aligner_spilled_store_vs_oracle(native, model, gpu_bgzf, tmp_path):
  """Bounded HBM (mh_bam_set_capacity, the counterpart of the reference's `samtools sort -m 2G`, god_aligner.py:100-116):
  a 150 kB record budget with 64 kB input chunks spills the store to host memory many times over; the coordinate
  sort still runs on the device (keys stay in HBM) and the sorted stream is assembled on the host, window by window
  (one BGZF block per window at this budget, deflated on the device for gpu_bgzf).  The BAM and its BAI equal the
  unbounded store's byte for byte, and the oracle's records and index (oracle/god.py)."""
  from mitty_amd.benchmarking import god_aligner as ga
  fa = _god_setup(tmp_path)
  fq1, fq2, b1, b2 = _god_inputs(model, tmp_path)
  a, b = str(tmp_path / 'a.bam'), str(tmp_path / 'b.bam')
  sa = ga.process_multi_threaded(fa, a, fq1, fq2, threads=2, chunk_bytes=65536, gpu_bgzf=gpu_bgzf)
  sb = ga.process_multi_threaded(fa, b, fq1, fq2, threads=2, chunk_bytes=65536, gpu_bgzf=gpu_bgzf,
                                 hbm_capacity=150_000)
  assert sa['spill_blocks'] == 0 and sb['spill_blocks'] > 5 and sb['spilled_bytes'] == sb['bam_bytes_uncompressed']
  assert sb["bam_bytes_uncompressed"] > 4 * 150_000
  assert open(a, 'rb').read() == open(b, 'rb').read()
  assert open(a + '.bai', 'rb').read() == open(b + '.bai', 'rb').read()
  _god_check(b, b1, b2)


def test_god_aligner_spill_from_device_arenas(native, tmp_path):
  """The configs[4] path (records straight from the FASTQ arenas, mh_bam_add_output) over a bounded store: four
  generate-reads jobs appended (each add spills the records before it), the device-deflated file equal to the
  unbounded store's, and the write's device memory held near the bound."""
  from mitty_amd.engine import Engine
  from mitty_amd.lib import fasta as mfasta, vcfio
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  c = G.load_json('e2e_config.json')['1kg-pcr-free']
  mod, mdl = get_read_model('1kg-pcr-free.pkl')
  rm = mod.read_model_params(mdl, c['coverage'])
  vdf = vcfio.load_variants_soa(G.path(c['vcf']), c['sample'], G.path(c['bed']))
  seqs = mfasta.read_fasta(G.path(c['fasta']))
  units = [(ps, w['region_idx'], w['region_cpy'], w['rng_seed'])
           for ps, w in enumerate(readgenerate.get_data_for_workers(rm, vdf, c['seed']))]
  out = {}
  for cap in (0, 200_000):
    eng = Engine(0)
    try:
      for ri, reg in enumerate(vdf):
        eng.load_region(ri, reg['region'], mfasta.fetch(seqs, *reg['region']))
      eng.ctx.bam_set_refs(['1', '2', '3'], [50000, 20000, 8000])
      eng.ctx.bam_set_capacity(cap)
      for job in range(4):
        eng.ctx.reset_output()
        eng.run_units(units, lambda r, cp: vdf[r]['copies'][cp], rm['p'], rm['rlen'], rm['cum_tlen'],
                      'S{}'.format(job))
        eng.ctx.bam_add_output()
      bam = str(tmp_path / 'c{}.bam'.format(cap))
      eng.ctx.bam_sort()
      native.device_cache_trim()
      live0, _ = native.device_live_bytes(reset_peak=True)
      eng.ctx.bam_write_gpu(bam, '@HD\tVN:1.0\tSO:coordinate\n', bai_path=bam + '.bai')
      peak = native.device_live_bytes()[1] - live0
      out[cap] = (open(bam, 'rb').read(), open(bam + '.bai', 'rb').read(), eng.ctx.bam_spilled(), peak,
                  eng.ctx.bam_records())
    finally:
      eng.close()
  assert out[0][2] == (0, 0) and out[200_000][2][1] >= 2
  assert out[0][0] == out[200_000][0] and out[0][1] == out[200_000][1]
  # the bounded store's write stays near its bound: two staging windows and two deflate ring slots of
  # one BGZF block each at this budget (a quarter of 200 kB is less than a 0xff00-byte block) plus the deflate's
  # per-launch scratch for that block — not an output buffer for the whole record stream, as the unbounded store has
  rec_bytes = out[200_000][4][1]
  peaks = 'record bytes {}, write peak bounded {} / unbounded {}'.format(rec_bytes, out[200_000][3], out[0][3])
  print(peaks)
  assert rec_bytes > 2_500_000, peaks
  assert out[200_000][3] < 1_000_000, peaks
  assert out[0][3] > rec_bytes, peaks   # (the unbounded store: one output buffer for the whole file)


def test_god_aligner_rejects_sequence_quality_mismatch(native, tmp_path):
  """pysam's AlignedSegment raises ValueError('quality and sequence mismatch') in write_perfect_reads; so do we."""
  from mitty_amd.benchmarking import god_aligner as ga
  fa = _god_setup(tmp_path)
  fq1, fq2 = G.path('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz'), G.path('e2e_hiseq-X-v2.5-Garvan.r2.fq.gz')
  with pytest.raises(ValueError, match='quality and sequence mismatch'):
    ga.process_multi_threaded(fa, str(tmp_path / 'x.bam'), fq1, fq2)


def test_god_aligner_single_end_and_max_templates(native, tmp_path):
  from mitty_amd.benchmarking import god_aligner as ga
  fa = _god_setup(tmp_path)
  fq1, fq2, b1, b2 = _god_inputs('hiseq-X-v2.5-Garvan', tmp_path)
  bam = str(tmp_path / 's.bam')
  ga.process_multi_threaded(fa, bam, fq1, None, sample_name='S1')
  dec = _god_check(bam, b1, None, sample='S1')
  assert all(d['flag'] & 0x1 == 0 for d in dec)
  bam = str(tmp_path / 'm.bam')
  st = ga.process_multi_threaded(fa, bam, fq1, fq2, max_templates=9)
  assert st['templates'] == 10   # the reference stops after template index max_templates
  _god_check(bam, b1, b2, max_templates=10)


def test_god_aligner_errors(native, tmp_path):
  ctx = native.Context(0)
  try:
    ctx.bam_set_refs(['1', '2'], [50000, 20000])
    rec = b'@S:0:0:1|3|0|0|10|4|4=||1|20|4|4=|\nACGT\n+\n~~~~\n'
    with pytest.raises(ValueError, match='chrom'):
      ctx.bam_add_fastq(rec, rec)
    long_q = b'@S:0:0:1|1|0|0|10|4|4=|' + b'1,' * 200 + b'1|1|20|4|4=|\nACGT\n+\n~~~~\n'
    with pytest.raises(ValueError, match='254'):
      ctx.bam_add_fastq(long_q, long_q)
    bad = b'@S:0:0:1|1|0|0|10|4|4Q||1|20|4|4=|\nACGT\n+\n~~~~\n'
    with pytest.raises(ValueError, match='CIGAR'):
      ctx.bam_add_fastq(bad, bad)
    # an incomplete trailing record is left for the next call
    ok = b'@S:0:0:1|1|0|0|10|4|4=||1|20|4|4=|\nACGT\n+\n~~~~\n'
    u1, u2, t = ctx.bam_add_fastq(ok + ok[:20], ok + ok[:30])
    assert (u1, u2, t) == (len(ok), len(ok), 1)
  finally:
    ctx.close()


def test_god_aligner_from_device_arenas(native, tmp_path):
  """generate-reads output fed to the BAM builder on the device (no FASTQ round trip) = the file-based BAM."""
  from mitty_amd.benchmarking import god_aligner as ga
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  # the 2x250 golden run: no read there is cut short by a deletion past the region end (see _god_inputs)
  c = G.load_json('e2e_config.json')['1kg-pcr-free']
  mod, mdl = get_read_model('1kg-pcr-free.pkl')
  f1, f2 = str(tmp_path / 'r1.fq'), str(tmp_path / 'r2.fq')
  readgenerate.process_multi_threaded(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], f1, f2, seed=c['seed'])
  fa = _god_setup(tmp_path)
  bam_a = str(tmp_path / 'a.bam')
  ga.process_multi_threaded(fa, bam_a, f1, f2)
  from mitty_amd.engine import Engine
  from mitty_amd.lib import fasta as mfasta, vcfio
  rm = mod.read_model_params(mdl, c['coverage'])
  vdf = vcfio.load_variants_soa(G.path(c['vcf']), c['sample'], G.path(c['bed']))
  seqs = mfasta.read_fasta(G.path(c['fasta']))
  units = [(ps, w['region_idx'], w['region_cpy'], w['rng_seed'])
           for ps, w in enumerate(readgenerate.get_data_for_workers(rm, vdf, c['seed']))]
  eng = Engine(0)
  try:
    for ri, reg in enumerate(vdf):
      eng.load_region(ri, reg['region'], mfasta.fetch(seqs, *reg['region']))
    eng.run_units(units, lambda r, cp: vdf[r]['copies'][cp], rm['p'], rm['rlen'], rm['cum_tlen'], c['sample'])
    eng.ctx.bam_set_refs(['1', '2', '3'], [50000, 20000, 8000])
    assert eng.ctx.bam_add_output() == open(f1, 'rb').read().count(b'\n') // 4
    text = open(bam_a, 'rb').read()
    from oracle import god
    header, recs_a, _, _ = god.record_voffsets(text)
    l_text = int.from_bytes(header[4:8], 'little')
    bam_b = str(tmp_path / 'b.bam')
    eng.ctx.bam_write(bam_b, header[8:8 + l_text].decode(), bai_path=bam_b + '.bai')
    bam_c = str(tmp_path / 'c.bam')   # the record blocks deflated on the device (mh_bam_write_gpu)
    n_c, _, fb = eng.ctx.bam_write_gpu(bam_c, header[8:8 + l_text].decode(), bai_path=bam_c + '.bai')
  finally:
    eng.close()
  _, recs_b, _, _ = god.record_voffsets(open(bam_b, 'rb').read())
  assert recs_a == recs_b
  # the device-deflated file: the same header and records (zlib inflates every member), and its BAI indexes its own
  # virtual offsets as the oracle computes them
  data_c = open(bam_c, 'rb').read()
  assert len(data_c) == fb and data_c[-28:] == open(bam_b, 'rb').read()[-28:]
  header_c, recs_c, vo, vend = god.record_voffsets(data_c)
  assert header_c == header and recs_c == recs_a and n_c == len(recs_a)
  sq = [(b'1', 50000), (b'2', 20000), (b'3', 8000)]
  assert open(bam_c + '.bai', 'rb').read() == god.bai(len(sq), [god.decode(r) for r in recs_c], vo, vend)


def test_tumor_normal_mix_god_aligner(native, tmp_path):
  """BASELINE configs[4] in small: a normal (sample S0, 6x) and a tumor (S1, 12x, the VCF's other sample) run of the
  2x250 model into the same device arenas — the mix is the two runs' FASTQ one after the other, each sample named in
  its qnames (Readme.md:14-16) — then the perfect BAM built from the arenas (parse, encode, coordinate sort in HBM).
  The FASTQ equals the oracle's two runs concatenated; the BAM records equal the oracle god-aligner's over it, and a
  store bounded far below the records' size (spilled to host memory) writes the same BAM and BAI."""
  from mitty_amd.engine import Engine
  from mitty_amd.lib import fasta as mfasta, vcfio
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  from oracle import god
  from oracle import oracle as O
  c = G.load_json('e2e_config.json')['1kg-pcr-free']
  mod, mdl = get_read_model('1kg-pcr-free.pkl')
  seqs = mfasta.read_fasta(G.path(c['fasta']))
  runs = (('S0', 6.0, 11), ('S1', 12.0, 12))
  want1, want2 = b'', b''
  eng = Engine(0)
  try:
    ri0 = 0
    for sample, cov, seed in runs:
      rm = mod.read_model_params(mdl, cov)
      vdf = vcfio.load_variants_soa(G.path(c['vcf']), sample, G.path(c['bed']))
      for k, reg in enumerate(vdf):   # each sample's regions in their own slots (own haplotypes)
        eng.load_region(ri0 + k, reg['region'], mfasta.fetch(seqs, *reg['region']))
      units = [(ps, ri0 + w['region_idx'], w['region_cpy'], w['rng_seed'])
               for ps, w in enumerate(readgenerate.get_data_for_workers(rm, vdf, seed))]
      eng.run_units(units, lambda r, cp, v=vdf, o=ri0: v[r - o]['copies'][cp], rm['p'], rm['rlen'], rm['cum_tlen'],
                    sample)
      o1, o2, _ = O.generate_reads_fastq(G.path(c['fasta']), G.path(c['vcf']), sample, G.path(c['bed']),
                                         G.model('1kg-pcr-free'), cov, seed)
      want1 += o1
      want2 += o2
      ri0 += len(vdf)
    d1, d2 = eng.ctx.fetch_output()
    G.check_same(d1, want1)
    G.check_same(d2, want2)
    assert b'@S0:' in d1 and b'@S1:' in d1
    eng.ctx.bam_set_refs(['1', '2', '3'], [50000, 20000, 8000])
    assert eng.ctx.bam_add_output() == want1.count(b'\n') // 4
    eng.ctx.bam_sort()
    bam = str(tmp_path / 'tn.bam')
    eng.ctx.bam_write(bam, '@HD\tVN:1.0\n', bai_path=bam + '.bai')   # the sort above is reused
    # more records after the direct sorted write (the sorted block becomes the input-order prefix)
    eng.ctx.bam_add_fastq(want1, want2)
    bam2 = str(tmp_path / 'tn2.bam')
    eng.ctx.bam_write(bam2, '@HD\tVN:1.0\n')
    # the same mix into a store bounded to 40 kB (mh_bam_set_capacity): the arenas go in pieces, the store spills
    # between them, and the file (BAM and BAI) is the unbounded store's, byte for byte
    eng.ctx.bam_set_refs(['1', '2', '3'], [50000, 20000, 8000])
    eng.ctx.bam_set_capacity(40_000)
    assert eng.ctx.bam_add_output() == want1.count(b'\n') // 4
    assert eng.ctx.bam_spilled()[1] > 5
    bam3 = str(tmp_path / 'tn3.bam')
    eng.ctx.bam_write(bam3, '@HD\tVN:1.0\n', bai_path=bam3 + '.bai')
    eng.ctx.bam_set_capacity(0)
  finally:
    eng.close()
  assert open(bam3, 'rb').read() == open(bam, 'rb').read()
  assert open(bam3 + '.bai', 'rb').read() == open(bam + '.bai', 'rb').read()
  refs = {'1': 0, '2': 1, '3': 2}
  _, recs, _, _ = god.record_voffsets(open(bam, 'rb').read())
  assert recs == [god.encode(r) for r in god.sorted_stream(god.god_records(want1, want2, refs))]
  _, recs2, _, _ = god.record_voffsets(open(bam2, 'rb').read())
  assert recs2 == [god.encode(r) for r in god.sorted_stream(god.god_records(want1 + want1, want2 + want2, refs))]


# ---- standalone corrupt-reads --------------------------------------------------------------
@pytest.mark.parametrize('rng', ['mitty', 'philox'])
@pytest.mark.parametrize('model', G.MODELS)
def test_corrupt_reads_over_fastq(native, model, rng, tmp_path):
  """corrupt-reads on the e2e FASTQ pair: names (file 1's) and lengths kept, substitutions only to other bases,
  BQ per position distributed as the model says, substitution rate = mean phred error; chunking does not change
  the output; the CLI gives the same files."""
  from click.testing import CliRunner
  from mitty_amd.cli import cli
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readcorrupt
  mod, mdl = get_read_model(model + '.pkl')
  i1, i2 = G.path('e2e_{}.r1.fq.gz'.format(model)), G.path('e2e_{}.r2.fq.gz'.format(model))
  o1, o2 = str(tmp_path / 'c1.fq'), str(tmp_path / 'c2.fq')
  st = readcorrupt.multi_process(mod, mdl, i1, o1, i2, o2, seed=11, rng=rng)
  a1, a2 = G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)), G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model))
  assert st['templates'] == a1.count(b'\n') // 4
  names = [ln.split(b' ')[0] for ln in a1.split(b'\n')[0::4][:-1]]
  rlen = int(mdl['mean_rlen'])
  for mate, (a, cfile) in enumerate(((a1, o1), (a2, o2))):
    c = open(cfile, 'rb').read()
    la, lc = a.split(b'\n'), c.split(b'\n')
    assert len(la) == len(lc)
    assert lc[0::4][:-1] == names and set(lc[2::4][:-1]) == {b'+'}
    sa, sc, q = la[1::4][:-1], lc[1::4][:-1], lc[3::4][:-1]
    assert [len(x) for x in sa] == [len(x) for x in sc] == [len(x) for x in q]
    full = [i for i, x in enumerate(sa) if len(x) == rlen]
    SA = np.frombuffer(b''.join(sa[i] for i in full), np.uint8).reshape(-1, rlen)
    SC = np.frombuffer(b''.join(sc[i] for i in full), np.uint8).reshape(-1, rlen)
    Q = np.frombuffer(b''.join(q[i] for i in full), np.uint8).reshape(-1, rlen).astype(np.int64) - 33
    n = len(full)
    for pos in (0, rlen // 2, rlen - 1):
      pmf = np.diff(np.concatenate([[0.0], mdl['cum_bq_mat'][mate, pos, :]]))
      h = np.bincount(Q[:, pos], minlength=94)[:94] / n
      assert np.abs(h - pmf).max() < 4.5 / np.sqrt(n) + 0.005, (mate, pos)
    err = SA != SC
    exp = (10 ** (-Q / 10.0)).mean()
    assert abs(err.mean() - exp) < 0.15 * exp + 5e-4
    assert not np.any(SC[err] == SA[err])
  # chunk size does not change the output
  o1b, o2b = str(tmp_path / 'd1.fq'), str(tmp_path / 'd2.fq')
  readcorrupt.multi_process(mod, mdl, i1, o1b, i2, o2b, seed=11, chunk_bytes=5003, flush_bytes=20000, rng=rng)
  assert open(o1b, 'rb').read() == open(o1, 'rb').read() and open(o2b, 'rb').read() == open(o2, 'rb').read()
  # CLI
  e1, e2 = str(tmp_path / 'e1.fq'), str(tmp_path / 'e2.fq')
  res = CliRunner().invoke(cli, ['corrupt-reads', model + '.pkl', i1, e1, '11', '--fastq2-in', i2, '--fastq2-out', e2,
                                 '--rng', rng])
  assert res.exit_code == 0, res.output + repr(res.exception)
  assert open(e1, 'rb').read() == open(o1, 'rb').read() and open(e2, 'rb').read() == open(o2, 'rb').read()


def test_corrupt_reads_single_end_and_errors(native, tmp_path):
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readcorrupt
  mod, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  i1 = G.path('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz')
  o1 = str(tmp_path / 's.fq')
  readcorrupt.multi_process(mod, mdl, i1, o1, seed=3)
  c = open(o1, 'rb').read()
  assert c.count(b'\n') == G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz').count(b'\n')
  long_read = tmp_path / 'long.fq'
  L = mdl['cum_bq_mat'].shape[1] + 1
  long_read.write_bytes(b'@r1\n' + b'A' * L + b'\n+\n' + b'~' * L + b'\n')
  with pytest.raises(ValueError, match='BQ model'):
    readcorrupt.multi_process(mod, mdl, str(long_read), str(tmp_path / 'x.fq'), seed=3)


# ---- exact corruption: the reference's single-worker MT19937 stream (readcorrupt.py:84, processes=1) ----------------
@pytest.mark.parametrize('chunk', [None, 3001])
@pytest.mark.parametrize('model', G.MODELS)
def test_corrupt_reads_exact_byte_identical_to_reference(native, model, chunk, tmp_path):
  """corrupt-reads --rng mitty on the reference's input pair reproduces the reference's processes=1 output
  (tests/golden/corrupt_*.fq.gz) byte for byte; small chunks carry the stream across calls."""
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readcorrupt
  mod, mdl = get_read_model(model + '.pkl')
  i1, i2 = G.path('corrupt_in_{}.r1.fq.gz'.format(model)), G.path('corrupt_in_{}.r2.fq.gz'.format(model))
  o1, o2 = str(tmp_path / 'c1.fq'), str(tmp_path / 'c2.fq')
  readcorrupt.multi_process(mod, mdl, i1, o1, i2, o2, processes=1, seed=7, chunk_bytes=chunk)
  G.check_same(open(o1, 'rb').read(), G.fastq_bytes('corrupt_{}.r1.fq.gz'.format(model)), 'corrupt file 1')
  G.check_same(open(o2, 'rb').read(), G.fastq_bytes('corrupt_{}.r2.fq.gz'.format(model)), 'corrupt file 2')


def test_corrupt_reads_exact_cli(native, tmp_path):
  from click.testing import CliRunner
  from mitty_amd.cli import cli
  model = 'hiseq-X-v2.5-Garvan'
  i1, i2 = G.path('corrupt_in_{}.r1.fq.gz'.format(model)), G.path('corrupt_in_{}.r2.fq.gz'.format(model))
  e1, e2 = str(tmp_path / 'e1.fq'), str(tmp_path / 'e2.fq')
  res = CliRunner().invoke(cli, ['corrupt-reads', model + '.pkl', i1, e1, '7', '--fastq2-in', i2, '--fastq2-out', e2,
                                 '--threads', '1'])
  assert res.exit_code == 0, res.output + repr(res.exception)
  G.check_same(open(e1, 'rb').read(), G.fastq_bytes('corrupt_{}.r1.fq.gz'.format(model)))
  G.check_same(open(e2, 'rb').read(), G.fastq_bytes('corrupt_{}.r2.fq.gz'.format(model)))


@pytest.mark.parametrize('model', G.MODELS)
def test_corrupt_template_plugin_api_vs_reference(native, model):
  """The plugin functions illumina.corrupt_template / corrupt_single_read (illumina.py:113-162) on a caller's
  RandomState: template by template they reproduce the reference's processes=1 output, and leave the RandomState
  where rand(n), rand(n), randint(0, 3, n) per mate leave it."""
  from mitty_amd.simulation import illumina
  mdl = G.model(model)
  r1 = G.parse_fastq(G.fastq_bytes('corrupt_in_{}.r1.fq.gz'.format(model)))
  r2 = G.parse_fastq(G.fastq_bytes('corrupt_in_{}.r2.fq.gz'.format(model)))
  want1 = G.parse_fastq(G.fastq_bytes('corrupt_{}.r1.fq.gz'.format(model)))
  want2 = G.parse_fastq(G.fastq_bytes('corrupt_{}.r2.fq.gz'.format(model)))
  seed = int(np.random.RandomState(7).randint((1 << 32) - 1))
  rng, shadow = np.random.RandomState(seed), np.random.RandomState(seed)
  for k, (a, b) in enumerate(zip(r1, r2)):
    if k % 7 == 3:   # the single-read form, mate by mate
      got = [(a[0],) + illumina.corrupt_single_read(s, mdl['cum_bq_mat'][m], rng) for m, s in ((0, a[1]), (1, b[1]))]
    else:
      got = illumina.corrupt_template(mdl, [a[0], a[1], b[1]], rng)
    assert got == [want1[k], want2[k]], k
    for s in (a[1], b[1]):
      shadow.rand(len(s))
      shadow.rand(len(s))
      shadow.randint(0, 3, size=len(s))
    st, sh = rng.get_state(), shadow.get_state()
    assert np.array_equal(st[1], sh[1]) and st[2] == sh[2], k
  with pytest.raises(IndexError):
    illumina.corrupt_single_read('A' * 301, mdl['cum_bq_mat'][0], rng)


# ---- counter-based sampling mode (--rng philox) ----------------------------------------------------------------------
def test_philox_sampling_properties(native):
  """--rng philox: deterministic per seed, positions and template lengths inside the reference's support
  (ts > p_min, te < p_max, tlen = max(searchsorted(cum_tlen, U), rlen)), the tlen distribution follows the model's,
  file-order bits are fair, the kept count matches the MT19937 mode's in expectation, and units sampled in one batch
  equal the same units sampled alone."""
  from mitty_amd.simulation import illumina
  mdl = G.model('hiseq-X-v2.5-Garvan')
  rm = illumina.read_model_params(mdl, 30.0)
  rlen, p_min, p_max = 150, 1000, 1000 + 20_000_000
  a = illumina.generate_reads(rm, p_min, p_max, 77, rng='philox')
  b = illumina.generate_reads(rm, p_min, p_max, 77, rng='philox')
  c = illumina.generate_reads(rm, p_min, p_max, 78, rng='philox')
  for k in (0, 1):
    assert np.array_equal(a[k]['pos'], b[k]['pos']) and np.array_equal(a[k]['file_order'], b[k]['file_order'])
  assert not np.array_equal(a[0]['pos'][:1000], c[0]['pos'][:1000])
  ts, te = a[0]['pos'], a[1]['pos'] + rlen
  m = len(ts)
  assert ts.min() > p_min and te.max() < p_max
  tl = te - ts
  assert tl.min() >= rlen and tl.max() <= len(mdl['cum_tlen'])
  want = np.clip(np.searchsorted(mdl['cum_tlen'], (np.arange(100_000) + 0.5) / 100_000), rlen, None)
  grid = np.arange(rlen, len(mdl['cum_tlen']) + 1)
  cdf_got = np.searchsorted(np.sort(tl), grid, side='right') / m
  cdf_want = np.searchsorted(np.sort(want), grid, side='right') / len(want)
  assert np.abs(cdf_got - cdf_want).max() < 0.01
  fo = a[0]['file_order']
  assert set(np.unique(fo)) <= {0, 1} and abs(fo.mean() - 0.5) < 5 / np.sqrt(m)
  assert np.array_equal(a[1]['file_order'], 1 - fo)
  mt = illumina.generate_reads(rm, p_min, p_max, 77)
  assert abs(m - len(mt[0]['pos'])) < 0.02 * m
  assert len(np.unique(ts)) > 0.97 * m   # geometric gaps >= 1: the starts are distinct
  # batched == alone
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  seq = synth.contig(3_000_000, 51)
  copies = synth.copies_soa(synth.variants(seq, 52))
  eng = Engine(0)
  try:
    eng.load_region(0, ('1', 0, len(seq)), seq)
    slots = [eng.haplotype(0, cpy, copies[cpy])[0] for cpy in (0, 1)]
    eng.ctx.sample_units([0, 1], slots, [901, 902], rm['p'], rlen, mdl['cum_tlen'], _native.MH_RNG_PHILOX)
    batched = []
    for k in (0, 1):
      eng.ctx.use_templates(k)
      batched.append(eng.ctx.get_templates())
    for k in (0, 1):
      eng.ctx.sample_units([5], [slots[k]], [901 + k], rm['p'], rlen, mdl['cum_tlen'], _native.MH_RNG_PHILOX)
      eng.ctx.use_templates(5)
      alone = eng.ctx.get_templates()
      for x, y in zip(batched[k], alone):
        assert np.array_equal(x, y)
  finally:
    eng.close()


# ---- device BGZF (mh_deflate.hip) ----------------------------------------------------------
def _bgzf_members(z):
  """The BGZF members of z: (BSIZE, ISIZE) each, checking the gzip header and the BC extra field."""
  out, o = [], 0
  while o < len(z):
    assert z[o:o + 4] == b'\x1f\x8b\x08\x04' and z[o + 12:o + 16] == b'BC\x02\x00', o
    bsize = int.from_bytes(z[o + 16:o + 18], 'little') + 1
    isize = int.from_bytes(z[o + bsize - 4:o + bsize], 'little')
    assert isize <= 0xff00
    out.append((bsize, isize))
    o += bsize
  assert o == len(z)
  return out


@pytest.mark.parametrize('name', ['fastq', 'random', 'zeros', 'one', 'block', 'block1', 'large', 'mixed', 'chunked'])
def test_device_bgzf_round_trip(ctx, name):
  """GPU deflate (a workgroup per BGZF block, eight dynamic-Huffman slices): every member a valid BGZF block, the
  whole inflating (zlib) to the input; incompressible blocks stored; FASTQ about as small as gzip -1.  'chunked':
  more than one launch's 8192 blocks (mh_deflate.hip bgzf_device: slots reused, output appended at the running
  offset across the seam)."""
  import os as _os
  fq = G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz')
  if name == 'chunked':
    n = 8192 * 0xff00 + 3 * 0xff00 + 12345                 # two launches: 8192 + 4 blocks
    noise = _os.urandom(1 << 20)
    data = ((fq + noise) * (n // (len(fq) + len(noise)) + 1))[:n]
  else:
    data = {'fastq': fq, 'random': _os.urandom(300_001), 'zeros': b'\0' * 1_000_000, 'one': b'@',
            'block': fq[:0xff00], 'block1': fq[:0xff01], 'large': (fq * 40)[:25_000_003],
            'mixed': fq[:100_000] + _os.urandom(70_000) + b'~' * 90_000 + fq[:50_000]}[name]
  z = ctx.bgzf_compress(data)
  members = _bgzf_members(z)
  assert sum(m[1] for m in members) == len(data)
  assert len(members) == (len(data) + 0xff00 - 1) // 0xff00
  from mitty_amd import _native
  assert gzip.decompress(z + _native.bgzf_eof()) == data
  if name in ('fastq', 'large'):
    assert len(z) < 1.1 * len(gzip.compress(data[:5_000_000], 1)) * max(1, len(data) / 5_000_000)


def test_device_bgzf_empty(ctx):
  assert ctx.bgzf_compress(b'') == b''


def test_device_bgzf_arena_ranges_equal_whole_arena(native):
  """generate-reads' chunked '.gz' path: ranges of the FASTQ arenas at multiples of 0xff00 deflated on the GPU
  (mh_output_bgzf_range) concatenate to the members of one call over the whole arena (mh_output_bgzf), which inflate
  to the arena's FASTQ."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, _ = _native.read_model_params(mdl['mean_rlen'], 30.0)
  seq = synth.contig(3_000_000, 5)
  copies = synth.copies_soa(synth.variants(seq, 6), 0, len(seq))
  eng = Engine(0)
  try:
    eng.load_region(0, ('7', 0, len(seq)), seq)
    eng.ctx.reset_output()
    eng.run_unit(0, 0, 0, 99, copies[0], p, mdl['mean_rlen'], mdl['cum_tlen'], 'SYN')
    d1, d2 = eng.ctx.fetch_output()
    u1, u2 = eng.ctx.output_size()
    whole = [_native.PinnedBuffer(), _native.PinnedBuffer()]
    w1, w2 = (bytes(v) for v in eng.ctx.output_bgzf_pinned(whole))
    part = [_native.PinnedBuffer(), _native.PinnedBuffer()]
    CH = 7 * 0xff00
    z1, z2 = b'', b''
    for off in range(0, max(u1, u2), CH):
      a, b = eng.ctx.output_bgzf_range_pinned(part, off, max(0, min(CH, u1 - off)), max(0, min(CH, u2 - off)))
      z1, z2 = z1 + bytes(a), z2 + bytes(b)
    assert z1 == w1 and z2 == w2
    eof = _native.bgzf_eof()
    assert gzip.decompress(z1 + eof) == d1 and gzip.decompress(z2 + eof) == d2
    with pytest.raises(ValueError):
      eng.ctx.output_bgzf_range_pinned(part, u1 - 10, 20, 0)   # past the arena
  finally:
    eng.close()


def test_scan_timeout_is_reported(ctx, native):
  """A look-back scan whose tile 0 never runs: the timed-out waits are reported (MH_E_STATE) instead of a fabricated
  zero prefix returned as success, and a correct scan after it succeeds (mh_scan.h's bounded wait)."""
  rc, msg = ctx.selftest_scan_fault()
  assert rc == native.MH_E_STATE, (rc, msg)
  assert 'timed out' in msg
  ctx.sync()   # the fault word was cleared by the report


@pytest.mark.parametrize('bits', [1, 9, 10, 18, 27, 32])
def test_lsd_sort_equals_stable_argsort(ctx, bits):
  """The permutation's radix sort (mh_sort.h, mh_selftest_sort) against numpy's stable argsort: key and index arrays
  equal, for sizes around the 8192-key tile (empty, one key, a partial tile, whole tiles, one past) and a
  multi-pass size, keys below 2^bits (few distinct values for small bits: long runs of equal keys keep their order)."""
  rng = np.random.default_rng(bits)
  for n in (0, 1, 5, 8191, 8192, 8193, 3 * 8192 + 17, 1_000_003):
    hi = (1 << bits) if bits < 32 else (1 << 32)
    k = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
    ko, vo = ctx.selftest_sort(k, bits)
    order = np.argsort(k, kind='stable')
    assert np.array_equal(vo, order.astype(np.uint32)), (bits, n)
    assert np.array_equal(ko, k[order]), (bits, n)


# ---- the single-pass writer (k_emit_fused) ---------------------------------------------------------------------
def _dense_records(seq, seed, start0, end):
  """Variants far denser than any VCF (test input): one every 2-12 bp; 60 % SNVs, 20 % insertions (2 % of them
  300-700 bp, so reads fall inside them: '>p:nI'), 20 % deletions (2 % of them 200-1500 bp: 4-digit CIGAR counts),
  GT 0|1 / 1|0 / 1|1.  Reads then span tens of nodes (the writer's node loop past its four preloaded nodes)."""
  rs = np.random.RandomState(seed)
  arr = np.frombuffer(seq, dtype=np.uint8)
  pos0 = start0 + np.cumsum(rs.randint(2, 13, size=(end - start0) // 4))
  pos0 = pos0[pos0 < end - 2000]
  pos0 = pos0[arr[pos0] != ord('N')]
  n = len(pos0)
  kind = rs.choice(3, size=n, p=[0.6, 0.2, 0.2])
  ln = 1 + rs.geometric(0.35, size=n)
  big = rs.rand(n) < 0.02
  ln[big & (kind == 1)] = rs.randint(300, 701, size=int((big & (kind == 1)).sum()))
  ln[big & (kind == 2)] = rs.randint(200, 1501, size=int((big & (kind == 2)).sum()))
  gt = np.array([[0, 1], [1, 0], [1, 1]], dtype=np.int8)[rs.choice(3, size=n)]
  ref_len = np.where(kind == 2, ln + 1, 1).astype(np.int64)
  acgt = np.frombuffer(b'ACGT', dtype=np.uint8)
  alts = []
  for i in range(n):
    b = seq[pos0[i]:pos0[i] + 1]
    if kind[i] == 0:
      alts.append(b'A' if b != b'A' else b'C')
    elif kind[i] == 1:
      alts.append(b + acgt[rs.randint(0, 4, size=int(ln[i]))].tobytes())
    else:
      alts.append(b)
  return {'pos': pos0.astype(np.int64) + 1, 'ref_len': ref_len, 'alt': alts, 'gt': gt}


@pytest.mark.parametrize('model', G.MODELS)
def test_single_pass_writer_dense_variants_vs_oracle(native, model):
  """mh_emit_reads_async's two writers — the chained two-pass path (mode 0: measure pass, tile scan and writer
  queued with no host readback, offsets passed on the device) and the single-pass writer (mode 3, k_emit_fused: no
  measure pass, tile offsets by a decoupled look-back) — with qname rows and arena reservation sized by the splice's
  bound (k_part_bound), on haplotypes far denser than any VCF, both read models (2x150, 2x250), N runs, reads inside
  long insertions.  Every unit's FASTQ equal to the oracle's (readgenerate.py:184-230, rpc.py:119-160) and to the
  host-readback path's (mode 2) bytes; the queued units' totals equal; the single-pass run had no measure pass."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model(model)
  rlen = int(mdl['mean_rlen'])
  p, passes = _native.read_model_params(rlen, 30.0)
  L = 400_000
  seq = synth.contig(L, 31)
  copies = synth.copies_soa(_dense_records(seq, 32, 0, L))
  units = _native.work_units(9, [2], passes)
  job = [(ps, 0, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)]
  outs = {}
  for mode in (0, 2, 3):
    eng = Engine(0)
    try:
      eng.ctx.set_emit_mode(mode)
      eng.ctx.enable_timing(True)
      eng.load_region(0, ('3', 0, L), seq)
      res = eng.run_units(job, lambda r, c: copies[c], p, rlen, mdl['cum_tlen'], 'DNS')
      d1, d2 = eng.ctx.fetch_output()
      names = {nm for nm, _ in eng.ctx.stage_times()}
    finally:
      eng.close()
    outs[mode] = (res, d1, d2)
    assert ('emit_measure' in names) == (mode != 3), names
  for mode in (2, 3):
    assert outs[0][0] == outs[mode][0]
    G.check_same(outs[0][1], outs[mode][1])
    G.check_same(outs[0][2], outs[mode][2])
  o1, o2 = [], []
  for ps, _, cpy, sd in job:
    k, b1, b2 = O.generate_unit_soa(seq, 0, copies[cpy], p, rlen, mdl['cum_tlen'], sd, 'DNS:0:{}'.format(ps), '3', cpy)
    assert outs[0][0][ps][1] == k and k > 500
    o1.append(b1)
    o2.append(b2)
  G.check_same(outs[0][1], b''.join(o1))
  G.check_same(outs[0][2], b''.join(o2))
  assert b'>' in outs[0][1] and b'I|' in outs[0][1]   # reads inside long insertions were among them


@pytest.mark.parametrize('mode', [0, 3])
def test_single_pass_writer_chain_across_resets_and_fallback(native, mode):
  """Units queued on the single-pass chain across an mh_output_reset (the next chain starts at 0; the earlier units'
  totals still collected in order), a unit the single-pass writer does not take (a sample name too long for its
  qname head: the two-pass path inside mh_emit_reads_async, at the chain's exact end) and an arena fetch in the middle
  (which resolves the chain): the bytes after each reset equal the oracle's concatenation."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 30.0)
  L = 600_000
  seq = synth.contig(L, 41)
  copies = synth.copies_soa(synth.variants(seq, 42))
  units = _native.work_units(17, [2], passes)
  job = [(ps, 0, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)]
  long_name = 'S' * 120
  eng = Engine(0, mode)
  try:
    eng.load_region(0, ('2', 0, L), seq)
    eng.run_units(job[:2], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'A', lazy=True)
    first = eng.ctx.fetch_output()
    eng.ctx.reset_output()
    eng.run_units(job[2:], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'A', lazy=True)
    eng.run_units(job[:1], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], long_name, lazy=True)
    eng.run_units(job[1:2], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'A', lazy=True)
    res = eng.collect()
    second = eng.ctx.fetch_output()
  finally:
    eng.close()

  def oracle(part, name):
    o = [O.generate_unit_soa(seq, 0, copies[cpy], p, 150, mdl['cum_tlen'], sd, '{}:0:{}'.format(name, ps), '2', cpy)
         for ps, _, cpy, sd in part]
    return o

  o_first = oracle(job[:2], 'A')
  o_second = oracle(job[2:], 'A') + oracle(job[:1], long_name) + oracle(job[1:2], 'A')
  assert [r[1:] for r in res] == [(k, len(b1), len(b2)) for k, b1, b2 in o_first + o_second]
  G.check_same(first[0], b''.join(o[1] for o in o_first))
  G.check_same(first[1], b''.join(o[2] for o in o_first))
  G.check_same(second[0], b''.join(o[1] for o in o_second))
  G.check_same(second[1], b''.join(o[2] for o in o_second))


@pytest.mark.parametrize('mode', [1, 2])
def test_emit_async_fallback_modes_vs_oracle(native, mode):
  """mh_emit_reads_async for units it hands to mh_emit_reads' path inside the call (mh_set_emit_mode 1: the LDS-image
  writer; 2: the two-pass path with its host readback), queued among chained units of the default mode: the totals
  come back in queue order from mh_emit_collect and the arenas hold the oracle's bytes; mh_emit_collect with too
  little room fails (MH_E_CAPACITY) and keeps the totals for the next call."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from oracle import oracle as O
  mdl = G.model('hiseq-X-v2.5-Garvan')
  p, passes = _native.read_model_params(150, 30.0)
  L = 400_000
  seq = synth.contig(L, 51)
  copies = synth.copies_soa(synth.variants(seq, 52))
  units = _native.work_units(23, [2], passes)
  job = [(ps, 0, cpy, sd) for ps, (ri, cpy, sd) in enumerate(units)]
  eng = Engine(0)
  try:
    eng.load_region(0, ('4', 0, L), seq)
    eng.run_units(job[:1], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'F', lazy=True)
    eng.ctx.set_emit_mode(mode)
    eng.run_units(job[1:3], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'F', lazy=True)
    eng.ctx.set_emit_mode(0)
    eng.run_units(job[3:], lambda r, c: copies[c], p, 150, mdl['cum_tlen'], 'F', lazy=True)
    import ctypes
    n = ctypes.c_int64()
    out = np.zeros(3, np.int64)
    rc = eng.ctx._L.mh_emit_collect(eng.ctx._h, out.ctypes.data_as(ctypes.c_void_p), 1, ctypes.byref(n))
    assert rc == native.MH_E_CAPACITY and n.value == len(job), (rc, n.value)
    res = eng.collect()
    d1, d2 = eng.ctx.fetch_output()
  finally:
    eng.close()
  o = [O.generate_unit_soa(seq, 0, copies[cpy], p, 150, mdl['cum_tlen'], sd, 'F:0:{}'.format(ps), '4', cpy)
       for ps, _, cpy, sd in job]
  assert [r[1:] for r in res] == [(k, len(b1), len(b2)) for k, b1, b2 in o]
  G.check_same(d1, b''.join(x[1] for x in o))
  G.check_same(d2, b''.join(x[2] for x in o))
