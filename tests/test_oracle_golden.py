"""The CPU oracle (oracle/mitty_oracle.c) against vectors captured from the reference itself.

This pins the oracle before anything else trusts it (tests/golden/make_golden.py captured every vector here).
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_io as G


@pytest.fixture(scope='module')
def rng():
  return G.load_json('rng.json')


@pytest.mark.parametrize('seed', ['0', '1', '7', '12345', '327741615', '4294967295'])
def test_mt19937_words(rng, seed):
  d = rng[seed]
  assert O.mt_words(int(seed), len(d['words'])).tolist() == d['words']


def test_read_model_params(rng):
  for m, by_cov in rng['read_model_params'].items():
    mdl = G.model(m)
    for cov, want in by_cov.items():
      p, passes = O.read_model_params(mdl['mean_rlen'], float(cov))
      assert p.hex() == want['p'] and passes == want['passes'] and want['rlen'] == mdl['mean_rlen']


def test_work_units():
  for key, d in G.load_json('units.json').items():
    seed, passes = map(int, key.split(':'))
    got = [list(u) for u in O.work_units(seed, d['ploidy'], passes)]
    assert got == d['units'], key


def test_templates():
  t = G.templates()
  keys = sorted({k.rsplit('|', 1)[0] for k in t.files})
  for key in keys:
    m, seed, p_min, p_max = key.split('|')
    mdl = G.model(m)
    p, _ = O.read_model_params(mdl['mean_rlen'], 30.0)
    fo, p0, p1 = O.generate_templates(p, int(mdl['mean_rlen']), mdl['cum_tlen'], int(p_min), int(p_max), int(seed))
    assert np.array_equal(fo, t[key + '|fo0']), key
    assert np.array_equal(p0, t[key + '|pos0']), key
    assert np.array_equal(p1, t[key + '|pos1']), key


def _vl(variants):
  return [O.Variant(*v) for v in variants]


def test_node_lists():
  seqs = {'syn': O.read_fasta(G.path('data/syn.fa')), 'tiny': O.read_fasta(G.path('data/tiny.fasta'))}
  nodes = G.load_json('nodes.json')
  assert len(nodes) >= 8
  for key, d in nodes.items():
    tag = key.split('|')[0]
    chrom, s0, e = d['region']
    got = O.create_node_list(seqs[tag][chrom][s0:e], s0 + 1, _vl(d['variants']))
    assert [list(n) for n in got] == d['nodes'], key


def test_variant_loading_matches_reference():
  nodes = G.load_json('nodes.json')
  vdf = O.load_variant_file(G.path('data/syn.vcf'), 'S1', G.path('data/syn.bed'))
  for ri, reg in enumerate(vdf):
    for cpy, vl in enumerate(reg['v']):
      assert [list(v.tuple()) for v in vl] == nodes['syn|{}|{}'.format(ri, cpy)]['variants']


def test_reference_unit_tests_vcfio():
  """Restates mitty/test/lib/test_vcfio.py:9-62 on the same fixture files."""
  v = O.load_variant_file(G.path('data/tiny.vcf'), 'g0_s0', G.path('data/tiny.8-14.bed'))
  assert v[0]['v'][1][0].tuple() == (11, 'CAA', 'C', 'D', 2)
  assert v[0]['v'][0][0].tuple() == (14, 'G', 'T', 'X', 0)
  assert len(v[0]['v'][0]) == 1
  with pytest.raises(ValueError):
    O.load_variant_file(G.path('data/flawed-tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))


@pytest.mark.parametrize('model', G.MODELS)
def test_e2e_fastq_byte_identical(model):
  c = G.load_json('e2e_config.json')[model]
  mdl = G.model(model)
  b1, b2, n = O.generate_reads_fastq(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mdl,
                                     c['coverage'], c['seed'])
  G.check_same(b1, G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)))
  G.check_same(b2, G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model)))


@pytest.mark.parametrize('model', G.MODELS)
def test_corruption_exact(model):
  r1 = G.parse_fastq(G.fastq_bytes('corrupt_in_{}.r1.fq.gz'.format(model)))
  r2 = G.parse_fastq(G.fastq_bytes('corrupt_in_{}.r2.fq.gz'.format(model)))
  b1, b2 = O.corrupt_fastq(G.model(model), [r[0] for r in r1], [r[1] for r in r1], [r[1] for r in r2], seed=7)
  G.check_same(b1, G.fastq_bytes('corrupt_{}.r1.fq.gz'.format(model)))
  G.check_same(b2, G.fastq_bytes('corrupt_{}.r2.fq.gz'.format(model)))


# ---- god-aligner (oracle/god.py) ------------------------------------------------------------------------------
def test_god_records_match_reference():
  """write_perfect_reads attributes (tests/golden/god.json, captured from the reference) from the e2e FASTQs."""
  from oracle import god
  want = {}
  for qn, recs in G.load_json('god.json'):
    want.setdefault(qn, []).append(recs)
  ref_dict = {'1': 0, '2': 1, '3': 2}
  hit = 0
  for m in G.MODELS:
    l1 = G.fastq_bytes('e2e_{}.r1.fq.gz'.format(m)).decode().split('\n')
    l2 = G.fastq_bytes('e2e_{}.r2.fq.gz'.format(m)).decode().split('\n')
    for i in range(len(l1) // 4):
      qn = l1[4 * i][1:]
      if qn not in want:
        continue
      got = god.perfect_reads(qn, ref_dict, [(l1[4 * i + 1], l1[4 * i + 3]), (l2[4 * i + 1], l2[4 * i + 3])])
      assert got in want[qn]
      hit += 1
  assert hit >= len(G.load_json('god.json'))


def test_god_encode_decode_roundtrip():
  from oracle import god
  for qn, recs in G.load_json('god.json')[:60]:
    for r in recs:
      d = god.decode(god.encode(r))
      assert {k: d[k] for k in r} == r
      assert d['bin'] == god.reg2bin(r['pos'], god.end_pos(r))


def test_god_header_text():
  from mitty_amd.benchmarking import god_aligner as ga
  hdr = {'HD': {'VN': '1.0'}, 'PG': [{'CL': 'mitty god-aligner x', 'ID': 'mitty-god-aligner', 'PN': 'god-aligner',
                                      'VN': '2.7.3.dev0'}],
         'RG': [{'ID': b'bWl0dHk=', 'SM': None}], 'SQ': G.load_json('god_header.json')}
  assert ga.header_text(hdr) == ('@HD\tVN:1.0\tSO:coordinate\n@SQ\tSN:1\tLN:50000\n@SQ\tSN:2\tLN:20000\n'
                                 '@SQ\tSN:3\tLN:8000\n@RG\tID:b\'bWl0dHk=\'\tSM:None\n'
                                 '@PG\tPN:god-aligner\tID:mitty-god-aligner\tVN:2.7.3.dev0\tCL:mitty god-aligner x\n')


def test_god_parse_ann(tmp_path):
  from mitty_amd.benchmarking import god_aligner as ga
  ann = tmp_path / 'x.ann'
  ann.write_text('1 1 11\n0 1 (null)\n0 50000 0\n0 2 (null)\n0 20000 0\n0 3 (null)\n0 8000 0\n')
  assert ga.parse_ann(str(ann)) == G.load_json('god_header.json')
