"""CPU-side checks: the C-ABI library loads and exports every declared symbol; host-side logic (model loading,
VCF parsing, work units, qname codec) against the reference's golden vectors.  No GPU compute here."""
import os
import re

import numpy as np
import pytest

from mitty_amd import _native, readmodel
from mitty_amd.lib import vcfio
from mitty_amd.simulation import readgenerate
from tests import golden_io as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
  with open(os.path.join(REPO, 'include', 'mitty_hip.h')) as fp:
    txt = fp.read()
  return sorted(set(re.findall(r'\b(mh_[a-z_0-9]+)\s*\(', txt)))


def test_header_matches_binding_list():
  assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_every_declared_symbol():
  import ctypes
  L = _native.lib()
  for name in _declared():
    assert hasattr(L, name), name
    assert isinstance(getattr(L, name), ctypes._CFuncPtr)
  assert L.mh_version() == 1


def test_library_is_gfx950_code_object():
  import subprocess
  out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', _native.LIB_PATH],
                       capture_output=True, text=True, cwd='/tmp')
  if out.returncode != 0:
    pytest.skip('llvm-objdump --offloading unavailable')
  assert 'gfx950' in out.stdout + out.stderr


def test_work_units_host_abi():
  for key, d in G.load_json('units.json').items():
    seed, passes = map(int, key.split(':'))
    got = [list(u) for u in _native.work_units(seed, d['ploidy'], passes)]
    assert got == d['units'], key


def test_read_model_params_host_abi():
  rng = G.load_json('rng.json')
  for m, by_cov in rng['read_model_params'].items():
    mdl = G.model(m)
    for cov, want in by_cov.items():
      p, passes = _native.read_model_params(mdl['mean_rlen'], float(cov))
      assert p.hex() == want['p'] and passes == want['passes']


def test_work_units_bad_seed():
  with pytest.raises(ValueError):
    _native.work_units(1 << 32, [2], 2)


def test_safe_model_parser_matches_builtin():
  mods = readmodel.builtin_models()
  assert 'hiseq-X-v2.5-Garvan.pkl' in mods and '1kg-pcr-free.pkl' in mods and len(mods) == 5
  _, m = readmodel.get_read_model('hiseq-X-v2.5-Garvan.pkl')
  assert m['mean_rlen'] == 150 and m['cum_bq_mat'].shape == (2, 300, 94) and m['cum_tlen'][-1] == 1.0
  _, m = readmodel.get_read_model('1kg-pcr-free.pkl')
  assert m['mean_rlen'] == 250


def test_safe_model_parser_refuses_code(tmp_path):
  import pickle

  class Evil:
    def __reduce__(self):
      return (os.system, ('echo pwned',))
  p = tmp_path / 'evil.pkl'
  p.write_bytes(pickle.dumps({'x': Evil()}, protocol=3))
  with pytest.raises(readmodel.UnsafeModelError):
    readmodel.load_model_file(str(p))


def test_safe_model_parser_roundtrip(tmp_path):
  import pickle
  m = {'model_class': 'illumina', 'model_description': 'x', 'mean_rlen': 100, 'r_cnt': 10 ** 12,
       'cum_tlen': np.linspace(0, 1, 7), 'bq_mat': np.arange(24, dtype=np.uint64).reshape(2, 3, 4)}
  p = tmp_path / 'm.pkl'
  p.write_bytes(pickle.dumps(m, protocol=3))
  got = readmodel.load_model_file(str(p))
  assert got['mean_rlen'] == 100 and got['r_cnt'] == 10 ** 12 and got['model_class'] == 'illumina'
  assert np.array_equal(got['cum_tlen'], m['cum_tlen']) and np.array_equal(got['bq_mat'], m['bq_mat'])


def test_vcf_loading_matches_reference():
  nodes = G.load_json('nodes.json')
  for vcf in ('syn.vcf', 'syn.vcf.gz'):
    vdf = vcfio.load_variant_file(G.path('data', vcf), 'S1', G.path('data/syn.bed'))
    for ri, reg in enumerate(vdf):
      for cpy, vl in enumerate(reg['v']):
        assert [list(v.tuple()) for v in vl] == nodes['syn|{}|{}'.format(ri, cpy)]['variants']
  soa = vcfio.load_variants_soa(G.path('data/syn.vcf'), 'S1', G.path('data/syn.bed'))
  assert [r['ploidy'] for r in soa] == [2, 2, 2, 1]


def test_vcfio_reference_unit_tests():
  """mitty/test/lib/test_vcfio.py:9-62 restated."""
  v = vcfio.load_variant_file(G.path('data/tiny.vcf'), 'g0_s0', G.path('data/tiny.8-14.bed'))
  assert v[0]['v'][1][0].tuple() == (11, 'CAA', 'C', 'D', 2)
  assert v[0]['v'][0][0].tuple() == (14, 'G', 'T', 'X', 0)
  assert len(v[0]['v'][0]) == 1
  with pytest.raises(ValueError):
    vcfio.load_variants_soa(G.path('data/flawed-tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))
  v = vcfio.load_variant_file(G.path('data/tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))
  assert (v[0]['v'][1][0].cigarop, v[0]['v'][1][0].oplen) == ('X', 0)
  assert (v[0]['v'][1][1].cigarop, v[0]['v'][1][1].oplen) == ('I', 3)
  assert (v[0]['v'][1][2].cigarop, v[0]['v'][1][2].oplen) == ('D', 2)


def test_parse_qname_matches_reference():
  for qn, want in G.load_json('qnames.json'):
    got = [list(r) for r in readgenerate.parse_qname(qn)]
    assert got == want


def test_native_fails_loudly_without_library(monkeypatch):
  monkeypatch.setattr(_native, '_lib', None)
  monkeypatch.setattr(_native, 'LIB_PATH', '/nonexistent/libmitty_hip.so')
  with pytest.raises(_native.NativeUnavailable):
    _native.Context(0)


def test_no_device_raises_here():
  if _native.device_count() > 0:
    pytest.skip('a GPU is visible')
  with pytest.raises(_native.NativeUnavailable):
    _native.Context(0)


def _raw_mt(seed, n):
  x = np.zeros(n, dtype=np.uint64)
  x[0] = seed
  for i in range(1, 624):
    x[i] = (1812433253 * (int(x[i - 1]) ^ (int(x[i - 1]) >> 30)) + i) & 0xffffffff
  xs = [int(v) for v in x[:624]]
  for t in range(624, n):
    y = (xs[t - 624] & 0x80000000) | (xs[t - 623] & 0x7fffffff)
    xs.append(xs[t - 227] ^ (y >> 1) ^ (0x9908b0df if y & 1 else 0))
  return xs


@pytest.mark.parametrize('seed', [7, 327741615, 4294967295])
def test_mt19937_jump_ahead_host(seed):
  """The jump polynomial x^J mod P (host GF(2) math the device segments use) lands on the same window as the plain
  recurrence, at offsets inside and across twist blocks."""
  xs = _raw_mt(seed, 200_000 + 624)
  for J in (0, 1, 623, 624, 1000, 12345, 199_680):
    w = _native.mt_window_at(seed, J)
    assert (int(w[0]) >> 31) == (xs[J] >> 31)
    assert [int(v) for v in w[1:]] == xs[J + 1:J + 624], J


# ---- compressed FASTQ sink (host BGZF, no device) -------------------------------------------------------------------
@pytest.mark.parametrize('n', [0, 1, 65279, 65280, 65281, 1_000_003])
def test_bgzf_compress_roundtrip(n):
  import gzip
  import os
  data = (os.urandom(n // 3) + b'ACGTN\n+\n~~~' * (n // 10 + 1))[:n]
  z = _native.bgzf_compress(data, level=6, threads=3) + _native.bgzf_eof()
  assert gzip.decompress(z) == data
  from oracle import god
  blocks = god.bgzf_blocks(z)          # framing + CRC of every block
  assert all(len(raw) <= 0xff00 for _, raw in blocks) and blocks[-1][1] == b''


def test_fastq_sink_gz(tmp_path):
  import gzip
  from mitty_amd.lib.fastq_stream import FastqSink
  s = FastqSink(str(tmp_path / 'a.fq.gz'), threads=2)
  parts = [b'@r%d\nACGT\n+\n~~~~\n' % i * 5000 for i in range(3)]
  for p in parts:
    s.write(p)
  s.close()
  assert gzip.open(str(tmp_path / 'a.fq.gz')).read() == b''.join(parts)
  s = FastqSink(str(tmp_path / 'b.fq'))
  s.write(parts[0])
  s.close()
  assert open(str(tmp_path / 'b.fq'), 'rb').read() == parts[0]


# ---- native VCF reader (mh_vcf.cpp) vs the Python restatement --------------------------------------------------------
@pytest.mark.parametrize('vcf,sample,bed', [('data/syn.vcf', 'S1', 'data/syn.bed'), ('data/syn.vcf.gz', 'S1', 'data/syn.bed'),
                                            ('data/syn.vcf', 'S0', 'data/syn.bed'),
                                            ('data/tiny.vcf', 'g0_s0', 'data/tiny.whole.bed'),
                                            ('data/tiny.vcf', 'g0_s0', 'data/tiny.8-14.bed')])
def test_native_vcf_matches_restatement(vcf, sample, bed):
  a = vcfio.load_variants_soa(G.path(vcf), sample, G.path(bed))
  b = vcfio._load_records_soa(G.path(vcf), sample, G.path(bed))
  assert len(a) == len(b)
  for ra, rb in zip(a, b):
    assert ra['region'] == rb['region'] and ra['ploidy'] == rb['ploidy']
    for ca, cb in zip(ra['copies'], rb['copies']):
      for k in ('pos', 'op', 'oplen', 'alt_off', 'alt_len'):
        assert np.array_equal(ca[k], cb[k]), k
      assert ca['alt_pool'] == cb['alt_pool']


def test_native_vcf_errors(tmp_path):
  with pytest.raises(ValueError, match='sample'):
    vcfio.load_variants_soa(G.path('data/syn.vcf'), 'nobody', G.path('data/syn.bed'))
  with pytest.raises(ValueError, match='Complex'):
    vcfio.load_variants_soa(G.path('data/flawed-tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))
  v = tmp_path / 'end.vcf'   # INFO END= widens the overlap span (htslib rlen)
  v.write_text('##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS\n'
               '1\t5\t.\tA\tG\t.\t.\tEND=20\tGT\t1|0\n1\t30\t.\tC\tT\t.\t.\t.\tGT\t0|1\n')
  b = tmp_path / 'r.bed'
  b.write_text('1\t15\t40\n')
  r = vcfio.load_variants_soa(str(v), 'S', str(b))[0]
  assert r['ploidy'] == 2 and list(r['copies'][0]['pos']) == [5] and list(r['copies'][1]['pos']) == [30]


def test_mitty_console_entry_point(tmp_path):
  """setup.py declares the reference's console command (`mitty = ...cli:cli`, reference setup.py:12) and
  `python -m mitty_amd` runs the same click group (the qname subcommand prints the reference's format text)."""
  import subprocess
  import sys
  repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  subprocess.check_call([sys.executable, 'setup.py', '-q', 'egg_info', '--egg-base', str(tmp_path)], cwd=repo,
                        stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
  eps = open(os.path.join(str(tmp_path), 'mitty_mi355x.egg-info', 'entry_points.txt')).read()
  assert 'mitty = mitty_amd.cli:cli' in eps
  out = subprocess.check_output([sys.executable, '-m', 'mitty_amd', 'qname'], cwd=repo).decode()
  from mitty_amd.simulation.readgenerate import __qname_format_details__
  assert out.strip() == __qname_format_details__.strip()
  out = subprocess.check_output([sys.executable, '-m', 'mitty_amd', 'generate-reads', '--help'], cwd=repo).decode()
  assert '--fastq2' in out and '--threads' in out


def test_host_cpp_under_asan_ubsan(tmp_path):
  """the host C++ that parses untrusted VCF (mh_vcf.cpp) and writes into caller buffers and files
  (mh_bgzf.cpp: BGZF, BAM framing, BAI) built with -fsanitize=address,undefined and driven over the golden VCFs,
  mutated / truncated VCFs (plain and gzip), empty and exact-capacity compression buffers: no sanitizer report."""
  import gzip
  import shutil
  import subprocess
  if shutil.which('g++') is None:
    pytest.skip('no g++')
  exe = str(tmp_path / 'san_driver')
  subprocess.check_call(['g++', '-std=c++17', '-O1', '-g', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
                         '-fno-sanitize-recover=undefined', os.path.join(REPO, 'tests', 'sanitize', 'san_driver.cpp'),
                         os.path.join(REPO, 'mitty_amd', 'csrc', 'mh_vcf.cpp'),
                         os.path.join(REPO, 'mitty_amd', 'csrc', 'mh_bgzf.cpp'), '-lz', '-lpthread', '-o', exe])
  src = open(G.path('data/syn.vcf'), 'rb').read()
  rs = np.random.RandomState(5)
  cmds = []
  for k in range(40):
    b = bytearray(src)
    kind = k % 5
    if kind == 0:     # truncated anywhere
      b = b[:rs.randint(0, len(b))]
    elif kind == 1:   # random byte flips
      for _ in range(20):
        b[rs.randint(len(b))] = rs.randint(256)
    elif kind == 2:   # fields dropped from random lines
      lines = bytes(b).split(b'\n')
      for _ in range(10):
        i = rs.randint(len(lines))
        f = lines[i].split(b'\t')
        lines[i] = b'\t'.join(f[:rs.randint(0, len(f) + 1)])
      b = bytearray(b'\n'.join(lines))
    elif kind == 3:   # absurd numbers / genotypes
      b = bytearray(bytes(b).replace(b'\t0|1', b'\t0|99').replace(b'\t1|0', b'\t.|-3').replace(b'1\t1', b'1\t99999999999999999999', 3))
    else:             # a gzip member cut short
      b = bytearray(gzip.compress(bytes(b))[:rs.randint(10, 2000)])
    fn = str(tmp_path / 'm{}.vcf'.format(k))
    open(fn, 'wb').write(bytes(b))
    for chrom, s0, e in (('1', 0, 60000), ('2', 100, 20000), ('3', 0, 10 ** 12)):
      cmds.append('vcf {} S1 {} {} {}'.format(fn, chrom, s0, e))
  for v, s, bed in (('syn.vcf', 'S1', 'syn.bed'), ('syn.vcf.gz', 'S1', 'syn.bed'), ('tiny.vcf', 'g0_s0', 'tiny.whole.bed'),
                    ('flawed-tiny.vcf', 'g0_s0', 'tiny.whole.bed'), ('syn.vcf', 'NOPE', 'syn.bed')):
    local = str(tmp_path / v)   # filter-variants writes <vcf>.filt.vcf next to its input
    shutil.copy(G.path('data', v), local)
    for line in open(G.path('data', bed)):
      chrom, s0, e = line.split()[:3]
      cmds.append('vcf {} {} {} {} {}'.format(local, s, chrom, s0, e))
  cmds += ['bgzf {} {} {} {}'.format(n, lvl, th, n) for n, lvl, th in
           ((0, 6, 1), (1, 0, 1), (65280, 1, 2), (65281, 9, 3), (300000, 6, 8))]
  cmds += ['bam {} {} {}'.format(tmp_path / 'b{}.bam'.format(n), n, n) for n in (0, 1, 5000)]
  env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0', UBSAN_OPTIONS='print_stacktrace=1')
  env.pop('LD_PRELOAD', None)
  r = subprocess.run([exe], input='\n'.join(cmds).encode(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env,
                     timeout=600)
  err = r.stderr.decode(errors='replace')
  assert r.returncode == 0 and 'ERROR: AddressSanitizer' not in err and 'runtime error' not in err, err[-4000:]
  assert r.stdout.count(b'\n') >= len(cmds)


@pytest.mark.parametrize('out_name', ['out.vcf', 'out.vcf.gz'])
def test_filter_variants_matches_reference(tmp_path, out_name):
  """filter-variants (vcfio.prepare_variant_file, vcfio.py:129-168) keeps exactly the records the reference writes
  (tests/golden/filter_variants.json, captured by make_golden_filter.py): BED order, records in two overlapping
  regions written twice, complex calls of the sample's genotype dropped, INFO END spans, haploid / missing GTs on
  single-base records.  Header text is parity-unpinned (htslib re-serialises it; no htslib here)."""
  import gzip
  from click.testing import CliRunner
  from mitty_amd.cli import cli
  want = G.load_json('filter_variants.json')
  out = str(tmp_path / out_name)
  res = CliRunner().invoke(cli, ['filter-variants', G.path('data/filt.vcf'), 'S1', G.path('data/filt.bed'), out])
  assert res.exit_code == 0, res.output + repr(res.exception)
  raw = open(out, 'rb').read()
  text = (gzip.decompress(raw) if out_name.endswith('.gz') else raw).decode()
  lines = text.rstrip('\n').split('\n')
  head = [ln for ln in lines if ln.startswith('#')]
  assert head[-1].split('\t')[9:] == ['S1'] and head[0] == '##fileformat=VCFv4.1'
  recs = [ln.split('\t') for ln in lines if not ln.startswith('#')]
  assert all(len(f) == 10 for f in recs)
  assert [[f[0], int(f[1]), f[2], f[3], f[4], f[9]] for f in recs] == want['records']
  w, f = vcfio.prepare_variant_file(G.path('data/filt.vcf'), 'S1', G.path('data/filt.bed'), str(tmp_path / 'b.vcf'))
  assert w == len(want['records']) and f > 0


def test_filter_variants_errors(tmp_path):
  bad = tmp_path / 'bad.vcf'
  bad.write_text('##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n'
                 '1\t5\t.\tAC\tA\t50\tPASS\t.\tGT\t.|1\n')
  bed = tmp_path / 'b.bed'
  bed.write_text('1\t0\t100\n')
  with pytest.raises(ValueError, match='missing genotype'):
    vcfio.prepare_variant_file(str(bad), 'S1', str(bed), str(tmp_path / 'o.vcf'))
  with pytest.raises(ValueError, match='sample'):
    vcfio.prepare_variant_file(str(bad), 'NOPE', str(bed), str(tmp_path / 'o.vcf'))
  # a BED contig the VCF knows neither from ##contig nor from records: pysam's fetch raises ValueError('invalid
  # contig'); a declared contig without records is an empty region
  ok = tmp_path / 'ok.vcf'
  ok.write_text('##fileformat=VCFv4.1\n##contig=<ID=2,length=100>\n'
                '#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n1\t5\t.\tA\tC\t50\tPASS\t.\tGT\t0|1\n')
  (tmp_path / 'c3.bed').write_text('1\t0\t100\n3\t0\t100\n')
  with pytest.raises(ValueError, match='invalid contig `3`'):
    vcfio.prepare_variant_file(str(ok), 'S1', str(tmp_path / 'c3.bed'), str(tmp_path / 'o.vcf'))
  (tmp_path / 'c2.bed').write_text('1\t0\t100\n2\t0\t100\n')
  assert vcfio.prepare_variant_file(str(ok), 'S1', str(tmp_path / 'c2.bed'), str(tmp_path / 'o.vcf'))[0] == 1
  # the generate-reads load path (load_variant_file, vcfio.py:62 — the same fetch) rejects the unknown contig too, and
  # a declared contig without records is an empty diploid region
  with pytest.raises(ValueError, match='invalid contig `3`'):
    vcfio.load_variants_soa(str(ok), 'S1', str(tmp_path / 'c3.bed'))
  r = vcfio.load_variants_soa(str(ok), 'S1', str(tmp_path / 'c2.bed'))
  assert r[1]['ploidy'] == 2 and all(len(c['pos']) == 0 for c in r[1]['copies'])


def test_native_fasta_reader(tmp_path):
  """mh_fasta.cpp (pysam.FastaFile's role, readgenerate.py:181,186) = the plain Python parse: plain and gzip input,
  CRLF line ends, header descriptions, empty contigs, lowercase / IUPAC bytes, a names filter."""
  import gzip
  from mitty_amd.lib import fasta
  txt = (b'>c1 some description\r\nACGTN\r\nacgtRYK\r\n>empty\n>c3\tx\n' + b'ACGT' * 5000 + b'\n' + b'GGN' * 33 +
         b'\n>last\nTTTT')
  plain, gz = tmp_path / 'a.fa', tmp_path / 'a.fa.gz'
  plain.write_bytes(txt)
  gz.write_bytes(gzip.compress(txt))
  for f in (str(plain), str(gz), G.path('data/syn.fa'), G.path('data/tiny.fasta')):
    assert fasta.read_fasta(f) == fasta.read_fasta_py(f), f
  assert fasta.read_fasta(str(plain))['c1'] == b'ACGTNacgtRYK'
  assert fasta.read_fasta(str(plain))['empty'] == b''
  assert set(fasta.read_fasta(str(gz), names={'c3', 'nope'})) == {'c3'}
  with pytest.raises(ValueError):
    fasta.read_fasta(str(tmp_path / 'missing.fa'))


def _bucket_tables(cum):
  """The Philox-mode tables of mh_set_corruption: T = min(floor(x * 2^16), 65535) and per row bk[k] = min(entries
  below k / 256, 93) | 0x80 when an entry lies in bucket k (and fewer than 93 are below it)."""
  T = np.minimum(np.floor(np.clip(cum, 0, None) * 65536.0), 65535).astype(np.int64)
  below = np.stack([(T < (k << 8)).sum(-1) for k in range(257)], -1)
  bk = np.minimum(below[..., :256], 93) | np.where((below[..., :256] < 93) & (below[..., 1:] > below[..., :256]),
                                                   0x80, 0)
  return T, bk


def _decide16(Trow, bkrow, n_bq, h1):
  """corrupt_base16's BQ step: (count below h1 capped at 93, ambiguous) from the bucket entry and the row walk."""
  e = int(bkrow[h1 >> 8])
  bq = e & 0x7f
  if not e & 0x80:
    return bq, False
  lim = min(n_bq, 93)
  v = int(Trow[bq]) if bq < lim else 1 << 32
  while v < h1:
    bq += 1
    v = int(Trow[bq]) if bq < lim else 1 << 32
  return bq, v == h1


def test_philox_u16_decision_rule_equals_f64():
  """The Philox-mode corruption decides on the high 16 bits h of a 53-bit uniform U = (h * 2^37 + l) / 2^53 against
  T = min(floor(x * 2^16), 65535), through a per-row bucket table (mh_corrupt.h corrupt_base16): T < h -> x < U,
  T > h -> not, T == h -> the f64 comparison with the low bits.  The rule must equal min(searchsorted(row, U,
  'left'), 93) and U < phred in f64 for every U, including h landing exactly on a table value."""
  rs = np.random.RandomState(3)
  phred = 10 ** (-np.arange(100) / 10)
  Fp = np.minimum(np.floor(phred * 65536.0), 65535).astype(np.int64)
  for m in G.MODELS:
    cum = G.model(m)['cum_bq_mat']
    T, bk = _bucket_tables(cum)
    n_bq = cum.shape[-1]
    for _ in range(200):
      f, n = rs.randint(2), rs.randint(int(G.model(m)['max_rlen']))
      row, Trow, bkrow = cum[f, n], T[f, n], bk[f, n]
      hs = np.concatenate([rs.randint(0, 2 ** 16, 64), Trow[rs.randint(0, n_bq, 16)], [0, 65535]])
      for h in hs:
        h = int(h)
        for l in (0, 1, rs.randint(0, 2 ** 37, dtype=np.int64), 2 ** 37 - 1):
          U = (float(h) * 2.0 ** 37 + float(l)) / 2.0 ** 53
          want = min(int(np.searchsorted(row, U, side='left')), 93)
          bq, amb = _decide16(Trow, bkrow, n_bq, h)
          got = want if amb else bq
          assert got == want, (m, f, n, h, l)
          sub_want = U < phred[want]
          sub_got = (U < phred[want]) if (amb or h == Fp[want]) else bool(h < Fp[want])
          assert sub_got == sub_want


def test_philox_restatement_known_answers():
  """tests/philox_ref.py (the Philox-mode parity restatement) against Random123's Philox4x32-10 known-answer
  vectors (ctr = key = 0; ctr = key = all ones)."""
  from tests import philox_ref as P
  assert [int(x[0]) for x in P.philox4x32_10([0], [0], [0], [0], 0, 0)] == \
      [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
  m = 0xffffffff
  assert [int(x[0]) for x in P.philox4x32_10([m], [m], [m], [m], m, m)] == \
      [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]


# ---- rpc's per-variant helpers over mh_expand_variant (reference test_rpc.py:24-108, restated) ----------------------
def _tiny_rpc():
  from mitty_amd.lib import vcfio
  ref_seq = open(G.path('data/tiny.fasta')).readlines()[1]
  vcf = vcfio.load_variant_file(G.path('data/tiny.vcf'), 'g0_s0', G.path('data/tiny.whole.bed'))
  return ref_seq, vcf


def test_rpc_variant_helpers_reference_cases():
  """The six expansion cases of the reference's test_rpc.py (:24-108): SNP / INS / DEL with and without an '=' node,
  node tuples and the cursors after the variant."""
  from mitty_amd.simulation import rpc
  ref_seq, vcf = _tiny_rpc()
  snp_v, ins_v, del_v = vcf[0]['v'][1][0], vcf[0]['v'][1][1], vcf[0]['v'][1][2]
  nodes, sp, rp = rpc.snp(ref_seq, 1, 5, snp_v, 1)                       # test_snp_expansion2
  assert [n.tuple() for n in nodes] == [(1, 5, 'X', 1, 'T', 0)] and (sp, rp) == (2, 6)
  nodes, sp, rp = rpc.snp(ref_seq, 1, 1, snp_v, 1)                       # test_snp_expansion3
  assert [n.tuple() for n in nodes] == [(1, 1, '=', 4, 'ATGA', None), (5, 5, 'X', 1, 'T', 0)]
  nodes, sp, rp = rpc.insertion(ref_seq, 9, 9, ins_v, 1)                 # test_ins_expansion2
  assert [n.tuple() for n in nodes] == [(9, 9, 'I', 3, 'TTT', 3)] and (sp, rp) == (12, 9)
  nodes, sp, rp = rpc.insertion(ref_seq, 6, 6, ins_v, 1)                 # test_ins_expansion3
  assert [n.tuple() for n in nodes] == [(6, 6, '=', 3, 'GTA', None), (9, 9, 'I', 3, 'TTT', 3)]
  nodes, sp, rp = rpc.deletion(ref_seq, 12, 12, del_v, 1)                # test_del_expansion2
  assert [n.tuple() for n in nodes] == [(11, 14, 'D', 2, '', -2)] and (sp, rp) == (12, 14)
  nodes, sp, rp = rpc.deletion(ref_seq, 12, 9, del_v, 1)                 # test_del_expansion3
  assert [n.tuple() for n in nodes] == [(12, 9, '=', 3, 'TCC', None), (14, 14, 'D', 2, '', -2)]
  assert rpc.create_nodes(ref_seq, 12, 9, del_v, 1)[0] == nodes


def test_rpc_variant_helpers_chain_equals_node_list_oracle():
  """Walking the helpers the way create_node_list does (skip pos < ref cursor, trailing '=' node) gives the oracle's
  node lists for both tiny copies and the SURVEY App. B edge cases."""
  from mitty_amd.simulation import rpc
  from oracle import oracle as O
  ref_seq, vcf = _tiny_rpc()
  cases = [(ref_seq, 1, vcf[0]['v'][c]) for c in range(2)]
  V = O.Variant
  cases.append(('ACGTACGTAC' * 3, 1, [V(27, 'CGTACG', 'C', 'D', 5)]))                                     # B1
  cases.append(('ACGTACGTAC' * 3, 1, [V(5, 'A', 'A' + 'T' * 20, 'I', 20)]))                               # B2
  cases.append(('ACGTACGTAC' * 3, 1, [V(5, 'ACGT', 'A', 'D', 3), V(6, 'C', 'T', 'X', 0), V(9, 'A', 'T', 'X', 0),
                                      V(9, 'A', 'AGG', 'I', 2)]))                                        # B3
  cases.append(('ACGTACGTAC' * 3, 1, [V(1, 'A', 'T', 'X', 0)]))                                           # B5
  cases.append(('ACGTACGTAC' * 3, 1, [V(1, 'A', 'AT', 'I', 1)]))
  for seq, rs, vl in cases:
    samp_pos = ref_pos = rs
    got = []
    for v in vl:
      if v.pos < ref_pos:
        continue
      nn, samp_pos, ref_pos = rpc.create_nodes(seq, samp_pos, ref_pos, v, rs)
      got += [n.tuple() for n in nn]
    off = ref_pos - rs
    if off <= len(seq):
      got.append((samp_pos, ref_pos, '=', len(seq) - off, seq[off:], None))
    want = [tuple(n) for n in O.create_node_list(seq.encode(), rs, vl)]
    assert got == want, (vl, got, want)


def test_engine_prefetch_slot_generations():
  """Engine's haplotype slots (no GPU: a stand-in context records the calls): a prefetch for the next step builds
  every key afresh into the slot generation its live slot does not use, kept apart until drop_haplotypes releases the
  current ones and adopts them; a prefetch within a step skips keys already built; builds alternate generations, so
  a key's new slot is never its live one (mh_prefetch_haplotypes_vset refuses live slots)."""
  from mitty_amd.engine import Engine

  class Ctx:
    def __init__(self):
      self.live, self.calls = set(), []

    def build_haplotypes_vset(self, slots, contig_ids, ref_starts, vsets):
      assert not self.live & set(slots)
      self.live |= set(slots)
      self.calls.append(('build', tuple(slots)))
      return [(3, 1, 9)] * len(slots)

    def prefetch_haplotypes_vset(self, slots, contig_ids, ref_starts, vsets, unit_slots=(), unit_seeds=(), p=1.0):
      assert not self.live & set(slots)
      self.live |= set(slots)
      self.calls.append(('prefetch', tuple(slots)))

    def release_haplotype(self, slot):
      self.live.remove(slot)

  eng = Engine.__new__(Engine)
  eng.ctx = Ctx()
  eng._regions = {0: ('1', 0, 100), 1: ('2', 0, 100)}
  eng._vsets = {(0, 0): 0, (0, 1): 1, (1, 0): 64, (1, 1): 65}
  eng._haps, eng._pre, eng._gen = {}, {}, {}
  a, b = [(0, 0), (0, 1)], [(1, 0), (1, 1)]
  ua, ub = [(0, ri, cpy, 5) for ri, cpy in a], [(0, ri, cpy, 5) for ri, cpy in b]
  eng.haplotypes(a)                        # step 1, batch 0
  eng.prefetch(ub)                         # batch 1 during batch 0
  eng.prefetch(ub)                         # (already built: nothing)
  eng.prefetch(ua, next_step=True)         # the next step's batch 0 during the last batch: fresh builds
  assert eng.ctx.calls == [('build', (0, 1)), ('prefetch', (64, 65)), ('prefetch', (2, 3))]
  assert set(eng._haps) == set(a + b) and set(eng._pre) == set(a)
  eng.drop_haplotypes()                    # step 2: the prefetched ones become current, the rest released
  assert eng.ctx.live == {2, 3} and set(eng._haps) == set(a) and not eng._pre
  eng.haplotypes(a + b)                    # a kept (built during step 1), b rebuilt in its other generation
  assert eng.ctx.calls[-1] == ('build', (66, 67))
  eng.prefetch(ua, next_step=True)
  assert eng.ctx.calls[-1] == ('prefetch', (0, 1))
