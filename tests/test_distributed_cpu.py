"""Multi-rank generate-reads orchestration (mitty_amd.distributed) with gloo on CPU.

Each rank runs generate_reads_distributed with a host stand-in backend (tests/dist_host.py, per-unit FASTQ from the
CPU oracle); the files the ranks pwrite together must equal the reference --threads 1 golden output byte for byte,
for whole-unit LPT sharding and for sliced units (cnt bases from the all-reduced slice counts).
"""
import os

import pytest

from mitty_amd import distributed as D
from tests import golden_io as G


def test_lpt_assign_balances():
  owner = D.lpt_assign([9, 7, 5, 3, 3, 1], 2)
  loads = [sum(w for w, o in zip([9, 7, 5, 3, 3, 1], owner) if o == r) for r in range(2)]
  assert sorted(loads) == [13, 15] and owner[0] != owner[1]   # LPT (4/3-approximate), not optimal


def test_plan_pieces_layouts():
  assert D.plan_pieces([5] * 8, 4) == [(u, 0, 1, u % 4) for u in range(8)]
  sl = D.plan_pieces([5] * 4, 8)              # chr1: 4 units on 8 GPUs -> every unit sliced 8 ways
  assert len(sl) == 32 and sl[9] == (1, 1, 8, 1)
  assert D.plan_pieces([5] * 8, 2, 'slice')[1] == (0, 1, 2, 1)
  m = 1_000_003
  assert [D.slice_range(m, s, 8)[0] for s in range(1, 9)] == [D.slice_range(m, s, 8)[1] for s in range(8)]
  assert D.exclusive_bases([(0, 0, 2, 0), (0, 1, 2, 1), (1, 0, 2, 0), (1, 1, 2, 1)], [3, 4, 5, 6]) == [0, 3, 0, 5]
  assert D.file_offsets([3, 0, 4]) == ([0, 3, 3], 7)


def _rank(rank, world, port, layout, model_name, outdir):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd.readmodel import get_read_model
    from tests.dist_host import OracleBackend
    c = G.load_json('e2e_config.json')[model_name]
    mod, mdl = get_read_model(model_name + '.pkl')
    st = D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'),
                                      seed=c['seed'], backend=OracleBackend(), layout=layout)
    assert st['world'] == world
    if layout == 'slice':   # every unit sampled exactly once over the ranks, then broadcast
      import torch
      t = torch.tensor([st.get('sampled', 0)], dtype=torch.int64)
      dist.all_reduce(t)
      assert int(t.item()) == st['units'], (int(t.item()), st['units'])
  finally:
    dist.destroy_process_group()


@pytest.mark.parametrize('world,layout', [(2, None), (2, 'slice'), (3, 'slice')])
def test_distributed_output_identical_to_single_process(tmp_path, world, layout):
  from tests._spawn import spawn_with_port
  model = 'hiseq-X-v2.5-Garvan'
  spawn_with_port(_rank, lambda port: (world, port, layout, model, str(tmp_path)), world)
  G.check_same(open(tmp_path / 'r1.fq', 'rb').read(), G.fastq_bytes('e2e_{}.r1.fq.gz'.format(model)))
  G.check_same(open(tmp_path / 'r2.fq', 'rb').read(), G.fastq_bytes('e2e_{}.r2.fq.gz'.format(model)))


@pytest.mark.parametrize('names', [('r1.fq.gz', 'r2.fq.gz'), ('r1.fq.gz', 'r2.fq'), ('r1.fq', 'r2.fq.gz')])
def test_distributed_gz_output(tmp_path, names):
  """'.gz' outputs (decided per file, as the single-GPU FastqSink decides): BGZF pieces at all-reduced offsets + EOF
  marker; each file decompresses (or reads) to the single-process bytes."""
  import gzip
  from tests._spawn import spawn_with_port
  spawn_with_port(_rank_gz, lambda port: (2, port, str(tmp_path), names), 2)
  model = 'hiseq-X-v2.5-Garvan'
  for k, fn in enumerate(names):
    raw = open(str(tmp_path / fn), 'rb').read()
    if fn.endswith('.gz'):
      assert raw[-28:] == bytes.fromhex('1f8b08040000000000ff0600424302001b0003000000000000000000')
      raw = gzip.decompress(raw)
    else:
      assert raw[:2] != b'\x1f\x8b'
    G.check_same(raw, G.fastq_bytes('e2e_{}.r{}.fq.gz'.format(model, k + 1)))


def _rank_gz(rank, world, port, outdir, names):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd.readmodel import get_read_model
    from tests.dist_host import OracleBackend
    model_name = 'hiseq-X-v2.5-Garvan'
    c = G.load_json('e2e_config.json')[model_name]
    mod, mdl = get_read_model(model_name + '.pkl')
    D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                 c['coverage'], os.path.join(outdir, names[0]), os.path.join(outdir, names[1]),
                                 seed=c['seed'], backend=OracleBackend(), layout='slice')
  finally:
    dist.destroy_process_group()


def _rank_wgs(rank, world, port, g, outdir):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd.readmodel import get_read_model
    from tests.dist_host import OracleBackend
    mod, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
    st = D.generate_reads_distributed(g['fa'], g['vcf'], 'SYN', g['bed'], mod, mdl, 30.0,
                                      os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'), seed=7,
                                      backend=OracleBackend(), max_batch_draws=100_000)
    assert st['units'] == 100 and st['pieces'] >= 20   # LPT: whole units, every rank has a share
  finally:
    dist.destroy_process_group()


def test_wgs_plan_four_ranks(tmp_path):
  """The whole-genome plan (GRCh37's 25 contigs, one BED interval each, 100 units dealt by LPT; the bench's and
  configs[3]'s shape) over 4 gloo ranks, at lengths x0.0005: the files equal the oracle's units in unit order."""
  import hashlib
  from mitty_amd import synth
  from mitty_amd.readmodel import get_read_model
  from oracle import oracle as O
  contigs = synth.genome_contigs(0.0005)
  data = synth.genome_regions(contigs, list(range(len(contigs))), workers=1)
  seqs = [(n, data[ri][0]) for ri, (n, _) in enumerate(contigs)]
  g = {'fa': str(tmp_path / 'g.fa'), 'vcf': str(tmp_path / 'g.vcf.gz'), 'bed': str(tmp_path / 'g.bed')}
  synth.write_fasta(g['fa'], seqs)
  synth.write_vcf(g['vcf'], seqs, {n: data[ri][1] for ri, (n, _) in enumerate(contigs)})
  with open(g['bed'], 'w') as fp:
    fp.write(''.join('{}\t0\t{}\n'.format(n, L) for n, L in contigs))
  from tests._spawn import spawn_with_port
  spawn_with_port(_rank_wgs, lambda port: (4, port, g, str(tmp_path)), 4)
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  units = O.unit_digests(dict(seqs), O.load_variant_file(g['vcf'], 'SYN', g['bed']), 'SYN', mdl, 30.0, 7, workers=4)
  assert len(units) == 100 and len({u[1] for u in units}) == 25
  for f, (li, hi) in (('r1.fq', (4, 5)), ('r2.fq', (6, 7))):
    b = open(str(tmp_path / f), 'rb').read()
    assert len(b) == sum(u[li] for u in units)
    off = 0
    for u in units:
      assert hashlib.sha256(b[off:off + u[li]]).hexdigest() == u[hi], (f, u[:3])
      off += u[li]


def test_bench_batch_plan():
  """bench.py's WGS batches: every unit once, in ps order; about the target size; at least min_batches per rank
  (a rank's share at N = 8 is ~1/8 of the genome); a ramp makes the first batches smaller."""
  import bench
  units = [(ps, ps % 5, ps % 2, 100 + ps) for ps in range(40)]
  draws = [10.0, 20.0, 30.0, 40.0, 50.0]
  for target, mb in ((100.0, 1), (1e9, 4), (100.0, 4), (25.0, 1)):
    b, size, total = bench.plan_batches(units, draws, target, mb)
    assert [u for x in b for u in x] == units
    assert total == sum(draws[u[1]] for u in units)
    assert size == min(target, total / mb)
    assert len(b) >= min(mb, len(units))
    for x in b[:-1]:   # every batch but the last reaches its size
      assert sum(draws[u[1]] for u in x) >= size


def _rank_few_units(rank, world, port, bed, outdir):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd.readmodel import get_read_model
    from tests.dist_host import OracleBackend
    c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
    mod, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
    st = D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], bed, mod, mdl,
                                      c['coverage'], os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'),
                                      seed=c['seed'], backend=OracleBackend(), layout='lpt')
    assert st['units'] == 4 and st['pieces'] == (0 if rank == 4 else 1), (rank, st)
  finally:
    dist.destroy_process_group()


def test_lpt_fewer_units_than_ranks(tmp_path):
  """LPT with fewer units than ranks (one diploid region, two passes: 4 units on 5 gloo ranks): the rank that owns no
  piece still joins every collective (the size all-reduce, the barriers, the totals), and the files equal the
  one-process run's (a rank-local condition had decided whether a rank joined the size all-reduce)."""
  from tests._spawn import spawn_with_port
  from mitty_amd.readmodel import get_read_model
  from tests.dist_host import OracleBackend
  bed = str(tmp_path / 'one.bed')
  with open(bed, 'w') as fp:
    fp.write('1\t1000\t40000\n')
  spawn_with_port(_rank_few_units, lambda port: (5, port, bed, str(tmp_path)), 5)
  c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
  mod, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  one = tmp_path / 'one'
  one.mkdir()
  D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], bed, mod, mdl, c['coverage'],
                               str(one / 'r1.fq'), str(one / 'r2.fq'), seed=c['seed'], backend=OracleBackend())
  for f in ('r1.fq', 'r2.fq'):
    a, b = open(tmp_path / f, 'rb').read(), open(one / f, 'rb').read()
    assert len(a) > 10000
    G.check_same(a, b)


def _rank_bam(rank, world, port, outdir, layout):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd.readmodel import get_read_model
    from tests.dist_host import OracleBackend
    c = G.load_json('e2e_config.json')['1kg-pcr-free']
    mod, mdl = get_read_model('1kg-pcr-free.pkl')
    st = D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'),
                                      seed=c['seed'], backend=OracleBackend(), layout=layout,
                                      bam_fname=os.path.join(outdir, 'g.bam'), bam_header_text='@HD\tVN:1.0\n',
                                      bam_refs=[('1', 50000), ('2', 20000), ('3', 8000)])
    assert st['bam_records'] > 1000 and st['bam_rounds'] >= 1
  finally:
    dist.destroy_process_group()


@pytest.mark.parametrize('world,layout', [(1, None), (2, None), (3, 'slice'), (4, 'lpt')])
def test_distributed_bam_leg(tmp_path, world, layout):
  """The configs[4] BAM leg over gloo ranks (host stand-in backend: records from oracle/god.py, host BGZF): every
  rank partitions its pieces' records by coordinate range and the all-to-all moves them to their range's rank; each
  rank sorts its range (equal keys by tie = global input order), writes the part of the file whose blocks start in
  its range (header on rank 0, the next ranges' heads completing its last block, EOF on the last rank); the parts
  are placed by their sizes and the BAI joined from the ranks' plans.  The file is the one-process BGZF of the
  god-aligner oracle's sorted stream, cut every 0xff00 bytes, and the BAI the oracle's over its virtual offsets."""
  import numpy as np
  from tests._spawn import spawn_with_port
  from oracle import god
  from mitty_amd import _native
  spawn_with_port(_rank_bam, lambda port: (world, port, str(tmp_path), layout), world)
  f1, f2 = open(tmp_path / 'r1.fq', 'rb').read(), open(tmp_path / 'r2.fq', 'rb').read()
  G.check_same(f1, G.fastq_bytes('e2e_1kg-pcr-free.r1.fq.gz'))
  stream = b''.join(god.encode(r) for r in god.sorted_stream(god.god_records(f1, f2, {'1': 0, '2': 1, '3': 2})))
  assert len(stream) > 10 * 0xff00
  refs = [('1', 50000), ('2', 20000), ('3', 8000)]
  want = (_native.bgzf_compress(god.header_bytes('@HD\tVN:1.0\n', [{'SN': n, 'LN': ln} for n, ln in refs])) +
          b''.join(_native.bgzf_compress(stream[o:o + 0xff00]) for o in range(0, len(stream), 0xff00)) +
          _native.bgzf_eof())
  got = open(tmp_path / 'g.bam', 'rb').read()
  assert got == want
  _, recs, vo, vend = god.record_voffsets(got)
  assert open(tmp_path / 'g.bam.bai', 'rb').read() == god.bai(3, [god.decode(r) for r in recs], vo, vend)
  assert not [f for f in os.listdir(tmp_path) if '.part' in f]


def test_range_splitters_and_bai_join():
  """range_splitters: ascending keys at equal shares of the regions' bases (in @SQ order); bai_join of one plan is
  bai_emit's layout (checked against god.bai on a tiny sorted set), and a run cut by a range boundary joins again."""
  import numpy as np
  from oracle import god
  refs = [('1', 50000), ('2', 20000), ('3', 8000)]
  sp = D.range_splitters([('2', 0, 20000), ('1', 0, 50000), ('3', 0, 8000)], refs, 3)
  assert sp == [D.sort_key(0, 26000), D.sort_key(1, 2000)]
  assert D.range_splitters([('1', 0, 10)], refs, 1) == []
  assert D.range_splitters([('1', 0, 4)], refs, 8) == sorted(D.range_splitters([('1', 0, 4)], refs, 8))
  # records: (tid, pos, end, bin) and voffsets; the same set as one plan or cut in two
  recs = [dict(reference_id=0, pos=p, cigarstring='100M', bin=god.reg2bin(p, p + 100)) for p in (10, 20, 16380, 40000)]
  vo = [100 << 16, 100 << 16 | 50, 100 << 16 | 90, 300 << 16]
  vend = 300 << 16 | 70
  ends = vo[1:] + [vend]

  def plan(ks):
    runs, win, nw = [], {}, 0
    for k in ks:
      r = recs[k]
      if runs and runs[-1][1] == r['bin'] and runs[-1][3] == k:
        runs[-1][3], runs[-1][5], runs[-1][6] = k + 1, ends[k], runs[-1][6] + 1
      else:
        runs.append([0, r['bin'], k, k + 1, vo[k], ends[k], 1])
      for w in range(r['pos'] >> 14, ((r['pos'] + 99) >> 14) + 1):
        win.setdefault(w, vo[k])
      nw = max(nw, ((r['pos'] + 99) >> 14) + 1)
    return {'runs': [tuple(x) for x in runs], 'win': {0: sorted(win.items())}, 'nwin': [nw, 0, 0]}
  want = god.bai(3, recs, vo, vend)
  assert D.bai_join([plan(range(4))], 3) == want
  assert D.bai_join([plan([0]), plan([1, 2]), plan([3])], 3) == want
