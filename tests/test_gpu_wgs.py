"""The metric's workload shape on the GPU: a whole-genome job (BASELINE configs[3]: GRCh37's 25 contigs, one BED
interval each, 100 work units, LPT deal over the ranks) through the product path
(mitty_amd.distributed.generate_reads_distributed -> DeviceBackend -> libmitty_hip.so), checked unit by unit against
the CPU oracle.

The genome is GRCh37 with every length scaled by GENOME_SCALE (the unit list, its seeds and order do not depend on
the lengths; the bench runs the same plan at scale 1).  Reference: readgenerate.py:129-159 (units), :76-126 (the
--threads 1 files are the units' pieces concatenated in unit order), SURVEY.md §8(e).
"""
import hashlib
import os

import pytest

pytestmark = pytest.mark.gpu

GENOME_SCALE = 0.02     # 62 Mbp, ~6.2 M templates, ~2.3 GB per FASTQ file
MODEL = 'hiseq-X-v2.5-Garvan'
COVERAGE, SEED, SAMPLE = 30.0, 7, 'SYN'


@pytest.fixture(scope='module')
def genome(tmp_path_factory):
  from mitty_amd import _native, synth
  if _native.device_count() == 0:
    pytest.fail('no HIP device: GPU tests must run on an MI355X')
  d = tmp_path_factory.mktemp('wgs')
  contigs = synth.genome_contigs(GENOME_SCALE)
  data = synth.genome_regions(contigs, list(range(len(contigs))), workers=8)
  seqs = [(name, data[ri][0]) for ri, (name, _) in enumerate(contigs)]
  fa, vcf, bed = str(d / 'g.fa'), str(d / 'g.vcf'), str(d / 'g.bed')
  synth.write_fasta(fa, seqs)
  synth.write_vcf(vcf, seqs, {name: data[ri][1] for ri, (name, _) in enumerate(contigs)}, sample=SAMPLE)
  with open(bed, 'w') as fp:
    for name, L in contigs:
      fp.write('{}\t0\t{}\n'.format(name, L))
  return {'dir': d, 'fa': fa, 'vcf': vcf, 'bed': bed, 'seqs': dict(seqs)}


@pytest.fixture(scope='module')
def oracle_units(genome):
  from mitty_amd.readmodel import get_read_model
  from oracle import oracle as O
  _, mdl = get_read_model(MODEL + '.pkl')
  vdf = O.load_variant_file(genome['vcf'], SAMPLE, genome['bed'])
  return O.unit_digests(genome['seqs'], vdf, SAMPLE, mdl, COVERAGE, SEED, workers=min(16, os.cpu_count() or 1))


def _rank(rank, world, port, g, outdir, names=('r1.fq', 'r2.fq')):
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  try:
    from mitty_amd import distributed as D
    from mitty_amd.readmodel import get_read_model
    mod, mdl = get_read_model(MODEL + '.pkl')
    st = D.generate_reads_distributed(g['fa'], g['vcf'], SAMPLE, g['bed'], mod, mdl, COVERAGE,
                                      os.path.join(outdir, names[0]), os.path.join(outdir, names[1]), seed=SEED,
                                      backend=D.DeviceBackend(0), max_batch_draws=32_000_000)
    assert st['units'] == 100 and st['world'] == world
  finally:
    dist.destroy_process_group()


def _run(world, g, outdir, names=('r1.fq', 'r2.fq')):
  from tests._spawn import spawn_with_port
  os.makedirs(outdir, exist_ok=True)
  gg = {k: v for k, v in g.items() if k in ('fa', 'vcf', 'bed')}
  spawn_with_port(_rank, lambda port: (world, port, gg, outdir, names), world)


def _check_units(fname, units, which):
  """The file = the oracle's unit pieces in unit order: compare length and digest piece by piece."""
  li, hi = (4, 5) if which == 1 else (6, 7)
  assert os.path.getsize(fname) == sum(u[li] for u in units)
  with open(fname, 'rb') as fp:
    for u in units:
      got = fp.read(u[li])
      assert hashlib.sha256(got).hexdigest() == u[hi], \
        'file {} unit ps={} (region {}, copy {}): bytes differ from the oracle'.format(which, u[0], u[1], u[2])


def _file_digest(fname):
  import gzip
  h = hashlib.sha256()
  with (gzip.open if fname.endswith('.gz') else open)(fname, 'rb') as fp:
    for chunk in iter(lambda: fp.read(64 << 20), b''):
      h.update(chunk)
  return h.hexdigest()


@pytest.mark.timeout(600)
def test_wgs_two_ranks_one_gpu_vs_oracle(genome, oracle_units):
  """2 ranks (gloo exchanges, both on GPU 0), 100 units dealt by LPT: every unit's bytes in both files equal the
  oracle's, and the files equal a one-rank run."""
  assert len(oracle_units) == 100
  assert sum(u[3] for u in oracle_units) > 5_000_000
  out2 = str(genome['dir'] / 'w2')
  _run(2, genome, out2)
  _check_units(os.path.join(out2, 'r1.fq'), oracle_units, 1)
  _check_units(os.path.join(out2, 'r2.fq'), oracle_units, 2)
  d2 = [_file_digest(os.path.join(out2, f)) for f in ('r1.fq', 'r2.fq')]
  for f in ('r1.fq', 'r2.fq'):
    os.remove(os.path.join(out2, f))
  out1 = str(genome['dir'] / 'w1')
  _run(1, genome, out1)
  assert [_file_digest(os.path.join(out1, f)) for f in ('r1.fq', 'r2.fq')] == d2
  for f in ('r1.fq', 'r2.fq'):
    os.remove(os.path.join(out1, f))
  # '.gz' outputs on 2 ranks: every piece deflated on its rank's device as it is emitted, placed by the all-reduced
  # compressed sizes; a plain file beside a '.gz' one is written piece by piece at its measured offset
  outz = str(genome['dir'] / 'wz')
  _run(2, genome, outz, ('r1.fq.gz', 'r2.fq'))
  assert [_file_digest(os.path.join(outz, f)) for f in ('r1.fq.gz', 'r2.fq')] == d2
  with open(os.path.join(outz, 'r1.fq.gz'), 'rb') as fp:
    assert fp.read(4) == b'\x1f\x8b\x08\x04'
  for f in ('r1.fq.gz', 'r2.fq'):
    os.remove(os.path.join(outz, f))
