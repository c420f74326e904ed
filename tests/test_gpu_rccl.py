"""The RCCL ('nccl' backend) branches of the multi-GPU path, executed on one GPU (reference
parallelism readgenerate.py:102-115).

A world-size-1 'nccl' process group runs in a spawned process that imports torch before libmitty_hip.so (one HIP
runtime per process, DESIGN.md "Multi-GPU"):
* DeviceBackend.share: a template set packed on the device, broadcast by RCCL, unpacked into a second set; both sets
  emit the same bytes, equal to the CPU oracle's unit;
* allreduce_i64 on cuda tensors;
* generate_reads_distributed under the nccl group (its piece-size / file-offset all-reduce runs through RCCL): the
  files equal the golden reference FASTQ;
* its configs[4] BAM leg under the nccl group (records partitioned into cuda tensors, RCCL all-to-all, imported from
  device memory): records and BAI equal the god-aligner oracle's.
"""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(rank, port, outdir, q):
  import sys
  import torch   # first: torch's HIP runtime serves libmitty_hip.so too
  import torch.distributed as dist
  sys.path.insert(0, REPO)
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group('nccl', rank=0, world_size=1)
  try:
    from mitty_amd import distributed as D
    from mitty_amd.lib import fasta as mfasta, vcfio
    from mitty_amd.readmodel import get_read_model
    from tests import golden_io as G
    out = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    # allreduce_i64 over RCCL on cuda tensors
    out['allreduce'] = D.allreduce_i64([3, -5, 1 << 40])
    # share: pack -> RCCL broadcast -> unpack into set 1; both sets emitted
    c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
    mod, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
    rm = mod.read_model_params(mdl, c['coverage'])
    vdf = vcfio.load_variants_soa(G.path(c['vcf']), c['sample'], G.path(c['bed']))
    seqs = mfasta.read_fasta(G.path(c['fasta']))
    be = D.DeviceBackend(0)
    ri, cpy, seed = 0, 1, 4242
    chrom, s0, e = vdf[ri]['region']
    be.load_region(ri, vdf[ri]['region'], mfasta.fetch(seqs, chrom, s0, e))
    unit = (0, ri, cpy, seed)
    ns = be.sample([unit], lambda r, cc: vdf[r]['copies'][cc], rm['p'], rm['rlen'], rm['cum_tlen'], 'mitty')
    n = ns[0]
    be._slots[1] = be._slots[0]   # set 1 emits from the same haplotype
    be.share(0, n, 0, rm['rlen'], into=1)
    res = []
    for k in (0, 1):
      kept, r1, r2 = be.emit(k, 'S1:0:0', chrom, cpy, True, seed, None, 0)
      d1, d2 = be.fetch(r1, r2)
      res.append((kept, d1, d2))
    be.close()
    out['n'] = n
    out['share_equal'] = res[0] == res[1]
    out['kept'] = res[0][0]
    out['unit'] = (res[0][1], res[0][2])
    out['unit_args'] = (s0, e, chrom, cpy, seed)
    # the whole CLI job under the nccl group (the piece sizes all-reduced through RCCL)
    st = D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], os.path.join(outdir, 'r1.fq'), os.path.join(outdir, 'r2.fq'),
                                      seed=c['seed'])
    out['dist_stats'] = {k: st[k] for k in ('world', 'units', 'job_kept')}
    # the configs[4] BAM leg under the nccl group: each piece's records partitioned into a cuda tensor, moved by
    # RCCL's all-to-all, imported into the range store from device memory
    c = G.load_json('e2e_config.json')['1kg-pcr-free']
    mod, mdl = get_read_model('1kg-pcr-free.pkl')
    st = D.generate_reads_distributed(G.path(c['fasta']), G.path(c['vcf']), c['sample'], G.path(c['bed']), mod, mdl,
                                      c['coverage'], os.path.join(outdir, 'b1.fq'), os.path.join(outdir, 'b2.fq'),
                                      seed=c['seed'], bam_fname=os.path.join(outdir, 'g.bam'),
                                      bam_header_text='@HD\tVN:1.0\tSO:coordinate\n',
                                      bam_refs=[('1', 50000), ('2', 20000), ('3', 8000)])
    out['bam_stats'] = {k: st[k] for k in ('bam_records', 'bam_rounds', 'bam_received')}
    q.put(out)
  except BaseException as ex:   # noqa: BLE001 — reported to the parent
    import traceback
    q.put({'error': repr(ex), 'tb': traceback.format_exc()})
  finally:
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world_one(tmp_path):
  import torch.multiprocessing as mp
  from mitty_amd.readmodel import get_read_model
  from oracle import oracle as O
  from tests import golden_io as G
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  p = ctx.Process(target=_child, args=(0, port, str(tmp_path), q))
  p.start()
  out = q.get(timeout=280)
  p.join(60)
  assert 'error' not in out, out.get('tb')
  assert p.exitcode == 0
  assert out['backend'] == 'nccl' and out['world'] == 1
  assert out['allreduce'] == [3, -5, 1 << 40]
  assert out['share_equal'] and out['kept'] > 100
  # the shared set's bytes are the oracle's unit
  c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
  _, mdl = get_read_model('hiseq-X-v2.5-Garvan.pkl')
  p_, _ = O.read_model_params(mdl['mean_rlen'], c['coverage'])
  s0, e, chrom, cpy, seed = out['unit_args']
  seqs = O.read_fasta(G.path(c['fasta']))
  vl = O.load_variant_file(G.path(c['vcf']), c['sample'], G.path(c['bed']))[0]['v'][cpy]
  _, o1, o2 = O.generate_unit(seqs[chrom][s0:e], s0, vl, p_, int(mdl['mean_rlen']), mdl['cum_tlen'], seed, 'S1:0:0',
                              chrom, cpy)
  assert out['unit'] == (o1, o2)
  # the nccl job's files = the golden reference FASTQ
  assert out['dist_stats']['world'] == 1
  G.check_same(open(tmp_path / 'r1.fq', 'rb').read(), G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz'))
  G.check_same(open(tmp_path / 'r2.fq', 'rb').read(), G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r2.fq.gz'))
  # the BAM leg over RCCL: records and BAI = the god-aligner oracle's over the reference FASTQ
  from oracle import god
  f1, f2 = G.fastq_bytes('e2e_1kg-pcr-free.r1.fq.gz'), G.fastq_bytes('e2e_1kg-pcr-free.r2.fq.gz')
  b = open(tmp_path / 'g.bam', 'rb').read()
  _, recs, vo, vend = god.record_voffsets(b)
  want = god.sorted_stream(god.god_records(f1, f2, {'1': 0, '2': 1, '3': 2}))
  assert out['bam_stats']['bam_records'] == out['bam_stats']['bam_received'] == len(recs) == len(want) > 1000
  assert recs == [god.encode(r) for r in want]
  assert open(tmp_path / 'g.bam.bai', 'rb').read() == god.bai(3, [god.decode(r) for r in recs], vo, vend)
