"""`mitty` command line (reference mitty/cli.py), MI355X build.

Implemented: generate-reads (GPU), corrupt-reads (GPU), god-aligner (GPU), filter-variants (host C++), qname,
list-read-models.  Additive options on generate-reads: --device,
--rng {mitty,philox}, --corrupt-seed (fused Philox corruption); on corrupt-reads: --device, --rng {mitty,philox}.  Multi-GPU: launch generate-reads under
`python -m torch.distributed.run --nproc-per-node N -m mitty_amd.cli generate-reads ...` (one process per GPU,
RCCL); the output files are identical to the one-GPU run.  Out of scope for this build (not on the
generate-reads path): filter-bam, gc-cov, bq, bam2illumina, describe-read-model, mq-plot, derr-plot.
"""
import logging
import os

import click


@click.group()
@click.version_option('2.7.3.dev0+mi355x')
@click.option('-v', '--verbose', type=int, default=0)
def cli(verbose):
  """A genomic data simulator for testing and debugging bio-informatics tools"""
  logging.basicConfig(level=[logging.ERROR, logging.WARNING, logging.INFO, logging.DEBUG][min(verbose, 3)])


@cli.command('filter-variants', short_help='Remove complex variants from VCF')
@click.argument('vcfin', type=click.Path(exists=True))
@click.argument('sample')
@click.argument('bed')
@click.argument('vcfout', type=click.Path())
def filter_vcf(vcfin, sample, bed, vcfout):
  """Subset VCF for given sample, apply BED file and filter out complex variants
   making it suitable to use for read generation (reference cli.py:20-35)"""
  from mitty_amd.lib import vcfio
  vcfio.prepare_variant_file(vcfin, sample, bed, vcfout)


@cli.command('list-read-models')
@click.option('-d', type=click.Path(exists=True), help='List models in this directory')
def list_read_models(d):
  """List read models"""
  import glob
  from mitty_amd import readmodel
  if d is None:
    files = [os.path.join(readmodel.BUILTIN_DIR, f) for f in sorted(os.listdir(readmodel.BUILTIN_DIR))]
  else:
    files = glob.glob(os.path.join(d, '*'))
  for f in files:
    try:
      m = readmodel.load_model_file(f)
      name = os.path.basename(f)
      if name.endswith('.npz'):
        name = name[:-4] + '.pkl'
      click.echo('\n----------\n{}:\n{}\n=========='.format(name, m['model_description']))
    except Exception:
      logging.debug('Skipping {}. Not a read model file'.format(f))


@cli.command()
def qname():
  """Display qname format"""
  from mitty_amd.simulation import readgenerate
  click.echo(readgenerate.__qname_format_details__)


def print_qname(ctx, param, value):
  if not value or ctx.resilient_parsing:
    return
  from mitty_amd.simulation import readgenerate
  click.echo(readgenerate.__qname_format_details__)
  ctx.exit()


@cli.command('generate-reads', short_help='Generate simulated reads.')
@click.argument('fasta')
@click.argument('vcf')
@click.argument('sample_name')
@click.argument('bed')
@click.argument('modelfile')
@click.argument('coverage', type=float)
@click.argument('seed', type=int)
@click.argument('fastq1', type=click.Path())
@click.option('--fastq2', type=click.Path())
@click.option('--threads', default=2, help='Accepted for compatibility; the work runs on the GPU')
@click.option('--qname', is_flag=True, callback=print_qname, expose_value=False, is_eager=True,
              help='Print documentation for information encoded in qname')
@click.option('--device', default=0, help='HIP device ordinal')
@click.option('--rng', type=click.Choice(['mitty', 'philox']), default='mitty',
              help='mitty: bit-exact with the reference; philox: counter-based fast mode')
@click.option('--corrupt-seed', type=int, default=None, help='Apply the BQ corruption model while writing')
def generate_reads(fasta, vcf, sample_name, bed, modelfile, coverage, seed, fastq1, fastq2, threads, device, rng,
                   corrupt_seed):
  """Generate simulated reads"""
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  read_module, model = get_read_model(modelfile)
  if int(os.environ.get('WORLD_SIZE', '1')) > 1:
    import torch
    import torch.distributed as dist
    from mitty_amd import distributed
    torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', '0')))
    dist.init_process_group('nccl')
    try:
      stats = distributed.generate_reads_distributed(fasta, vcf, sample_name, bed, read_module, model, coverage,
                                                     fastq1, fastq2, seed=seed, rng=rng, corrupt_seed=corrupt_seed)
    finally:
      dist.destroy_process_group()
    logging.info('generate-reads: {}'.format(stats))
    return
  stats = readgenerate.process_multi_threaded(fasta, vcf, sample_name, bed, read_module, model, coverage, fastq1,
                                              fastq2, threads=threads, seed=seed, device=device, rng=rng,
                                              corrupt_seed=corrupt_seed)
  logging.info('generate-reads: {}'.format(stats))


@cli.command('corrupt-reads', short_help='Apply corruption model to FASTQ file of reads')
@click.argument('modelfile')
@click.argument('fastq1_in', type=click.Path(exists=True))
@click.argument('fastq1_out', type=click.Path())
@click.argument('seed', type=int)
@click.option('--fastq2-in', type=click.Path(exists=True))
@click.option('--fastq2-out', type=click.Path())
@click.option('--threads', default=2)
@click.option('--device', default=0, help='HIP device ordinal')
@click.option('--rng', type=click.Choice(['mitty', 'philox']), default='mitty',
              help='mitty: the reference\'s --threads 1 MT19937 stream, byte for byte; philox: counter-based')
def read_corruption(modelfile, fastq1_in, fastq1_out, seed, fastq2_in, fastq2_out, threads, device, rng):
  """Apply corruption model to FASTQ file of reads (reference cli.py:144-157)"""
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readcorrupt as rc
  read_module, read_model = get_read_model(modelfile)
  rc.multi_process(read_module, read_model, fastq1_in, fastq1_out, fastq2_in, fastq2_out, processes=threads, seed=seed,
                   device=device, rng=rng)


@cli.command('god-aligner', short_help='Create a perfect BAM from simulated FASTQs')
@click.argument('fasta', type=click.Path(exists=True))
@click.argument('fastq1', type=click.Path(exists=True))
@click.argument('bam')
@click.option('--fastq2', type=click.Path(exists=True), help='If a paired-end FASTQ, second file goes here')
@click.option('--sample-name', help='If supplied, this is put into the BAM header')
@click.option('--max-templates', type=int, help='For debugging: quits after processing these many templates')
@click.option('--threads', default=2)
@click.option('--device', default=0, help='HIP device ordinal')
@click.option('--gpu-bgzf', is_flag=True, help='Deflate the BAM record blocks on the GPU (additive option)')
@click.option('--hbm-gb', type=float, default=0.0,
              help='BAM records held in HBM before they spill to host memory, GB (0: no limit; additive option, the '
                   'counterpart of the reference\'s samtools sort -m)')
def god_aligner(fasta, bam, sample_name, fastq1, fastq2, max_templates, threads, device, gpu_bgzf, hbm_gb):
  """Given a FASTA.ann file and FASTQ made of simulated reads,
     construct a perfectly aligned BAM from them (reference cli.py:183-204).

     Note: The program uses the fasta.ann file to construct the BAM header"""
  from mitty_amd.benchmarking import god_aligner as god
  god.process_multi_threaded(fasta, bam, fastq1, fastq2, threads, max_templates, sample_name, device=device,
                             gpu_bgzf=gpu_bgzf, hbm_capacity=int(hbm_gb * 1e9))


def main():
  cli()


if __name__ == '__main__':
  main()
