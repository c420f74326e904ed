#!/usr/bin/env python3
"""Benchmark: paired 2x150 bp templates/s for `generate-reads` on chr1 (249 Mbp) diploid at 30x, MI355X.

Workload (BASELINE.json configs[1], per GPU): a synthetic chr1-shaped contig (249,250,621 bp, N caps + centromere
gap) with ~1.3 variants/kbp (SNV/INS/DEL, long insertions, deliberate overlaps), phased diploid, read model
hiseq-X-v2.5-Garvan (the built-in 2x150 model; SURVEY.md Finding 3), coverage 30, seed 7, perfect reads.
One step = the whole job for that chromosome: splice both haplotypes on the GPU, then the reference's 4 work units
(2 copies x 2 passes) — MT19937-exact template sampling + read emission — with the FASTQ output left in HBM.
Inputs (contig bytes) are resident before timing; variant arrays are re-uploaded inside the step (13 MB).

Multi-GPU (torchrun, one process per GPU): every rank simulates its own chr1-shaped chromosome (weak scaling, no
data-path collective); an RCCL all-reduce of the per-rank template counts closes each step.

Prints one JSON line (rank 0).  `roofline` is for the emission writer (k_emit_direct; k_emit_write with
--emit-mode 1 or --corrupt): algorithmic bytes per launch =
sum over kept templates of 2*rlen (haplotype bases gathered) + FASTQ bytes written (both files), divided by the
launch's HIP-event duration; `stage_ms` gives every stage per step so the dominant kernel is visible.
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CHR1 = 249_250_621
PEAK_HBM_GBS = 8000.0


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=10)
  ap.add_argument('--warmup', type=int, default=2)
  ap.add_argument('--model', default='hiseq-X-v2.5-Garvan')
  ap.add_argument('--coverage', type=float, default=30.0)
  ap.add_argument('--length', type=int, default=CHR1)
  ap.add_argument('--seed', type=int, default=7)
  ap.add_argument('--rng', default='mitty', choices=['mitty', 'philox'])
  ap.add_argument('--corrupt', action='store_true', help='fused BQ corruption (BASELINE configs[2])')
  ap.add_argument('--cpu-baseline-mbp', type=float, default=100.0,
                  help='bounded CPU-oracle sample: one unit on the first N Mbp of the contig (0 = skip)')
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--stages', action='store_true', help='print per-stage timings to stderr')
  ap.add_argument('--emit-mode', type=int, default=0, help='0: direct writer, 1: LDS-image writer')
  return ap.parse_args()


def main():
  a = parse()
  rank = int(os.environ.get('RANK', '0'))
  world = int(os.environ.get('WORLD_SIZE', '1'))
  local = int(os.environ.get('LOCAL_RANK', '0'))
  dist = None
  if world > 1:
    import torch
    import torch.distributed as tdist
    torch.cuda.set_device(local)
    tdist.init_process_group('nccl')
    dist = tdist

  import numpy as np
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model

  _, model = get_read_model(a.model + '.pkl')
  rlen = int(model['mean_rlen'])
  p, passes = _native.read_model_params(rlen, a.coverage)
  t_in = time.time()
  seq = synth.contig(a.length, 1000 + rank)
  recs = synth.variants(seq, 2000 + rank)
  copies = synth.copies_soa(recs)
  units = _native.work_units(a.seed + rank, [2], passes)
  t_in = time.time() - t_in

  eng = Engine(local)
  if a.corrupt:
    eng.ctx.set_corruption(True, model['cum_bq_mat'], 10 ** (-np.arange(100) / 10), a.seed)
  eng.load_region(0, ('1', 0, a.length), seq)
  for cpy in range(len(copies)):   # inputs resident in HBM before timing: contig and both copies' variants
    eng.upload_variants(0, cpy, copies[cpy])
  eng.ctx.set_emit_mode(a.emit_mode)
  kernel = 'k_emit_write' if a.emit_mode else 'k_emit_direct'

  def step():
    # one chr1 job; consecutive jobs pipeline on the device (this job's splice and sampling run while the previous
    # job's last FASTQ writers drain); the timed region ends with a full synchronisation
    eng.drop_haplotypes()
    eng.ctx.reset_output()
    res = eng.run_units([(ps, ri, cpy, s) for ps, (ri, cpy, s) in enumerate(units)], lambda r, c: copies[c], p, rlen,
                        model['cum_tlen'], 'SYN', 0, True, a.rng)
    return sum(r[1] for r in res), sum(r[2] for r in res), sum(r[3] for r in res)

  def barrier():
    if dist is not None:
      dist.barrier()

  for _ in range(a.warmup):
    step()
  eng.ctx.enable_timing(True)
  barrier()
  eng.ctx.sync()
  t0 = time.perf_counter()
  kept = b1 = b2 = 0
  for _ in range(a.steps):
    k, x1, x2 = step()
    kept += k
    b1 += x1
    b2 += x2
  eng.ctx.sync()
  barrier()
  dt = time.perf_counter() - t0
  stages = eng.ctx.stage_times()
  eng.ctx.enable_timing(False)

  if dist is not None:
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device='cuda')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    c = torch.tensor([kept, b1, b2], dtype=torch.int64, device='cuda')
    dist.all_reduce(c)    # RCCL reduce of read counts over xGMI
    kept_all, b1_all, b2_all = (int(x) for x in c.tolist())
  else:
    kept_all, b1_all, b2_all = kept, b1, b2

  # per-stage totals (this rank) and the emission roofline
  agg = {}
  for name, ms in stages:
    agg.setdefault(name, [0.0, 0])
    agg[name][0] += ms
    agg[name][1] += 1
  ew_ms, ew_n = agg.get('emit_write', [0.0, 0])
  alg_bytes = 2 * rlen * kept + b1 + b2                       # this rank's algorithmic bytes over the timed steps
  achieved = alg_bytes / (ew_ms * 1e-3) / 1e9 if ew_ms > 0 else None
  traffic = None
  pmc = sorted(glob.glob(os.path.join(REPO, 'profiles', 'pmc_{}_*.json'.format(kernel))))
  if pmc:
    try:
      with open(pmc[-1]) as fp:
        d = json.load(fp)
      if d.get('rlen') == rlen and d.get('length') == a.length:
        traffic = d.get('hbm_bytes_per_launch')
    except Exception:
      traffic = None

  cpu = None
  if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_baseline_mbp > 0:
    cpu = cpu_baseline(a, seq, recs, p, rlen, model, units)

  if rank == 0:
    ms_per_step = dt / a.steps * 1e3
    stage_ms = {k: round(v[0] / a.steps, 3) for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])}
    out = {
      'metric': 'paired 2x150bp reads/sec at 30x WGS, 1/2/4/8 MI355X; qname POS/CIGAR bit-exact',
      'value': kept_all / a.steps / (dt / a.steps),
      'unit': 'templates/s',
      'n_gpus': world,
      'steps': a.steps,
      'warmup': a.warmup,
      'ms_per_step': ms_per_step,
      'higher_is_better': True,
      'scaling': 'weak',
      'vs_baseline': None,
      'dtype': 'int64+u8',
      'data': 'synthetic chr1-shaped contig + ~1.3/kbp phased diploid variants (mitty_amd.synth), seed-fixed',
      'config': {'workload': 'generate-reads chr1 (249,250,621 bp) diploid, {} 2x{} PE, {}x, rng={}{}, '
                             'one chr1-sized chromosome per GPU'.format(a.model, rlen, a.coverage, a.rng,
                                                                         ', +BQ corruption' if a.corrupt else ''),
                 'read_model': a.model, 'coverage': a.coverage, 'contig_bp': a.length, 'units_per_gpu': len(units),
                 'templates_per_step': kept_all // a.steps, 'parallelism': 'unit-shard x{}'.format(world)},
      'roofline': {'kernel': kernel, 'bound': 'hbm', 'achieved': achieved, 'peak': PEAK_HBM_GBS,
                   'unit': 'GB/s', 'frac': (achieved / PEAK_HBM_GBS) if achieved else None,
                   'traffic': traffic,
                   'algorithmic_bytes_per_launch': alg_bytes / max(ew_n, 1),
                   'avg_launch_ms': ew_ms / max(ew_n, 1)},
      'cpu_baseline': cpu,
      'stage_ms': stage_ms,
      'fastq_bytes_per_template': (b1_all + b2_all) / max(kept_all, 1),
    }
    print(json.dumps(out), flush=True)
  eng.close()
  if dist is not None:
    dist.destroy_process_group()


def _cpu_unit(args):
  """One work unit through the CPU oracle in a worker process; returns (templates, start, end) wall-clock stamps."""
  ref, soa, p, rlen, cum_tlen, seed, stub, cpy = args
  sys.path.insert(0, REPO)
  from oracle import oracle as O
  t0 = time.time()
  n = O.generate_unit_soa(ref, 0, soa, p, rlen, cum_tlen, seed, stub, '1', cpy, keep_output=False)[0]
  return n, t0, time.time()


def cpu_baseline(a, seq, recs, p, rlen, model, units):
  """The CPU oracle (oracle/mitty_oracle.c, a scalar port of the reference path) laid out like the reference's
  multiprocessing path (`readgenerate.process_multi_threaded`: one worker process per work unit, `--threads` <=
  #units): the job's work units run side by side in spawned worker processes (no GPU state in them) on the first
  `cpu_baseline_mbp` Mbp of the same contig.  Rate = templates / (last unit's end - first unit's start)."""
  import multiprocessing as mp
  from mitty_amd import synth
  L = int(a.cpu_baseline_mbp * 1e6)
  sub = synth.copies_soa(recs, 0, L)
  ref = bytes(seq[:L])
  jobs = [(ref, sub[cpy], p, rlen, model['cum_tlen'], s, 'SYN:0:{}'.format(k), cpy)
          for k, (ri, cpy, s) in enumerate(units)]
  with mp.get_context('spawn').Pool(len(jobs)) as pool:
    res = pool.map(_cpu_unit, jobs)
  n = sum(r[0] for r in res)
  dt = max(r[2] for r in res) - min(r[1] for r in res)
  return {'value': n / dt, 'unit': 'templates/s', 'cores': len(jobs), 'kind': 'port',
          'sample': '{} work units (2 copies x {} passes, one worker process each) on chr1[0:{:.0f} Mbp), {} templates '
                    'in {:.2f} s'.format(len(jobs), len(jobs) // 2, a.cpu_baseline_mbp, n, dt)}


if __name__ == '__main__':
  main()
