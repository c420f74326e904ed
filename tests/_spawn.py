"""Multi-process test launcher: torch.multiprocessing ranks on a rendezvous port picked free on 127.0.0.1.  A port
picked this way can be taken by another process before rank 0's TCP store listens on it (EADDRINUSE, seen on a
shared GPU box); the ranks are then started again on a new port (at most three tries)."""
import socket


def free_port():
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    return s.getsockname()[1]


def spawn_with_port(fn, make_args, nprocs):
  """mp.start_processes(fn, args=make_args(port), nprocs) with a fresh free port per try."""
  import torch.multiprocessing as mp
  for attempt in range(3):
    try:
      mp.start_processes(fn, args=make_args(free_port()), nprocs=nprocs, join=True, start_method='spawn')
      return
    except mp.ProcessRaisedException as e:
      if 'EADDRINUSE' not in str(e) or attempt == 2:
        raise
